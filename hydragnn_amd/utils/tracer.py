"""Region tracer (reference ``hydragnn/utils/profiling_and_tracing/tracer.py:14-167``).

Back-ends (enable any subset with ``initialize([...])``):
* ``"timer"``  – host wall-clock + optional device sync per region, aggregated
  into count / total / min / max per name (``summary()``, ``save(path)``);
* ``"roctx"``  – ROCTx ranges (``libroctx64``) so regions appear in
  ``rocprofv3 --marker-trace`` timelines (replaces GPTL / Score-P);
* ``"chrome"`` – Chrome-trace JSON events (``save_chrome(path)``).

API matches the reference: ``start(name, cudasync=False, sync=False)``,
``stop(...)``, ``enable()``, ``disable()``, ``reset()``, ``@profile(name)``,
``with timer(name)``.  ``HYDRAGNN_TRACE_LEVEL>0`` in the training loop turns on
device sync + barriers at region boundaries like the reference.
"""
import contextlib
import ctypes
import functools
import json
import os
import time

import torch

_backends = {}
_enabled = False


class _TimerBackend:
    def __init__(self):
        self.reset()

    def reset(self):
        self.t0 = {}
        self.stats = {}

    def start(self, name):
        self.t0[name] = time.perf_counter()

    def stop(self, name):
        t = self.t0.pop(name, None)
        if t is None:
            return
        dt = time.perf_counter() - t
        s = self.stats.setdefault(name, [0, 0.0, float("inf"), 0.0])
        s[0] += 1
        s[1] += dt
        s[2] = min(s[2], dt)
        s[3] = max(s[3], dt)


class _RoctxBackend:
    def __init__(self):
        self.lib = None
        cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"), "/opt/rocm/lib/libroctx64.so",
                 "libroctx64.so"]
        for c in cands:
            try:
                self.lib = ctypes.CDLL(c)
                break
            except OSError:
                continue
        if self.lib is not None:
            self.lib.roctxRangePushA.argtypes = [ctypes.c_char_p]

    def reset(self):
        pass

    def start(self, name):
        if self.lib is not None:
            self.lib.roctxRangePushA(name.encode())

    def stop(self, name):
        if self.lib is not None:
            self.lib.roctxRangePop()


class _ChromeBackend:
    def __init__(self):
        self.reset()

    def reset(self):
        self.events = []
        self.open = {}

    def start(self, name):
        self.open[name] = time.perf_counter_ns() // 1000

    def stop(self, name):
        t = self.open.pop(name, None)
        if t is not None:
            now = time.perf_counter_ns() // 1000
            self.events.append({"name": name, "ph": "X", "ts": t, "dur": now - t, "pid": os.getpid(), "tid": 0})


def initialize(trlist=("timer",), verbose=False):
    for n in trlist:
        if n in ("timer", "GPTL", "gptl"):
            _backends["timer"] = _TimerBackend()
        elif n in ("roctx", "SCOREP", "scorep"):
            _backends["roctx"] = _RoctxBackend()
        elif n == "chrome":
            _backends["chrome"] = _ChromeBackend()


def has(name):
    return name in _backends


def _sync(cudasync, sync):
    if cudasync and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    if sync:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.barrier()


def start(name, cudasync=False, sync=False):
    if not _enabled or not _backends:
        return
    _sync(cudasync, sync)
    for b in _backends.values():
        b.start(name)


def stop(name, cudasync=False, sync=False):
    if not _enabled or not _backends:
        return
    _sync(cudasync, sync)
    for b in _backends.values():
        b.stop(name)


def enable():
    global _enabled
    _enabled = True


def disable():
    global _enabled
    _enabled = False


def reset():
    for b in _backends.values():
        b.reset()


def profile(name):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **k):
            start(name)
            try:
                return fn(*a, **k)
            finally:
                stop(name)

        return wrapper

    return deco


@contextlib.contextmanager
def timer(name, cudasync=False):
    start(name, cudasync)
    try:
        yield
    finally:
        stop(name, cudasync)


def summary():
    b = _backends.get("timer")
    if b is None:
        return {}
    return {k: {"count": v[0], "total": v[1], "min": v[2], "max": v[3], "avg": v[1] / max(v[0], 1)}
            for k, v in b.stats.items()}


def save(path):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(summary(), f, indent=1)


def save_chrome(path):
    b = _backends.get("chrome")
    if b is None:
        return
    with open(path, "w") as f:
        json.dump({"traceEvents": b.events}, f)
