"""Wall-clock timers (reference ``utils/profiling_and_tracing/time_utils.py:22-138``).

Unlike the reference (3 collectives on every ``stop()``, which deadlocks when a
subset of ranks times a region — Appendix D #13) the statistics are kept
locally and reduced across ranks once, in ``print_timers``.
"""
import time

import torch

from .print_utils import print_distributed


class Timer:
    timers_local = {}
    number_calls = {}
    _t0 = {}

    def __init__(self, name, cudasync=False):
        self.name = name
        self.cudasync = cudasync
        Timer.timers_local.setdefault(name, 0.0)
        Timer.number_calls.setdefault(name, 0)

    def start(self):
        if self.cudasync and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        Timer._t0[self.name] = time.perf_counter()

    def stop(self):
        if self.cudasync and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        t0 = Timer._t0.pop(self.name, None)
        if t0 is None:
            return 0.0
        dt = time.perf_counter() - t0
        Timer.timers_local[self.name] += dt
        Timer.number_calls[self.name] += 1
        return dt

    @staticmethod
    def reset():
        Timer.timers_local.clear()
        Timer.number_calls.clear()
        Timer._t0.clear()


def gather_timers():
    """Return {name: (min, max, avg, calls)} over ranks.

    Ranks may have timed different regions (a branch-only timer, an early-stop path),
    so the name sets are first unioned (one ``all_gather_object``) and every rank then
    reduces the SAME aligned vector; a rank that never ran a timer contributes 0 s to
    the sum and is excluded from min/max.  Sorting only the local names (the round-1
    code, and the reference's per-name collectives, Appendix D #13) mismatches or hangs."""
    import torch.distributed as dist

    names = sorted(Timer.timers_local)
    distributed = dist.is_initialized() and dist.get_world_size() > 1
    if distributed:
        from ..parallel.distributed import host_group

        g = host_group()
        lists = [None] * dist.get_world_size()
        dist.all_gather_object(lists, names, group=g)
        names = sorted(set().union(*lists))
    have = torch.tensor([n in Timer.timers_local for n in names], dtype=torch.bool)
    vals = torch.tensor([Timer.timers_local.get(n, 0.0) for n in names], dtype=torch.float64)
    calls = torch.tensor([Timer.number_calls.get(n, 0) for n in names], dtype=torch.float64)
    if distributed and names:
        inf = torch.full_like(vals, float("inf"))
        mn = torch.where(have, vals, inf)
        mx = torch.where(have, vals, -inf)
        sm, cnt, nr = vals.clone(), calls.clone(), have.double()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=g)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=g)
        for t in (sm, cnt, nr):
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=g)
        avg = sm / nr.clamp(min=1)
        calls = cnt
    else:
        mn = mx = avg = vals
    return {n: (float(mn[i]), float(mx[i]), float(avg[i]), int(calls[i])) for i, n in enumerate(names)}


def print_timers(verbosity):
    stats = gather_timers()
    print_distributed(verbosity, "%30s %12s %12s %12s %8s" % ("timer", "min", "max", "avg", "calls"))
    for n, (mn, mx, av, c) in stats.items():
        print_distributed(verbosity, "%30s %12.4f %12.4f %12.4f %8d" % (n, mn, mx, av, c))
    return stats
