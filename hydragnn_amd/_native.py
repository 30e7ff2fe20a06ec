"""Loader for the in-tree gfx950 native library (``_C.so``, ops under ``torch.ops.hydra``).

Policy: GPU tensors ALWAYS run the HIP kernels. If the library is missing or
fails to load while a GPU op is requested we raise instead of silently falling
back to an eager PyTorch path.  CPU tensors use the plain-torch reference
implementations in ``hydragnn_amd/ops`` (the numerics oracle for tests).
"""
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# HYDRA_NATIVE_LIB: load an alternative build of the library (A/B experiments with
# compile-time variants); default is the in-tree _C.so
LIB_PATH = os.environ.get("HYDRA_NATIVE_LIB") or os.path.join(_HERE, "_C.so")

_loaded = False
_error = None


def load():
    global _loaded, _error
    if _loaded:
        return True
    if not os.path.exists(LIB_PATH):
        _error = f"{LIB_PATH} not found (run `python -m hydragnn_amd.csrc.build`)"
        return False
    stale = _stale_reason()
    if stale:
        _error = stale
        return False
    try:
        torch.ops.load_library(LIB_PATH)
        _loaded = True
    except Exception as e:  # pragma: no cover - depends on the build
        _error = f"failed to load {LIB_PATH}: {e}"
    return _loaded


def _stale_reason():
    """The in-tree library must match the sources it was built from (``_C.so.srchash``,
    written by ``csrc/build.py``); an alternative library (HYDRA_NATIVE_LIB) is not checked."""
    if os.environ.get("HYDRA_NATIVE_LIB"):
        return None
    from .csrc import build as _b

    side = LIB_PATH + ".srchash"
    if not os.path.exists(side):
        return f"{LIB_PATH} has no source digest ({side}): rebuild with `python -m hydragnn_amd.csrc.build`"
    with open(side) as fh:
        built = fh.read().strip()
    if built != _b.source_digest():
        return (f"{LIB_PATH} is stale: the native sources changed since it was built "
                "(run `python -m hydragnn_amd.csrc.build`)")
    return None


def available():
    return load()


class _SyncOps:
    """``HYDRA_DEBUG_SYNC=1`` (SURVEY §5.2 debug mode): every native op is followed by a
    device synchronisation, so an asynchronous kernel fault (bad index, NaN trap, launch
    failure) is reported at the op that caused it, with the op's name, instead of at a later
    unrelated sync.  Not capture-safe; debugging only."""

    def __init__(self, ns):
        self._ns = ns

    def __getattr__(self, name):
        op = getattr(self._ns, name)

        def run(*args, **kwargs):
            if _TRACE:  # HYDRA_DEBUG_SYNC=2: name every native op (and its tensor shapes) before it launches
                shapes = [tuple(a.shape) + ((str(a.dtype)[6:], tuple(a.stride())),) for a in args
                          if isinstance(a, torch.Tensor)]
                print(f"[hydra op] {name} {shapes}", flush=True)
            out = op(*args, **kwargs)
            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                try:
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    raise RuntimeError(f"HYDRA_DEBUG_SYNC: device error after hydra::{name}: {e}") from e
            return out

        return run


_TRACE = os.environ.get("HYDRA_DEBUG_SYNC", "0") == "2"


def debug_sync():
    return os.environ.get("HYDRA_DEBUG_SYNC", "0") in ("1", "2")


def ops():
    """Return ``torch.ops.hydra``; raise loudly if the native library is unavailable."""
    if not load():
        raise RuntimeError(
            "hydragnn_amd native HIP library is required for GPU tensors but is unavailable: " + str(_error)
        )
    return _SyncOps(torch.ops.hydra) if debug_sync() else torch.ops.hydra
