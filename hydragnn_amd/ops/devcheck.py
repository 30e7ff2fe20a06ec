"""Device-side input checks that need no host synchronisation per step.

Kernels that would otherwise index out of range on malformed input (element ids outside
the element table, a triplet count above its static capacity) clamp for memory safety and
fold what they saw into a persistent int32 flag per (device, name).  ``check_all`` — called
once per epoch by the training loop, and at once outside graph capture under
``HYDRA_DEBUG_SYNC=1`` — turns a non-zero flag into an error, so a bad batch never trains
silently on clamped data."""
import os

import torch

_FLAGS = {}
_WHAT = {
    "elem_range": "element ids outside [0, num_elements)",
    "triplet_cap": "triplets above the static capacity (largest excess)",
    "radius_graph_size": "a graph above the store's largest graph in the radius builder (its size)",
}


def flag(device, name):
    """The persistent flag tensor of ``name`` on ``device`` (allocated outside capture: the
    capture warm-up always runs the same ops eagerly first)."""
    key = (str(device), name)
    f = _FLAGS.get(key)
    if f is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"devcheck: flag {name!r} first requested inside graph capture")
        f = _FLAGS[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return f


def debug_check(name, device):
    """Immediate check of one flag (eager runs under HYDRA_DEBUG_SYNC=1)."""
    if os.environ.get("HYDRA_DEBUG_SYNC") == "1" and not torch.cuda.is_current_stream_capturing():
        _raise_if_set((str(device), name))


def _raise_if_set(key):
    f = _FLAGS.get(key)
    if f is None:
        return
    v = int(f.item())
    if v > 0:
        f.zero_()
        raise RuntimeError(f"device input check failed on {key[0]}: {_WHAT.get(key[1], key[1])} = {v}")


def check_all():
    """Raise on the first set flag (and clear it)."""
    for key in list(_FLAGS):
        _raise_if_set(key)
