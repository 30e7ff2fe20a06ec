"""Capture-safe dropout randomness for the fused HIP kernels.

``torch``'s dropout keeps its philox offset on the host and relies on graph-
registration hooks; the fused kernels (``csrc/norm_fused.hip``) instead hash
(seed, call-site salt, element index) with the seed read from a per-device
int64 *device* counter.  The counter is advanced by one captured kernel per
training forward, so every hipGraph replay draws fresh masks, and backward
recomputes the forward mask from the same (unchanged) counter.
"""
import itertools

import torch

from .. import _native

_counters = {}
_salts = itertools.count(1)


def new_salt():
    """Distinct id for a dropout call site (renumbered per model by ``assign_salts``)."""
    return next(_salts)


def assign_salts(model):
    """Number every dropout call site of ``model`` 1, 2, ... in module order, so the masks
    of a model depend only on the model (not on how many models were built before)."""
    k = 0
    for m in model.modules():
        if hasattr(m, "_salts"):
            m._salts = list(range(k + 1, k + 1 + len(m._salts)))
            k += len(m._salts)
        if hasattr(m, "_salt"):  # single-site modules (GATv2Conv)
            m._salt = k + 1
            k += 1


def _key(device):
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def counter(device):
    """Per-device counter seeded from ``torch.initial_seed()``; re-seeded in place when
    ``torch.manual_seed`` changed the seed since (so a run's dropout masks depend only on
    its own seed, not on what ran earlier in the process — torch.Generator semantics)."""
    key = _key(device)
    seed = torch.initial_seed() & 0x7FFFFFFF
    ent = _counters.get(key)
    if ent is None:
        ent = [torch.tensor([seed], dtype=torch.int64, device=device), seed]
        _counters[key] = ent
    elif ent[1] != seed and not (ent[0].is_cuda and torch.cuda.is_current_stream_capturing()):
        ent[0].fill_(seed)
        ent[1] = seed
    return ent[0]


_folded = set()


def fold_next_advance(device):
    """The next ``advance`` on ``device`` is already done by a launch that precedes it in the
    same stream (the captured step's device-side plan expansion increments the counter)."""
    _folded.add(_key(device))


def clear_fold(device):
    _folded.discard(_key(device))


def advance(device):
    """Advance the device counter (one tiny kernel; capturable) — or nothing, when a preceding
    launch already did (``fold_next_advance``)."""
    k = _key(device)
    if k in _folded:
        _folded.discard(k)
        return
    _native.ops().rng_advance(counter(device))


def dropout(x, p, training, salt):
    """Dropout with the counter hash on GPU (graph-safe), torch dropout elsewhere."""
    if not training or p <= 0.0:
        return x
    if x.is_cuda and x.dtype == torch.float32:
        return _HashDropout.apply(x, p, salt)
    return torch.nn.functional.dropout(x, p, True)


class _HashDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, salt):
        ctx.p, ctx.salt = p, salt
        ctx.dev = x.device
        return _native.ops().dropout_hash(x, counter(x.device), salt, p)

    @staticmethod
    def backward(ctx, g):
        return _native.ops().dropout_hash(g, counter(ctx.dev), ctx.salt, ctx.p), None, None
