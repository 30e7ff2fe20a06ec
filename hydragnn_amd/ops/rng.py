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
    """Distinct, creation-order-deterministic id for a dropout call site."""
    return next(_salts)


def _key(device):
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def counter(device):
    key = _key(device)
    c = _counters.get(key)
    if c is None:
        c = torch.tensor([torch.initial_seed() & 0x7FFFFFFF], dtype=torch.int64, device=device)
        _counters[key] = c
    return c


def advance(device):
    """Advance the device counter (one tiny kernel; capturable)."""
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
