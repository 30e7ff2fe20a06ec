"""Batch normalisation over node rows with an optional valid-row count.

Reference: PyG ``BatchNorm`` -> ``torch.nn.BatchNorm1d`` (``Base.py:206,215,466``,
``gps.py:80-83``).  ``num_valid`` (python int or int32 device scalar) restricts the
statistics to the first rows so statically padded batches (hipGraph capture) keep
exact reference statistics.

GPU training mode runs the two-pass HIP kernels of ``csrc/batchnorm.hip``
(2 launches forward, 2 backward); CPU / eval / composite mode use torch ops.
"""
import torch
import torch.nn.functional as F

from .. import _native
from . import pna as _mode


class _BNFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, nv, rmean, rvar, momentum, eps):
        y, mean, invstd = _native.ops().bn_forward(x, nv, weight, bias, rmean, rvar, momentum, eps, False)
        ctx.save_for_backward(x, mean, invstd, weight, nv)
        ctx.has_w = weight is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, invstd, weight, nv = ctx.saved_tensors
        dx, dw, db = _native.ops().bn_backward(dy, x, nv, mean, invstd, weight if ctx.has_w else None)
        if not ctx.has_w:
            dw = db = None
        return dx, dw, db, None, None, None, None, None


def _as_nv(num_valid, device):
    if num_valid is None:
        return None
    if torch.is_tensor(num_valid):
        return num_valid.to(torch.int32).reshape(1) if num_valid.dtype != torch.int32 or num_valid.dim() else \
            num_valid.reshape(1)
    return torch.tensor([int(num_valid)], dtype=torch.int32, device=device)


def batch_norm(x, bn, num_valid=None):
    training = bn.training or not bn.track_running_stats
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and training and _mode.fused("norm")
            and bn.momentum is not None):
        if bn.track_running_stats and bn.num_batches_tracked is not None and bn.training:
            bn.num_batches_tracked.add_(1)
        nv = _as_nv(num_valid, x.device)
        rm = bn.running_mean if (bn.training and bn.track_running_stats) else None
        rv = bn.running_var if (bn.training and bn.track_running_stats) else None
        return _BNFused.apply(x, bn.weight, bn.bias, nv, rm, rv, float(bn.momentum), float(bn.eps))
    if num_valid is None or not training:
        return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, training, bn.momentum, bn.eps)
    return _masked_batch_norm(x, bn, num_valid)


def _masked_batch_norm(x, bn, num_valid):
    """Reference (torch ops) masked statistics; same update rule as BatchNorm1d."""
    n = x.shape[0]
    rows = torch.arange(n, device=x.device).view(-1, 1)
    m = (rows < num_valid).to(x.dtype)
    cnt = m.sum()
    mean = (x * m).sum(0) / cnt
    xc = (x - mean) * m
    var = (xc * xc).sum(0) / cnt
    if bn.training and bn.track_running_stats and bn.running_mean is not None:
        with torch.no_grad():
            unbiased = var * cnt / (cnt - 1).clamp(min=1)
            bn.running_mean.mul_(1 - bn.momentum).add_(bn.momentum * mean)
            bn.running_var.mul_(1 - bn.momentum).add_(bn.momentum * unbiased)
            bn.num_batches_tracked.add_(1)
    y = (x - mean) * torch.rsqrt(var + bn.eps)
    if bn.weight is not None:
        y = y * bn.weight + bn.bias
    return y


class _BNAddFused(torch.autograd.Function):
    """y = [relu](BN(dropout_p(a) + b)), rows >= num_valid zeroed if zero_pad (one kernel each way)."""

    @staticmethod
    def forward(ctx, a, b, weight, bias, nv, rmean, rvar, nbt, rng, salt, p, momentum, eps, relu, zero_pad):
        y, z, mean, invstd = _native.ops().bn_fused_fwd(a, b, nv, weight, bias, rmean, rvar, nbt, rng, salt, p,
                                                         momentum, eps, relu, zero_pad)
        if z.numel() == 0 and a.numel() != 0:
            z = a
        ctx.save_for_backward(z, mean, invstd, weight, bias, nv, rng)
        ctx.cfg = (salt, p, relu, zero_pad, b is not None, weight is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        z, mean, invstd, weight, bias, nv, rng = ctx.saved_tensors
        salt, p, relu, zero_pad, has_b, has_w = ctx.cfg
        dz, da, dw, db = _native.ops().bn_fused_bwd(dy, z, nv, mean, invstd, weight, bias, rng, salt, p, relu,
                                                    zero_pad)
        if not (rng is not None and p > 0):
            da = dz
        return (da, dz if has_b else None, dw if has_w else None, db if has_w else None,
                None, None, None, None, None, None, None, None, None, None, None)


FUSED_MAX_ROWS = 1 << 30  # two-launch slab kernels scale with N


def norm_add(a, bn, num_valid=None, residual=None, p=0.0, relu=False, zero_pad=False, salt=0, training=None):
    """``[relu](BN(dropout_p(a) + residual))``, optionally zeroing rows >= num_valid.

    The GPS / encoder epilogue (reference gps.py:120-150, Base.py:466) as a single
    HIP launch forward and backward in GPU training mode; torch ops otherwise.
    ``bn`` may be None (no normalisation).
    """
    from . import rng as _rng

    if training is None:
        training = bn.training if bn is not None else False
    drop_p = float(p) if (training and p > 0) else 0.0
    mod = bn.module if (bn is not None and hasattr(bn, "module")) else bn
    bn_train = mod is not None and (mod.training or not mod.track_running_stats)
    if (mod is not None and bn_train and a.is_cuda and a.dtype == torch.float32 and a.dim() == 2
            and a.shape[0] <= FUSED_MAX_ROWS and _mode.fused("norm") and mod.momentum is not None):
        nv = _as_nv(num_valid, a.device)
        track = mod.training and mod.track_running_stats
        rm = mod.running_mean if track else None
        rv = mod.running_var if track else None
        nbt = mod.num_batches_tracked if (track and mod.num_batches_tracked is not None) else None
        rng = _rng.counter(a.device) if drop_p > 0 else None
        b = residual.contiguous() if residual is not None else None
        return _BNAddFused.apply(a.contiguous(), b, mod.weight, mod.bias, nv, rm, rv, nbt, rng, int(salt), drop_p,
                                 float(mod.momentum), float(mod.eps), bool(relu), bool(zero_pad))
    h = _rng.dropout(a, drop_p, drop_p > 0, salt)
    if residual is not None:
        h = h + residual
    if mod is not None:
        h = batch_norm(h, mod, num_valid)
    if relu:
        h = torch.relu(h)
    if zero_pad and num_valid is not None:
        rows = torch.arange(h.shape[0], device=h.device).view(-1, 1)
        h = h * (rows < num_valid).to(h.dtype)
    return h
