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
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and training and not _mode._state["composite"]
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
