"""Batch normalisation over node rows with an optional valid-row count.

Reference: PyG ``BatchNorm`` -> ``torch.nn.BatchNorm1d`` (``Base.py:206,215,466``,
``gps.py:80-83``).  ``num_valid`` (python int or 0-dim device tensor) restricts the
statistics to the first rows so statically-padded batches (graph capture) keep
exact reference statistics.
"""
import torch
import torch.nn.functional as F


def batch_norm(x, bn, num_valid=None):
    if num_valid is None or not bn.training:
        return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                            bn.training or not bn.track_running_stats, bn.momentum, bn.eps)
    # masked statistics (padded rows excluded); same update rule as BatchNorm1d
    n = x.shape[0]
    rows = torch.arange(n, device=x.device).view(-1, 1)
    m = (rows < num_valid).to(x.dtype)
    cnt = m.sum()
    mean = (x * m).sum(0) / cnt
    xc = (x - mean) * m
    var = (xc * xc).sum(0) / cnt
    if bn.track_running_stats and bn.running_mean is not None:
        with torch.no_grad():
            unbiased = var * cnt / (cnt - 1).clamp(min=1)
            bn.running_mean.mul_(1 - bn.momentum).add_(bn.momentum * mean)
            bn.running_var.mul_(1 - bn.momentum).add_(bn.momentum * unbiased)
            bn.num_batches_tracked.add_(1)
    y = (x - mean) * torch.rsqrt(var + bn.eps)
    if bn.weight is not None:
        y = y * bn.weight + bn.bias
    return y
