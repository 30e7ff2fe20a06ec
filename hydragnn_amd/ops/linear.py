"""Linear layer for tall-skinny (edge / node row) activations.

Forward and input-gradient use the BLAS GEMM (rocBLAS/hipBLASLt: a plain
library GEMM tiled over many rows).  The weight/bias gradient — a reduction
over all rows into a tiny [out, in] matrix, which library heuristics map onto
1-4 workgroups — runs on the split-K HIP kernel in ``csrc/linear.hip``.
Composite mode (double backward) and CPU tensors use ``F.linear``.
"""
import torch
import torch.nn.functional as F

from .. import _native
from . import pna as _mode

MIN_ROWS = 1024  # below this the library GEMM is already latency-bound and fine


class _TallLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return F.linear(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dx = dy @ W if ctx.needs_input_grad[0] else None
        dW = db = None
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            dW, db = _native.ops().linear_wgrad(dy, x, ctx.has_b)
            if not ctx.has_b:
                db = None
        return dx, dW, db


def linear(x, W, b=None):
    if (x.is_cuda and x.dim() == 2 and x.shape[0] >= MIN_ROWS and x.dtype == torch.float32
            and W.dtype == torch.float32 and not _mode._state["composite"] and torch.is_grad_enabled()
            and (W.requires_grad or x.requires_grad)):
        return _TallLinear.apply(x, W, b)
    return F.linear(x, W, b)


class _TallLinearSum(torch.autograd.Function):
    """y = sum_k x_k @ W_k^T + b  (one output, several inputs; e.g. a concat-linear
    split into its column blocks so the concat is never materialised)."""

    @staticmethod
    def forward(ctx, b, *xw):
        xs, ws = xw[0::2], xw[1::2]
        ctx.save_for_backward(*xs, *ws)
        ctx.k = len(xs)
        ctx.has_b = b is not None
        y = F.linear(xs[0], ws[0], b)
        for x, w in zip(xs[1:], ws[1:]):
            y = torch.addmm(y, x, w.t())
        return y

    @staticmethod
    def backward(ctx, dy):
        t = ctx.saved_tensors
        xs, ws = t[:ctx.k], t[ctx.k:]
        grads = []
        db = None
        for j, (x, w) in enumerate(zip(xs, ws)):
            dx = dy @ w if ctx.needs_input_grad[1 + 2 * j] else None
            dW = None
            want_b = ctx.has_b and j == 0 and ctx.needs_input_grad[0]
            if ctx.needs_input_grad[2 + 2 * j] or want_b:
                dW, dbj = _native.ops().linear_wgrad(dy, x, want_b)
                if want_b:
                    db = dbj
            grads += [dx, dW]
        return (db, *grads)


def linear_sum(pairs, b=None):
    """sum_k F.linear(x_k, W_k) + b with the split-K weight-gradient kernel."""
    x0 = pairs[0][0]
    if (x0.is_cuda and x0.shape[0] >= MIN_ROWS and x0.dtype == torch.float32 and not _mode._state["composite"]
            and torch.is_grad_enabled()):
        flat = []
        for x, w in pairs:
            flat += [x, w]
        return _TallLinearSum.apply(b, *flat)
    y = F.linear(pairs[0][0], pairs[0][1], b)
    for x, w in pairs[1:]:
        y = y + F.linear(x, w)
    return y
