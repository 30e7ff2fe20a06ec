"""Fused Bessel radial basis + per-layer radial projections of a PNAPlus stack
(``csrc/radial.hip``).

Reference: ``PNAPlusStack`` (``hydragnn/models/PNAPlusStack.py:40-304``) computes
``rbf = BesselBasisLayer(dist)`` once and, in every conv layer l,
``r_l = ReLU(rbf_emb_l(rbf))`` and ``G_l = rbf_lin_l(rbf)``.  On the GPU all of it
is one forward and two backward launches for the whole stack (instead of ~50 small
torch kernels); CPU tensors and composite (double-backward) mode use the modules.
"""
import torch

from .. import _native
from . import pna as _mode

MAX_K = 8
MAX_L = 8


class _Radial(torch.autograd.Function):
    """Outputs: the L per-layer r_l then the L per-layer G_l, each its own output, so
    the backward receives one gradient per layer (returning the stacked [L, E, F]
    tensors and indexing them made autograd build each layer's gradient as
    zeros(L, E, F) + slice copy + add: 18 launches / 120 us per OC20 step)."""

    @staticmethod
    def forward(ctx, dist, freq, Wemb, bemb, Wlin, cutoff, exponent):
        R, Gt = _native.ops().radial_fwd(dist, freq, Wemb, bemb, Wlin, cutoff, exponent)
        ctx.save_for_backward(R, dist, freq, Wemb, Wlin)
        ctx.cfg = (cutoff, exponent)
        ctx.L = R.shape[0]
        return (*R.unbind(0), *Gt.unbind(0))

    @staticmethod
    def backward(ctx, *grads):
        R, dist, freq, Wemb, Wlin = ctx.saved_tensors
        L = ctx.L

        def fill(gs):  # per-layer gradients, read in place by the kernel (no stacking copy)
            return [g if g is not None else torch.zeros_like(R[0]) for g in gs]

        dR = fill(grads[:L])
        dG = fill(grads[L:])
        ddist, dfreq, dWemb, dbemb, dWlin = _native.ops().radial_bwd(dR, dG, R, dist, freq, Wemb, Wlin, *ctx.cfg)
        return ddist, dfreq, dWemb, dbemb, dWlin, None, None


def fused_ok(dist, basis, convs):
    if not (dist.is_cuda and dist.dtype == torch.float32 and _mode.fused("radial")
            and 0 < len(convs) <= MAX_L and basis.freq.numel() <= MAX_K):
        return False
    shape = convs[0].rbf_emb[0].weight.shape  # [F, K]: all layers equal
    return all(c.rbf_emb[0].weight.shape == shape for c in convs)


def radial_features(dist, basis, convs):
    """[(r_l, G_l)] for PNAPlus convs ``convs`` sharing the Bessel basis ``basis``."""
    if not fused_ok(dist, basis, convs):
        rbf = basis(dist)
        return [(c.rbf_emb(rbf), c.rbf_lin(rbf)) for c in convs]
    Wemb = torch.stack([c.rbf_emb[0].weight for c in convs])
    bemb = torch.stack([c.rbf_emb[0].bias for c in convs])
    Wlin = torch.stack([c.rbf_lin.weight for c in convs])
    outs = _Radial.apply(dist.contiguous(), basis.freq, Wemb, bemb, Wlin, float(basis.cutoff),
                         int(basis.envelope.p - 1))
    L = len(convs)
    return [(outs[i], outs[L + i]) for i in range(L)]
