"""Fused PNA message + degree-scaler aggregation (see ``csrc/pna.hip``).

Z = cat[x, cat_{s in scalers} s(deg) * cat[mean, min, max, std](m)]  with
m_e = (A[dst_e] + B[src_e] + C_e) * G_e.

Reference: PyG ``DegreeScalerAggregation`` as used by
``hydragnn/models/PNAPlusStack.py:164`` / ``PNAStack.py:42-67``; message at
``PNAPlusStack.py:250-279``.

Two paths:
* fused (HIP, GPU, first-order autograd): one forward kernel, one backward
  kernel + one CSR segment-sum over sources.
* composite (CPU, or whenever a double-backward is needed): built from the
  differentiable primitives in ``ops.segment``.
"""
import math

import torch

from .. import _native
from . import segment as seg

import os

_state = {"composite": False, "off": set(filter(None, os.environ.get("HYDRA_UNFUSED", "").split(",")))}


def fused(name):
    """True when the fused HIP path of op family ``name`` may run: not in composite mode
    (double backward) and not switched off with ``HYDRA_UNFUSED=name[,name...]`` (bisecting
    numerics: pna, wprep, linear, mlp, norm, radial, attn, tp, segment)."""
    return not _state["composite"] and name not in _state["off"]


class composite_mode:
    """Force the composite (infinitely differentiable) path, e.g. for force training."""

    def __init__(self, enabled=True):
        self.enabled = enabled

    def __enter__(self):
        self.prev = _state["composite"]
        _state["composite"] = self.enabled

    def __exit__(self, *a):
        _state["composite"] = self.prev


def pna_avg_deg(deg_hist):
    """avg_deg dict of PyG DegreeScalerAggregation from a degree histogram."""
    deg = torch.as_tensor(deg_hist, dtype=torch.float64)
    num_nodes = float(deg.sum())
    bins = torch.arange(deg.numel(), dtype=torch.float64)
    return {
        "lin": float((bins * deg).sum()) / num_nodes,
        "log": float(((bins + 1).log() * deg).sum()) / num_nodes,
        "exp": float((bins.exp() * deg).sum()) / num_nodes,
    }


def degree_scalers(deg, avg_deg, scalers):
    d = deg.clamp(min=1.0).view(-1, 1)
    out = []
    for s in scalers:
        if s == "identity":
            out.append(torch.ones_like(d))
        elif s == "amplification":
            out.append(torch.log(d + 1) / avg_deg["log"])
        elif s == "attenuation":
            out.append(avg_deg["log"] / torch.log(d + 1))
        elif s == "linear":
            out.append(d / avg_deg["lin"])
        elif s == "inverse_linear":
            out.append(avg_deg["lin"] / d)
        else:
            raise ValueError(f"unknown PNA scaler {s}")
    return out


def pna_aggregate_composite(m, dst_si, avg_deg, aggregators=("mean", "min", "max", "std"),
                            scalers=("identity", "amplification", "attenuation", "linear")):
    """Differentiable reference: [N, len(aggr)*len(scalers)*F]."""
    aggs = []
    for a in aggregators:
        if a == "mean":
            aggs.append(seg.segment_mean(m, dst_si))
        elif a == "min":
            aggs.append(seg.segment_min(m, dst_si))
        elif a == "max":
            aggs.append(seg.segment_max(m, dst_si))
        elif a == "std":
            aggs.append(seg.segment_std(m, dst_si))
        elif a == "sum":
            aggs.append(seg.segment_sum(m, dst_si))
        elif a == "var":
            mean = seg.segment_mean(m, dst_si)
            aggs.append(seg.segment_mean(m * m, dst_si) - mean * mean)
        else:
            raise ValueError(f"unknown PNA aggregator {a}")
    out = torch.cat(aggs, dim=-1)
    deg = dst_si.degree(out.dtype).to(out.device)
    return torch.cat([out * s for s in degree_scalers(deg, avg_deg, scalers)], dim=-1)


_SCALER_CODE = {"identity": 0, "amplification": 1, "attenuation": 2, "linear": 3, "inverse_linear": 4}
_STD_EPS = 1e-5


class _PNAAggFused(torch.autograd.Function):
    """[mean, min, max, std] x scalers of a per-row table in one HIP pass each way
    (``csrc/segment.hip`` seg_pna_agg / seg_pna_agg_bwd); first-order only."""

    @staticmethod
    def forward(ctx, m, si, S, codes, avg_log, avg_lin):
        out, stat, arg = _native.ops().seg_pna_agg(m, si.rowptr, si.perm, S, codes, avg_log, avg_lin, _STD_EPS,
                                                   _STD_EPS ** 0.5)
        ctx.save_for_backward(m, stat, arg)
        ctx.si, ctx.cfg = si, (S, codes, avg_log, avg_lin)
        return out

    @staticmethod
    def backward(ctx, g):
        m, stat, arg = ctx.saved_tensors
        dm = _native.ops().seg_pna_agg_bwd(g.contiguous(), m, ctx.si.rowptr, ctx.si.perm, stat, arg, *ctx.cfg)
        return dm, None, None, None, None, None


def pna_aggregate(m, si, avg_deg, aggregators=("mean", "min", "max", "std"),
                  scalers=("identity", "amplification", "attenuation", "linear")):
    """Degree-scaler aggregation [N, len(aggr)*len(scalers)*F] of a per-row table ``m``
    over ``si`` (sorted or permuted CSR).  GPU fp32 with the [mean, min, max, std]
    aggregator set: one fused kernel each way; otherwise (CPU, other aggregators, double
    backward) the composite.  Captured steps use the fused op too: a captured step with it
    is bitwise identical to the eager padded step, gradients included
    (tools/pnaeq_capture_debug.py MODE=compare, 400 steps of the PNAEq conv-head CI run).  The
    round-4 divergence of that run was not this op: replayed steps ignored lr changes
    (ReduceLROnPlateau), fixed in TrainStep._sync_opt_hparams."""
    if (m.is_cuda and fused("pna") and m.dtype == torch.float32 and m.dim() == 2 and si.limit is None
            and tuple(aggregators) == ("mean", "min", "max", "std") and 1 <= len(scalers) <= 8):
        codes = 0
        for i, s in enumerate(scalers):
            if s not in _SCALER_CODE:
                raise ValueError(f"unknown PNA scaler {s}")
            codes |= _SCALER_CODE[s] << (3 * i)
        return _PNAAggFused.apply(m.contiguous(), si, len(scalers), codes, float(avg_deg["log"]),
                                  float(avg_deg["lin"]))
    return pna_aggregate_composite(m, si, avg_deg, aggregators, scalers)


class _PNAFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, AB, C, G, dst_si, src_si, avg_log, avg_lin):
        Z, amin, amax = _native.ops().pna_fwd(x, AB, C, G, src_si.index, dst_si.rowptr, avg_log, avg_lin)
        ctx.save_for_backward(Z, AB, C, G, amin, amax)
        ctx.has_C, ctx.has_G = C is not None, G is not None
        ctx.dst_si, ctx.src_si = dst_si, src_si
        ctx.avg = (avg_log, avg_lin)
        return Z

    @staticmethod
    def backward(ctx, dZ):
        Z, AB, C, G, amin, amax = ctx.saved_tensors
        F = Z.shape[1] // 17
        # pna_bwd writes dA into the left half of a [N, 2F] buffer; dB (segment sum of the edge
        # gradient over sources) lands in the right half: no concatenation launch
        dpre, dG, dAB = _native.ops().pna_bwd(dZ, Z, AB, C, G, ctx.src_si.index, ctx.dst_si.rowptr, amin,
                                              amax, ctx.avg[0], ctx.avg[1])
        _native.ops().seg_sum_out(dpre, ctx.src_si.rowptr, ctx.src_si.perm, dAB[:, F:])
        dx = dZ[:, :F]
        dC = dpre if ctx.has_C else None
        dG = dG if ctx.has_G else None
        return dx, dAB, dC, dG, None, None, None, None


class _PNAWeightPrep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W, b, encW, encb):
        out = _native.ops().pna_wprep_fwd(W, b, encW, encb)
        ctx.save_for_backward(W, encW, encb)
        return out

    @staticmethod
    def backward(ctx, dWab, dWr, dWd, dbc):
        W, encW, encb = ctx.saved_tensors
        return _native.ops().pna_wprep_bwd(dWab, dWr, dWd, dbc, W, encW, encb)


def pna_weight_prep(W, b, encW, encb):
    """Derived weights of a PNAPlus conv with edge encoder (``csrc/pna.hip``):
    ``Wab = [W_i; W_j]``, ``Wr = W_e encW[:, d:]``, ``Wd = W_e encW[:, :d]``,
    ``bc = W_e encb + b`` for ``pre_nn`` weight ``W = [W_i | W_j | W_e]``.  One HIP
    launch each way on the GPU; torch algebra on CPU / in composite mode."""
    F = W.shape[0]
    d = encW.shape[1] - F
    if W.is_cuda and fused("wprep") and W.dtype == torch.float32 and encW.dtype == torch.float32:
        return _PNAWeightPrep.apply(W, b, encW, encb)
    We = W[:, 2 * F:]
    return torch.cat([W[:, :F], W[:, F:2 * F]], 0), We @ encW[:, d:], We @ encW[:, :d], We @ encb + b


def pna_message_aggregate(x, AB, C, G, dst_si, src_si, avg_deg):
    """Z = cat[x, PNA-aggregate((A[dst] + B[src] + C) * G)] with default aggregators/scalers.

    ``AB`` is [N, 2F]: columns [0,F) multiply the destination (x_i) and
    [F,2F) the source (x_j) node features.
    """
    F = x.shape[1]
    use_fused = (
        x.is_cuda
        and fused("pna")
        and x.dtype == torch.float32
        and AB.dtype == torch.float32
        and (C is None or C.dtype == torch.float32)
        and (G is None or G.dtype == torch.float32)
        and dst_si.perm is None
    )
    if use_fused:
        return _PNAFused.apply(x.contiguous(), AB, None if C is None else C.contiguous(),
                               None if G is None else G.contiguous(), dst_si, src_si,
                               float(avg_deg["log"]), float(avg_deg["lin"]))
    A, B = AB[:, :F], AB[:, F:]
    m = seg.gather(A, dst_si) + seg.gather(B, src_si)
    if C is not None:
        m = m + C
    if G is not None:
        m = m * G
    agg = pna_aggregate_composite(m, dst_si, avg_deg)
    return torch.cat([x, agg], dim=-1)
