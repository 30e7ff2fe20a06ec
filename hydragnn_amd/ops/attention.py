"""Segment-block-diagonal multi-head self-attention (GPS global attention).

GPU: ``csrc/attention.hip`` flash kernels (fwd + atomic-free bwd).  CPU (and the
composite/double-backward mode): dense masked softmax reference.

Reference semantics: ``hydragnn/globalAtt/gps.py:126-133`` —
``torch.nn.MultiheadAttention`` over ``to_dense_batch(x, None)``: all nodes of
the local mini-batch in one sequence (``scope="batch"``).  ``scope="graph"``
restricts attention to nodes of the same graph.
"""
import math
import os

import torch

from .. import _native
from . import streams as _streams
from . import pna as _pna_mode


def make_segments(num_nodes, scope="batch", ptr=None, num_valid=None, device=None):
    """Return (seg_id int32 [N], seg_ptr int32 [S+1]) for the requested attention scope.

    ``num_valid`` (< N) marks trailing padding rows which form their own segment.
    """
    N = int(num_nodes)
    nv = N if num_valid is None else int(num_valid)
    if scope == "batch":
        if nv < N:
            seg_ptr = torch.tensor([0, nv, N], dtype=torch.int32, device=device)
            seg_id = torch.zeros(N, dtype=torch.int32, device=device)
            seg_id[nv:] = 1
        else:
            seg_ptr = torch.tensor([0, N], dtype=torch.int32, device=device)
            seg_id = torch.zeros(N, dtype=torch.int32, device=device)
        return seg_id, seg_ptr
    if scope == "graph":
        assert ptr is not None
        ptr = ptr.to(device=device, dtype=torch.int32)
        G = ptr.numel() - 1
        if int(ptr[-1]) < N:
            ptr = torch.cat([ptr, torch.tensor([N], dtype=torch.int32, device=device)])
        counts = (ptr[1:] - ptr[:-1]).long()
        seg_id = torch.repeat_interleave(torch.arange(ptr.numel() - 1, device=device, dtype=torch.int32), counts)
        return seg_id, ptr
    raise ValueError(f"unknown attention scope {scope}")


def attention_reference(qkv, heads, seg_id, scale=None, seg_ptr=None):
    """Plain-torch segment attention (the numerics oracle, and the twice-differentiable path
    of force training).  In composite mode (force training, eager), with ``seg_ptr`` and many
    short segments (graph scope) it runs on a
    dense per-segment batch [S, H, L, L] (the reference's to_dense_batch form) instead of
    masking an [H, N, N] score matrix: memory O(sum of L^2), not O(N^2)."""
    if seg_ptr is not None and seg_ptr.numel() > 2 and _pna_mode._state["composite"] and \
            not (qkv.is_cuda and torch.cuda.is_current_stream_capturing()):
        out = _attention_dense_batch(qkv, heads, seg_id, seg_ptr, scale)
        if out is not None:
            return out
    N, F3 = qkv.shape
    F = F3 // 3
    D = F // heads
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    q, k, v = qkv[:, :F], qkv[:, F:2 * F], qkv[:, 2 * F:]
    q = q.reshape(N, heads, D).transpose(0, 1)
    k = k.reshape(N, heads, D).transpose(0, 1)
    v = v.reshape(N, heads, D).transpose(0, 1)
    s = torch.matmul(q, k.transpose(1, 2)) * scale
    mask = seg_id.view(-1, 1) == seg_id.view(1, -1)
    s = s.masked_fill(~mask.unsqueeze(0), float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v)
    return o.transpose(0, 1).reshape(N, F)


def _attention_dense_batch(qkv, heads, seg_id, seg_ptr, scale):
    N, F3 = qkv.shape
    F = F3 // 3
    D = F // heads
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    S = seg_ptr.numel() - 1
    ptr = seg_ptr.long()
    lens = ptr[1:] - ptr[:-1]
    L = int(lens.max())  # host sync: the composite (eager) path only
    if S * L * L * 2 > N * N:  # one long segment dominates: the masked form is no larger
        return None
    sid = seg_id.long()
    pos = torch.arange(N, device=qkv.device) - ptr[sid]
    idx = sid * L + pos  # row of each token in the dense [S * L] layout
    dense = qkv.new_zeros(S * L, F3).index_copy(0, idx, qkv)  # differentiable in qkv (any order)
    dense = dense.view(S, L, 3, heads, D).permute(2, 0, 3, 1, 4)  # [3, S, H, L, D]
    q, k, v = dense[0], dense[1], dense[2]
    s = torch.matmul(q, k.transpose(-1, -2)) * scale  # [S, H, L, L]
    valid = torch.arange(L, device=qkv.device).view(1, L) < lens.view(S, 1)  # [S, L] real keys
    s = s.masked_fill(~valid.view(S, 1, 1, L), float("-inf"))
    o = torch.matmul(torch.softmax(s, dim=-1), v)  # [S, H, L, D]
    o = o.permute(0, 2, 1, 3).reshape(S * L, F)
    return o.index_select(0, idx)


_SPLITS = int(os.environ.get("HYDRA_ATTN_SPLITS", "0"))  # 0 = kernel heuristic


def _max_span(n, seg_ptr):
    """Host-side bound on the longest segment (shape arithmetic only: capture-safe).
    Only the split heuristic uses it; correctness never depends on it."""
    nseg = seg_ptr.numel() - 1
    if nseg <= 2:
        return n
    return min(n, 4 * ((n + nseg - 1) // nseg))


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, seg_id, seg_ptr, heads, scale):
        span = _max_span(qkv.shape[0], seg_ptr)
        O, LSE = _native.ops().attn_fwd(qkv, seg_id, seg_ptr, heads, scale, span, _SPLITS)
        ctx.save_for_backward(qkv, O, LSE, seg_id, seg_ptr)
        ctx.heads, ctx.scale, ctx.span = heads, scale, span
        return O

    @staticmethod
    def backward(ctx, dO):
        qkv, O, LSE, seg_id, seg_ptr = ctx.saved_tensors
        ops = _native.ops()
        # HYDRA_ATTN_BWD_FORK=1: dQ and dK/dV passes on two streams.  Off by default: measured
        # on MI355X (OC20 GPS headline) it loses to forking the whole attention branch
        # (13.3k vs 15.6k graphs/s), and the two cannot nest (hipGraph capture of a fork
        # from an already-forked stream crashed at capture end on ROCm 7).
        nested = _streams.enabled(qkv) and torch.cuda.current_stream(qkv.device) == _streams.side_stream(qkv.device)
        if not _streams.enabled(qkv) or nested or os.environ.get("HYDRA_ATTN_BWD_FORK", "0") != "1":
            dqkv = ops.attn_bwd(dO, qkv, O, LSE, seg_id, seg_ptr, ctx.heads, ctx.scale, ctx.span, _SPLITS)
            return dqkv, None, None, None, None
        # the dQ and dK/dV passes only share read-only inputs: dK/dV on a second side stream,
        # concurrently with dQ (each ~50 us and below the chip's width for GPS shapes)
        dO = dO.contiguous()
        delta = ops.attn_bwd_delta(dO, O, ctx.heads)
        args = (dO, qkv, LSE, delta, seg_id, seg_ptr, ctx.heads, ctx.scale, ctx.span, _SPLITS)
        with _streams.Fork(*args[:6], slot=1) as fork:
            pkv = ops.attn_bwd_part(*args, 1)
        pq = ops.attn_bwd_part(*args, 0)
        fork.join(pkv)
        return ops.attn_bwd_combine(pq, pkv), None, None, None, None


class _Attn8(torch.autograd.Function):
    """8-wide heads on the MFMA attention of csrc/attention8.hip (the fused GPS encoder's
    kernels) for the module path: pack (pair / quad layouts), one forward launch, one backward
    launch.  The QM9 SchNet + GPS layers (hidden 64, 8 heads) ran the packed-fp32 VALU
    kernels here (~100 us per layer each way at 1.1 k tokens)."""

    @staticmethod
    def forward(ctx, qkv, seg_id, seg_ptr, heads, scale):
        ops = _native.ops()
        N = qkv.shape[0]
        Qp, Qq, Kp, Kq, Vp, Vq = ops.attn8_pack(qkv, heads)
        O, L2 = ops.attn8_fwd(Qp, Kp, Vq, seg_id, seg_ptr, N, scale, 0)
        ctx.save_for_backward(O, L2, Qp, Qq, Kp, Kq, Vp, seg_id, seg_ptr)
        ctx.scale = scale
        return O

    @staticmethod
    def backward(ctx, dO):
        O, L2, Qp, Qq, Kp, Kq, Vp, seg_id, seg_ptr = ctx.saved_tensors
        dqkv = _native.ops().attn8_bwd(dO.contiguous(), O, L2, Qp, Qq, Kp, Kq, Vp, seg_id, seg_ptr, ctx.scale, 0)
        return dqkv, None, None, None, None


def segment_attention(qkv, heads, seg_id, seg_ptr, scale=None):
    """Multi-head self-attention on packed ``qkv`` [N, 3F] -> [N, F]."""
    F = qkv.shape[1] // 3
    D = F // heads
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if (qkv.is_cuda and qkv.dtype == torch.float32 and D == 8 and _pna_mode.fused("attn")
            and _pna_mode.fused("attn8") and qkv.shape[0] > 0):
        return _Attn8.apply(qkv.contiguous(), seg_id, seg_ptr, heads, scale)
    if (qkv.is_cuda and qkv.dtype == torch.float32 and D in (4, 8, 16, 32, 64)
            and _pna_mode.fused("attn")):
        return _FlashAttn.apply(qkv, seg_id, seg_ptr, heads, scale)
    return attention_reference(qkv, heads, seg_id, scale, seg_ptr=seg_ptr)
