"""Differentiable CSR segment ops (gather / segment-sum / mean / min / max / softmax).

Replaces torch_scatter and PyG aggregation (reference call sites:
``hydragnn/models/Base.py:599`` scatter_add, ``hydragnn/utils/model/model.py:279-286``
unsorted_segment_mean, ``EGCLStack.py:292-298`` unsorted_segment_sum,
``PAINNStack.py:256-257`` index_add_, PyG ``MessagePassing`` aggr).

A :class:`SegIndex` describes how E rows map onto N segments:
``index[e]`` is the owner segment of row e; ``rowptr``/``perm`` list, for each
segment, the rows it owns (``perm=None`` means rows are already sorted by
owner).  Because ``gather`` and ``segment_sum`` over the same SegIndex are each
other's adjoint, every op here is differentiable to any order (needed for
force training via double backward, ``Base.py:614-620``).

GPU tensors run the HIP kernels in ``csrc/segment.hip``; CPU tensors run the
plain-torch reference below (also the numerics oracle for the tests).
"""
import torch

from .. import _native


class SegIndex:
    """Row -> segment mapping with a CSR view (all index tensors int32)."""

    __slots__ = ("index", "rowptr", "perm", "num_segments", "limit", "_deg", "_index64", "_onehot_t", "_invdeg")

    def __init__(self, index, rowptr, perm, num_segments, limit=None):
        self.index = index
        self.rowptr = rowptr
        self.perm = perm
        self.num_segments = int(num_segments)
        # optional device int32 scalar: CSR positions at or past it are padding (their rows
        # contribute zero / are never read): the native segment sums stop there, so a padded
        # tail owned by one segment is not summed serially (static in-forward radius graph)
        self.limit = limit
        self._deg = None
        self._invdeg = None
        self._index64 = None
        self._onehot_t = None

    @property
    def num_rows(self):
        return self.index.numel()

    def onehot_t(self, dtype=torch.float32):
        """[num_segments, rows] 0/1 matrix, built once per index: a segment sum over FEW,
        LONG segments (element-indexed weight tables: a handful of elements over every node
        of the batch) is then one GEMM instead of a serial walk down each segment."""
        if self._onehot_t is None or self._onehot_t.dtype != dtype:
            oh = torch.zeros(self.num_segments, self.num_rows, device=self.index.device, dtype=dtype)
            oh.scatter_(0, self.index64.view(1, -1), 1.0)
            self._onehot_t = oh
        return self._onehot_t

    @property
    def index64(self):
        if self._index64 is None:
            self._index64 = self.index.long()
        return self._index64

    def degree(self, dtype=torch.float32):
        if self._deg is None:
            self._deg = (self.rowptr[1:] - self.rowptr[:-1]).to(dtype)
        return self._deg

    def inv_degree(self, dtype=torch.float32):
        """1 / max(degree, 1) per segment (cached with the index)."""
        d = getattr(self, "_invdeg", None)
        if d is None or d.dtype != dtype:
            d = 1.0 / self.degree(dtype).clamp(min=1.0)
            self._invdeg = d
        return d

    def to(self, device):
        p = None if self.perm is None else self.perm.to(device, non_blocking=True)
        lim = None if self.limit is None else self.limit.to(device, non_blocking=True)
        return SegIndex(self.index.to(device, non_blocking=True), self.rowptr.to(device, non_blocking=True), p,
                        self.num_segments, lim)

    @staticmethod
    def from_index(index, num_segments, sorted_=False):
        """Build from an owner index (any integer dtype)."""
        index = index.reshape(-1)
        dev = index.device
        counts = torch.bincount(index.long(), minlength=num_segments)
        rowptr = torch.zeros(num_segments + 1, dtype=torch.int32, device=dev)
        rowptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        perm = None
        if not sorted_:
            perm = torch.argsort(index.long(), stable=True).to(torch.int32)
        return SegIndex(index.to(torch.int32), rowptr, perm, num_segments)


def _use_native(t):
    return t.is_cuda


def _width(tail):
    w = 1
    for d in tail:
        w *= int(d)
    return w


# ------------------------------------------------------------------ CPU reference

def _cpu_segment_sum(x, si):
    out = x.new_zeros((si.num_segments,) + tuple(x.shape[1:]))
    return out.index_add_(0, si.index64.to(x.device), x)


def _cpu_segment_minmax(x, si, is_max):
    N = si.num_segments
    idx = si.index64
    out = x.new_zeros((N,) + tuple(x.shape[1:]))
    if x.numel() == 0:
        return out, torch.full(out.shape, -1, dtype=torch.int32)
    red = "amax" if is_max else "amin"
    shp = idx.view(-1, *([1] * (x.dim() - 1))).expand_as(x)
    out = out.scatter_reduce(0, shp, x, reduce=red, include_self=False)
    # arg: first row attaining the extremum (ties -> smallest row id)
    rows = torch.arange(x.shape[0], device=x.device).view(-1, *([1] * (x.dim() - 1))).expand_as(x)
    hit = x == out[idx]
    big = torch.full_like(rows, x.shape[0])
    cand = torch.where(hit, rows, big)
    arg = torch.full(out.shape, x.shape[0], dtype=torch.long, device=x.device)
    arg = arg.scatter_reduce(0, shp, cand, reduce="amin", include_self=True)
    arg = torch.where(arg >= x.shape[0], torch.full_like(arg, -1), arg).to(torch.int32)
    return out, arg


# ------------------------------------------------------------------ autograd fns

class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, si):
        ctx.si = si
        ctx.n = x.shape[0]
        if _use_native(x) and x.dtype == torch.float32:
            tail = x.shape[1:]
            out = _native.ops().gather_rows(x.reshape(x.shape[0], _width(tail)), si.index)
            return out.view((out.shape[0],) + tuple(tail))
        return x.index_select(0, si.index64.to(x.device))

    @staticmethod
    def backward(ctx, g):
        return _SegSum.apply(g, ctx.si), None


class _SegSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, si, limit=None):
        ctx.si = si
        if _use_native(x) and x.dtype == torch.float32:
            tail = x.shape[1:]
            lim = limit if limit is not None else si.limit
            if lim is not None and not (lim.dtype == torch.int32 and (si.perm is None or si.limit is lim)):
                lim = None
            out = _native.ops().seg_sum(x.reshape(x.shape[0], _width(tail)), si.rowptr, si.perm, si.num_segments,
                                        False, lim)
            return out.view((si.num_segments,) + tuple(tail))
        return _cpu_segment_sum(x, si)

    @staticmethod
    def backward(ctx, g):
        return _Gather.apply(g, ctx.si), None, None


class _ScatterArg(torch.autograd.Function):
    """out[E] = 0; out[arg[n,f], f] = g[n,f]."""

    @staticmethod
    def forward(ctx, g, arg, E):
        ctx.save_for_backward(arg)
        if _use_native(g) and g.dtype == torch.float32:
            return _native.ops().scatter_arg(g, arg, E)
        out = g.new_zeros((E,) + tuple(g.shape[1:]))
        valid = arg >= 0
        a = torch.where(valid, arg, torch.zeros_like(arg)).long()
        out.scatter_add_(0, a, torch.where(valid, g, torch.zeros_like(g)))
        return out

    @staticmethod
    def backward(ctx, go):
        (arg,) = ctx.saved_tensors
        return _GatherArg.apply(go, arg), None, None


class _GatherArg(torch.autograd.Function):
    """out[n,f] = x[arg[n,f], f] (0 when arg<0)."""

    @staticmethod
    def forward(ctx, x, arg):
        ctx.save_for_backward(arg)
        ctx.E = x.shape[0]
        if _use_native(x) and x.dtype == torch.float32:
            return _native.ops().gather_arg(x, arg)
        valid = arg >= 0
        a = torch.where(valid, arg, torch.zeros_like(arg)).long()
        return torch.where(valid, torch.gather(x, 0, a), torch.zeros((), dtype=x.dtype, device=x.device))

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        return _ScatterArg.apply(g, arg, ctx.E), None


class _SegMinMax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, si, is_max):
        if _use_native(x) and x.dtype == torch.float32 and x.dim() == 2:
            out, arg = _native.ops().seg_minmax(x, si.rowptr, si.num_segments, is_max, si.perm)
        else:
            out, arg = _cpu_segment_minmax(x, si, is_max)
        ctx.save_for_backward(arg)
        ctx.E = x.shape[0]
        ctx.mark_non_differentiable(arg)
        return out, arg

    @staticmethod
    def backward(ctx, g, _garg):
        (arg,) = ctx.saved_tensors
        return _ScatterArg.apply(g, arg, ctx.E), None, None


class _GatherMulSum(torch.autograd.Function):
    """out[n] = sum_{rows e of segment n of ssi} w[e] * x[gsi.index[e]] — gather, multiply by
    a per-row filter and segment-sum in one pass (csrc/segment.hip).  The op family
    {gather_mul_sum, gather_mul2} is closed under differentiation, so any derivative
    order stays on the native path:
        d/dw  = gather_mul2(x, gsi, g, ssi)
        d/dx  = gather_mul_sum(g, w, ssi, gsi)"""

    @staticmethod
    def forward(ctx, x, w, gsi, ssi):
        ctx.gsi, ctx.ssi = gsi, ssi
        ctx.save_for_backward(x, w)
        if _use_native(x) and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 2:
            return _native.ops().gather_mul_sum(x, w, gsi.index, ssi.rowptr, ssi.perm, ssi.num_segments, ssi.limit)
        return _cpu_segment_sum(x.index_select(0, gsi.index64.to(x.device)) * w, ssi)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        dx = _GatherMulSum.apply(g, w, ctx.ssi, ctx.gsi) if ctx.needs_input_grad[0] else None
        dw = _GatherMul2.apply(x, ctx.gsi, g, ctx.ssi) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None


class _GatherMul2(torch.autograd.Function):
    """out[e] = x[asi.index[e]] * y[bsi.index[e]]."""

    @staticmethod
    def forward(ctx, x, asi, y, bsi):
        ctx.asi, ctx.bsi = asi, bsi
        ctx.save_for_backward(x, y)
        if _use_native(x) and x.dtype == torch.float32 and y.dtype == torch.float32 and x.dim() == 2:
            return _native.ops().gather_mul2(x, asi.index, y, bsi.index)
        return x.index_select(0, asi.index64.to(x.device)) * y.index_select(0, bsi.index64.to(y.device))

    @staticmethod
    def backward(ctx, go):
        x, y = ctx.saved_tensors
        dx = _GatherMulSum.apply(y, go, ctx.bsi, ctx.asi) if ctx.needs_input_grad[0] else None
        dy = _GatherMulSum.apply(x, go, ctx.asi, ctx.bsi) if ctx.needs_input_grad[2] else None
        return dx, None, dy, None


def gather_mul_sum(x, w, gsi, ssi):
    """``segment_sum(gather(x, gsi) * w, ssi)`` without the [E, F] message tensor."""
    return _GatherMulSum.apply(x, w, gsi, ssi)


# ------------------------------------------------------------------ public API

def gather(x, si):
    """x[si.index] — row gather; backward is a deterministic CSR segment-sum."""
    return _Gather.apply(x, si)


def segment_sum(x, si, limit=None):
    """``limit`` (optional device int32 scalar): rows at or past it are padding and skipped
    (their values must be zero for the result to be exact; the GPU kernel then does no
    serial work on the padding graph's long segment)."""
    return _SegSum.apply(x, si, limit)


class _SegMean(torch.autograd.Function):
    """Native segment mean: the division rides in the segment-sum kernel (one launch instead
    of sum + clamp + divide); backward = gather of g / degree."""

    @staticmethod
    def forward(ctx, x, si, limit):
        ctx.si = si
        tail = x.shape[1:]
        lim = limit if limit is not None else si.limit
        if lim is not None and not (lim.dtype == torch.int32 and (si.perm is None or si.limit is lim)):
            lim = None
        out = _native.ops().seg_sum(x.reshape(x.shape[0], _width(tail)), si.rowptr, si.perm, si.num_segments, True,
                                    lim)
        return out.view((si.num_segments,) + tuple(tail))

    @staticmethod
    def backward(ctx, g):
        si = ctx.si
        inv = si.inv_degree(g.dtype)
        return _Gather.apply(g * inv.view(-1, *([1] * (g.dim() - 1))), si), None, None


def segment_mean(x, si, limit=None):
    if _use_native(x) and x.dtype == torch.float32 and x.dim() >= 1 and x.shape[0] > 0:
        return _SegMean.apply(x, si, limit)
    s = _SegSum.apply(x, si, limit)
    deg = si.degree(s.dtype).clamp(min=1.0).to(s.device)
    return s / deg.view(-1, *([1] * (s.dim() - 1)))


def segment_max(x, si):
    return _SegMinMax.apply(x, si, True)[0]


def segment_min(x, si):
    return _SegMinMax.apply(x, si, False)[0]


def segment_std(x, si, eps=1e-5):
    """PyG StdAggregation: sqrt(clamp(E[x^2]-E[x]^2, eps)), zeroed where <= sqrt(eps)."""
    mean = segment_mean(x, si)
    mean2 = segment_mean(x * x, si)
    var = mean2 - mean * mean
    out = var.clamp(min=eps).sqrt()
    return out.masked_fill(out <= eps ** 0.5, 0.0)


def segment_softmax(logits, si):
    """Softmax of edge logits within each destination segment (GATv2)."""
    mx = segment_max(logits.detach(), si)
    z = logits - gather(mx, si)
    ez = torch.exp(z)
    den = segment_sum(ez, si)
    return ez / (gather(den, si) + 1e-16)


def scatter_sum_index(x, index, num_segments):
    """Convenience: unsorted index -> segment sum (builds a SegIndex on the fly)."""
    si = SegIndex.from_index(index, num_segments)
    return segment_sum(x, si)


def scatter_mean_index(x, index, num_segments):
    si = SegIndex.from_index(index, num_segments)
    return segment_mean(x, si)
