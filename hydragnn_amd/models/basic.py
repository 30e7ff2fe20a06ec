"""Non-geometric stacks: GIN, SAGE, MFC (reference ``models/GINStack.py``,
``SAGEStack.py``, ``MFCStack.py``; PyG GINConv / SAGEConv / MFConv semantics).

All aggregations are CSR segment reductions over destination-sorted edges
(``ops.segment``): deterministic, atomic-free, differentiable to any order.
"""
import torch
from torch import nn

from ..ops import segment as seg
from ..ops.pna import fused
from .base import Base
from .layers import Linear


class GINConv(nn.Module):
    """out = nn((1 + eps) * x_i + sum_j x_j), eps learnable (init 100, ``GINStack.py:26-35``)."""

    def __init__(self, mlp, eps=0.0, train_eps=False):
        super().__init__()
        self.nn = mlp
        self.initial_eps = eps
        if train_eps:
            self.eps = nn.Parameter(torch.tensor([float(eps)]))
        else:
            self.register_buffer("eps", torch.tensor([float(eps)]))

    def forward(self, inv, equiv, ctx):
        agg = seg.segment_sum(seg.gather(inv, ctx.src_si), ctx.dst_si)
        return self.nn((1 + self.eps) * inv + agg), equiv


class SAGEConv(nn.Module):
    """out = lin_l(mean_j x_j) + lin_r(x_i) (PyG SAGEConv defaults, ``SAGEStack.py:26-31``)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.lin_l = Linear(in_channels, out_channels, bias=True)
        self.lin_r = Linear(in_channels, out_channels, bias=False)

    def forward(self, inv, equiv, ctx):
        agg = seg.segment_mean(seg.gather(inv, ctx.src_si), ctx.dst_si)
        return self.lin_l(agg) + self.lin_r(inv), equiv


class _MFBanks(torch.autograd.Function):
    """Per-node degree bank (csrc/conv_misc.hip): each node multiplies only its own bank
    forward and input-gradient; the weight gradient is one GEMM against the gradient
    scattered into its degree column block."""

    @staticmethod
    def forward(ctx, h, x, Wl, bl, Wr, rowptr, maxd):
        from .. import _native

        out = _native.ops().mf_fwd(h, x, Wl, bl, Wr, rowptr, maxd)
        ctx.save_for_backward(h, x, Wl, Wr, rowptr)
        ctx.maxd, ctx.has_b = maxd, bl is not None
        return out

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        h, x, Wl, Wr, rowptr = ctx.saved_tensors
        D1 = ctx.maxd + 1
        N, O = g.shape
        dh, dx = _native.ops().mf_dgrad(g, Wl, Wr, rowptr, ctx.maxd, h.shape[1])
        d = (rowptr[1:] - rowptr[:-1]).clamp(max=ctx.maxd).long()
        gexp = g.new_zeros(N, D1, O).scatter_(1, d.view(-1, 1, 1).expand(-1, 1, O), g.view(N, 1, O)).view(N, D1 * O)
        dWl = gexp.t() @ h
        dWr = gexp.t() @ x
        dbl = gexp.sum(0) if ctx.has_b else None
        return dh, dx, dWl, dbl, dWr, None, None


class MFConv(nn.Module):
    """Degree-specific weights: out_i = W_l[d_i] sum_j x_j + W_r[d_i] x_i, d_i = min(deg_i, max_degree).

    Implemented without host syncs: one GEMM against the stacked [D+1] weight
    banks, then a per-node gather of its degree block (PyG MFConv loops over
    degrees with ``nonzero``)."""

    def __init__(self, in_channels, out_channels, max_degree=10, bias=True):
        super().__init__()
        self.max_degree = max_degree
        self.out_channels = out_channels
        self.lins_l = nn.ModuleList([Linear(in_channels, out_channels, bias=bias) for _ in range(max_degree + 1)])
        self.lins_r = nn.ModuleList([Linear(in_channels, out_channels, bias=False) for _ in range(max_degree + 1)])

    def forward(self, inv, equiv, ctx):
        h = seg.segment_sum(seg.gather(inv, ctx.src_si), ctx.dst_si)
        Wl = torch.cat([l.weight for l in self.lins_l], 0)
        Wr = torch.cat([l.weight for l in self.lins_r], 0)
        bl = torch.cat([l.bias for l in self.lins_l], 0) if self.lins_l[0].bias is not None else None
        if inv.is_cuda and inv.dtype == torch.float32 and fused("mfconv"):
            return _MFBanks.apply(h.contiguous(), inv.contiguous(), Wl, bl, Wr, ctx.dst_si.rowptr,
                                  self.max_degree), equiv
        deg = ctx.dst_si.degree().to(inv.device).clamp(max=self.max_degree).long()
        y = torch.nn.functional.linear(h, Wl, bl) + torch.nn.functional.linear(inv, Wr)
        D1, O = self.max_degree + 1, self.out_channels
        y = y.view(-1, D1, O)
        out = torch.gather(y, 1, deg.view(-1, 1, 1).expand(-1, 1, O)).squeeze(1)
        return out, equiv


class GINStack(Base):
    is_edge_model = False

    def get_conv(self, input_dim, output_dim, edge_dim=None):
        return GINConv(nn.Sequential(Linear(input_dim, output_dim), nn.ReLU(), Linear(output_dim, output_dim)),
                       eps=100.0, train_eps=True)

    def __str__(self):
        return "GINStack"


class SAGEStack(Base):
    is_edge_model = False

    def get_conv(self, input_dim, output_dim, edge_dim=None):
        return SAGEConv(input_dim, output_dim)

    def __str__(self):
        return "SAGEStack"


class MFCStack(Base):
    is_edge_model = False

    def __init__(self, input_args, conv_args, max_degree, *args, **kwargs):
        self.max_degree = max_degree
        super().__init__(input_args, conv_args, *args, **kwargs)

    def get_conv(self, input_dim, output_dim, edge_dim=None):
        return MFConv(input_dim, output_dim, max_degree=self.max_degree)

    def __str__(self):
        return "MFCStack"
