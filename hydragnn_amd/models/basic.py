"""Non-geometric stacks: GIN, SAGE, MFC (reference ``models/GINStack.py``,
``SAGEStack.py``, ``MFCStack.py``; PyG GINConv / SAGEConv / MFConv semantics).

All aggregations are CSR segment reductions over destination-sorted edges
(``ops.segment``): deterministic, atomic-free, differentiable to any order.
"""
import torch
from torch import nn

from ..ops import segment as seg
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
        deg = ctx.dst_si.degree().to(inv.device).clamp(max=self.max_degree).long()
        Wl = torch.cat([l.weight for l in self.lins_l], 0)
        Wr = torch.cat([l.weight for l in self.lins_r], 0)
        bl = torch.cat([l.bias for l in self.lins_l], 0) if self.lins_l[0].bias is not None else None
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
