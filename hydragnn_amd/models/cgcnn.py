"""CGCNN stack (reference ``hydragnn/models/CGCNNStack.py:19-113`` over PyG ``CGConv``).

    z_e = cat[x_i, x_j, e_e]          (i = destination, j = source)
    x'  = x + sum_{e -> i} sigmoid(lin_f z_e) * softplus(lin_s z_e)

``lin_f`` and ``lin_s`` act on the same concatenation: both are evaluated as ONE
fused node-level GEMM for the x_i / x_j blocks ([N, 4C]: f_i, s_i, f_j, s_j),
gathered per edge, plus an edge-level GEMM for the e block.  Without GPS the
hidden dimension equals the input dimension (CGConv keeps its width).
"""
import torch
import torch.nn.functional as F
from torch import nn

from .. import _native
from ..ops import segment as seg
from ..ops.linear import linear
from ..ops.pna import fused
from .layers import Linear
from .base import Base


class _CGGate(torch.autograd.Function):
    """sum_{e->i} sigmoid(z_e) softplus(s_e) in one launch (csrc/conv_misc.hip); backward:
    one launch for the per-edge gate gradients + one by-source CSR segment sum."""

    @staticmethod
    def forward(ctx, nb, et, bias, dst_si, src_si):
        out = _native.ops().cg_gate_fwd(nb, et, bias, dst_si.rowptr, src_si.index)
        ctx.save_for_backward(nb, et, bias)
        ctx.si = (dst_si, src_si)
        return out

    @staticmethod
    def backward(ctx, g):
        nb, et, bias = ctx.saved_tensors
        dst_si, src_si = ctx.si
        G, dnd = _native.ops().cg_gate_bwd(g, nb, et, bias, dst_si.rowptr, src_si.index)
        dnb = torch.cat([dnd, seg.segment_sum(G, src_si)], 1)
        return dnb, (G if et is not None else None), (G.sum(0) if bias is not None else None), None, None


class CGConv(nn.Module):
    def __init__(self, channels, dim=0, aggr="add", batch_norm=False, bias=True):
        super().__init__()
        assert aggr == "add" and not batch_norm, "HydraGNN uses CGConv(aggr='add', batch_norm=False)"
        self.channels = channels
        self.dim = dim or 0
        self.lin_f = Linear(2 * channels + self.dim, channels, bias=bias)
        self.lin_s = Linear(2 * channels + self.dim, channels, bias=bias)

    def forward(self, inv, equiv, ctx):
        x = inv
        C = self.channels
        Wf, Ws = self.lin_f.weight, self.lin_s.weight
        # node blocks: [f_i | s_i | f_j | s_j]
        Wn = torch.cat([Wf[:, :C], Ws[:, :C], Wf[:, C:2 * C], Ws[:, C:2 * C]], 0)
        nb = linear(x, Wn)
        bias = None
        if self.lin_f.bias is not None:
            bias = torch.cat([self.lin_f.bias, self.lin_s.bias])
        if x.is_cuda and x.dtype == torch.float32 and fused("cggate"):
            et = None
            if self.dim and ctx.edge_attr is not None:
                et = linear(ctx.edge_attr, torch.cat([Wf[:, 2 * C:], Ws[:, 2 * C:]], 0), bias).contiguous()
            m = _CGGate.apply(nb.contiguous(), et, bias if et is None else None, ctx.dst_si, ctx.src_si)
            return x + m, equiv
        ij = seg.gather(nb[:, :2 * C], ctx.dst_si) + seg.gather(nb[:, 2 * C:], ctx.src_si)
        if self.dim and ctx.edge_attr is not None:
            ij = ij + linear(ctx.edge_attr, torch.cat([Wf[:, 2 * C:], Ws[:, 2 * C:]], 0), bias)
        elif bias is not None:
            ij = ij + bias
        m = torch.sigmoid(ij[:, :C]) * F.softplus(ij[:, C:])
        return x + seg.segment_sum(m, ctx.dst_si), equiv

    def __repr__(self):
        return f"CGConv({self.channels}, dim={self.dim})"


class CGCNNStack(Base):
    is_edge_model = True

    def __init__(self, input_args, conv_args, edge_dim, input_dim, hidden_dim, output_dim, *args, **kwargs):
        self.edge_dim = edge_dim
        super().__init__(input_args, conv_args, input_dim, hidden_dim, output_dim, *args, **kwargs)

    def get_conv(self, input_dim, _, edge_dim=None):
        return CGConv(channels=input_dim, dim=edge_dim, aggr="add", batch_norm=False, bias=True)

    def _init_node_conv(self):
        node_feature_ind = [i for i, t in enumerate(self.head_type) if t == "node"]
        if not node_feature_ind:
            return
        for b in self.config_heads["node"]:
            if b["architecture"]["type"] != "conv":
                return
        raise ValueError('"conv" for node features decoder part in CGCNN is not ready yet. Please set '
                         'config["NeuralNetwork"]["Architecture"]["output_heads"]["node"]["type"] to be "mlp" or '
                         '"mlp_per_node" in input file.')

    def __str__(self):
        return "CGCNNStack"
