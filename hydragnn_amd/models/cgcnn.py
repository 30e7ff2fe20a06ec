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

from ..ops import segment as seg
from ..ops.linear import linear
from .layers import Linear
from .base import Base


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
        ij = seg.gather(nb[:, :2 * C], ctx.dst_si) + seg.gather(nb[:, 2 * C:], ctx.src_si)
        bias = None
        if self.lin_f.bias is not None:
            bias = torch.cat([self.lin_f.bias, self.lin_s.bias])
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
