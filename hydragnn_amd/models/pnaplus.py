"""PNA and PNAPlus stacks (reference ``hydragnn/models/PNAStack.py:19-70``,
``hydragnn/models/PNAPlusStack.py:40-304``).

PNAPlus message (towers=1, pre/post_layers=1):
    m_e = pre_nn(cat[x_i, x_j, edge_encoder(cat[e, relu(rbf_emb(rbf))])]) * rbf_lin(rbf)
PNA message:
    m_e = pre_nn(cat[x_i, x_j(, edge_encoder(e))])
Both: Z = cat[x, aggr(m)] (4 aggregators x 4 degree scalers) -> post_nn -> lin.

MI355X mapping: ``pre_nn`` is split column-wise (concat-linear decomposition):
the x_i / x_j blocks are applied at node level in ONE GEMM producing
``AB = x @ [W_i; W_j]^T`` [N, 2F]; the edge block is pre-multiplied into the
edge encoder (``W_e @ W_enc``), so the only edge-row GEMM per layer is
[E, F+d] x [F+d, F].  Gather + add + gate + 4-way segment statistics + scalers +
concat run in one fused HIP kernel (``ops.pna.pna_message_aggregate``).
Parameter names match the reference (``pre_nns.0.0``, ``post_nns.0.0``, ``lin``,
``rbf_lin``, ``rbf_emb.0``, ``edge_encoder``).
"""
import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import ModuleList, Sequential

from ..ops.geometry import BesselBasis, edge_vectors_and_lengths
from ..ops.linear import linear, linear_sum
from ..ops.pna import pna_avg_deg, pna_message_aggregate
from .base import Base
from .layers import Linear


class PNAConvFused(nn.Module):
    def __init__(self, in_channels, out_channels, deg, edge_dim=None, num_radial=None, plus=True,
                 aggregators=("mean", "min", "max", "std"),
                 scalers=("identity", "amplification", "attenuation", "linear")):
        super().__init__()
        assert tuple(aggregators) == ("mean", "min", "max", "std") and \
            tuple(scalers) == ("identity", "amplification", "attenuation", "linear"), \
            "fused PNA kernel implements the reference aggregator/scaler set"
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.edge_dim = edge_dim
        self.plus = plus
        Fi = in_channels
        self.F_in, self.F_out = Fi, out_channels
        n_in = 3 if (plus or edge_dim is not None) else 2
        self.pre_nns = ModuleList([Sequential(Linear(n_in * Fi, Fi))])
        self.post_nns = ModuleList([Sequential(Linear(17 * Fi, out_channels))])
        self.lin = Linear(out_channels, out_channels)
        if plus:
            self.rbf_lin = Linear(num_radial, Fi, bias=False)
            self.rbf_emb = Sequential(Linear(num_radial, Fi), nn.ReLU())
            if edge_dim is not None:
                self.edge_encoder = Linear(Fi + edge_dim, Fi)
        elif edge_dim is not None:
            self.edge_encoder = Linear(edge_dim, Fi)
        self.register_buffer("deg", torch.as_tensor(deg, dtype=torch.float32))
        self.avg_deg = pna_avg_deg(self.deg)

    def forward(self, inv, equiv, ctx):
        x = inv
        Fi = self.F_in
        pre = self.pre_nns[0][0]
        W, b = pre.weight, pre.bias
        # AB[:, :F] = W_i x + b (x_i, destination), AB[:, F:] = W_j x (x_j, source): one node GEMM
        AB = linear(x, torch.cat([W[:, :Fi], W[:, Fi:2 * Fi]], 0), torch.cat([b, torch.zeros_like(b)]))
        C = None
        G = None
        if self.plus:
            rbf = ctx.rbf
            r = self.rbf_emb(rbf)
            We = W[:, 2 * Fi:]
            if self.edge_dim is not None and ctx.edge_attr is not None:
                enc = self.edge_encoder
                Wc = We @ enc.weight  # [F, d + F]
                bc = We @ enc.bias
                d = self.edge_dim
                C = linear_sum([(r, Wc[:, d:]), (ctx.edge_attr, Wc[:, :d])], bc)
            else:
                C = linear(r, We, None)
            G = self.rbf_lin(rbf)
        elif self.edge_dim is not None and ctx.edge_attr is not None:
            We = W[:, 2 * Fi:]
            C = linear(ctx.edge_attr, We @ self.edge_encoder.weight, We @ self.edge_encoder.bias)
        Z = pna_message_aggregate(x, AB, C, G, ctx.dst_si, ctx.src_si, self.avg_deg)
        out = self.post_nns[0](Z)
        return self.lin(out), equiv

    def __repr__(self):
        return f"PNAConv{'Plus' if self.plus else ''}({self.in_channels}, {self.out_channels}, edge_dim={self.edge_dim})"


class PNAPlusStack(Base):
    is_edge_model = True

    def __init__(self, input_args, conv_args, deg, edge_dim, envelope_exponent, num_radial, radius, *args,
                 **kwargs):
        self.aggregators = ["mean", "min", "max", "std"]
        self.scalers = ["identity", "amplification", "attenuation", "linear"]
        self.deg = torch.as_tensor(deg, dtype=torch.float32)
        self.edge_dim = edge_dim
        self.envelope_exponent = envelope_exponent
        self.num_radial = num_radial
        self.radius = radius
        super().__init__(input_args, conv_args, *args, **kwargs)
        self.rbf = BesselBasis(num_radial, radius, envelope_exponent)

    def get_conv(self, input_dim, output_dim, edge_dim=None):
        return PNAConvFused(input_dim, output_dim, self.deg, edge_dim=edge_dim, num_radial=self.num_radial,
                            plus=True)

    def _embedding(self, data):
        x, pos, ctx = super()._embedding(data)
        assert data.pos is not None, "PNA+ requires node positions (data.pos) to be set."
        _, dist = edge_vectors_and_lengths(data.pos, ctx.dst_si, ctx.src_si, data.get("edge_shifts"))
        ctx.rbf = self.rbf(dist.squeeze(-1))
        return x, pos, ctx

    def __str__(self):
        return "PNAPlusStack"


class PNAStack(Base):
    is_edge_model = True

    def __init__(self, input_args, conv_args, deg, edge_dim, *args, **kwargs):
        self.aggregators = ["mean", "min", "max", "std"]
        self.scalers = ["identity", "amplification", "attenuation", "linear"]
        self.deg = torch.as_tensor(deg, dtype=torch.float32)
        self.edge_dim = edge_dim
        super().__init__(input_args, conv_args, *args, **kwargs)

    def get_conv(self, input_dim, output_dim, edge_dim=None):
        return PNAConvFused(input_dim, output_dim, self.deg, edge_dim=edge_dim, plus=False)

    def __str__(self):
        return "PNAStack"
