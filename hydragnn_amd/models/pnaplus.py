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
from ..ops.pna import pna_avg_deg, pna_message_aggregate, pna_weight_prep
from ..ops.radial import fused_ok, radial_features
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
        # parameter creation and initialisation in the reference's order, draw for draw (the
        # init seed then reproduces the reference's initial weights): PyG PNAConv creates its
        # edge encoder first; the PNAPlus conv (PNAPlusStack.py:180-210) creates it last; both
        # then re-draw edge encoder, pre-, post-NN and lin in reset_parameters
        # (PNAPlusStack.py:212-220, PyG PNAConv.reset_parameters)
        if not plus and edge_dim is not None:
            self.edge_encoder = Linear(edge_dim, Fi)
        self.pre_nns = ModuleList([Sequential(Linear(n_in * Fi, Fi))])
        self.post_nns = ModuleList([Sequential(Linear(17 * Fi, out_channels))])
        self.lin = Linear(out_channels, out_channels)
        if plus:
            self.rbf_lin = Linear(num_radial, Fi, bias=False)
            self.rbf_emb = Sequential(Linear(num_radial, Fi), nn.ReLU())
            if edge_dim is not None:
                self.edge_encoder = Linear(Fi + edge_dim, Fi)
        self.register_buffer("deg", torch.as_tensor(deg, dtype=torch.float32))
        self.avg_deg = pna_avg_deg(self.deg)
        self.reset_parameters()

    def reset_parameters(self):
        if getattr(self, "edge_encoder", None) is not None:
            self.edge_encoder.reset_parameters()
        self.pre_nns[0][0].reset_parameters()
        self.post_nns[0][0].reset_parameters()
        self.lin.reset_parameters()

    def forward(self, inv, equiv, ctx):
        x = inv
        Fi = self.F_in
        pre = self.pre_nns[0][0]
        W, b = pre.weight, pre.bias
        C = None
        G = None
        if self.plus and self.edge_dim is not None and ctx.edge_attr is not None:
            # all weight algebra in one launch; the pre_nn bias rides on the edge term C
            enc = self.edge_encoder
            Wab, Wr, Wd, bc = pna_weight_prep(W, b, enc.weight, enc.bias)
            AB = linear(x, Wab, None)
            r, G = self._radial(ctx)
            C = linear_sum([(r, Wr), (ctx.edge_attr, Wd)], bc)
        else:
            # AB[:, :F] = W_i x + b (x_i, destination), AB[:, F:] = W_j x (x_j, source): one node GEMM
            AB = linear(x, torch.cat([W[:, :Fi], W[:, Fi:2 * Fi]], 0), torch.cat([b, torch.zeros_like(b)]))
            We = W[:, 2 * Fi:]
            if self.plus:
                r, G = self._radial(ctx)
                C = linear(r, We, None)
            elif self.edge_dim is not None and ctx.edge_attr is not None:
                C = linear(ctx.edge_attr, We @ self.edge_encoder.weight, We @ self.edge_encoder.bias)
        Z = pna_message_aggregate(x, AB, C, G, ctx.dst_si, ctx.src_si, self.avg_deg)
        out = self.post_nns[0](Z)
        return self.lin(out), equiv

    def _radial(self, ctx):
        """(ReLU(rbf_emb(rbf)), rbf_lin(rbf)): precomputed for the whole stack by the
        fused radial kernel when available (``ctx.radial``), else from ``ctx.rbf``."""
        rad = ctx.get("radial")
        if rad is not None and id(self) in rad:
            return rad[id(self)]
        rbf = ctx.rbf if ctx.get("rbf") is not None else ctx.rbf_basis(ctx.dist)
        return self.rbf_emb(rbf), self.rbf_lin(rbf)

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
        ctx.geom = (data.pos, data.get("edge_shifts"))
        if ctx.get("gps_lazy") and not data.pos.requires_grad:
            ctx.dist = None  # the fused encoder computes the distances inside its radial launch
        else:
            ctx.dist = self._edge_dist(ctx)
        ctx.rbf_basis, ctx.rbf, ctx.radial = self.rbf, None, None
        return x, pos, ctx

    @staticmethod
    def _edge_dist(ctx):
        pos, shifts = ctx.geom
        return edge_vectors_and_lengths(pos, ctx.dst_si, ctx.src_si, shifts)[1].squeeze(-1)

    def _materialize_radial(self, ctx):
        """Radial features of the module path (the fused encoder computes its own)."""
        if ctx.get("dist") is None:
            ctx.dist = self._edge_dist(ctx)
        if ctx.get("radial") is not None or ctx.get("rbf") is not None:
            return
        convs = self._stack_convs()
        if fused_ok(ctx.dist, self.rbf, convs):
            # Bessel basis + every layer's rbf_emb/rbf_lin in one launch (ops/radial.py)
            ctx.radial = {id(c): rg for c, rg in zip(convs, radial_features(ctx.dist, self.rbf, convs))}
        else:
            ctx.rbf = self.rbf(ctx.dist)

    def _gps_embed_lazy(self, data):
        from ..ops import gps_encoder

        return gps_encoder.pre_eligible(self, data)

    def _fused_encode(self, inv, equiv, ctx):
        # GPS + PNAPlus training on the GPU: embedding + radial basis + the whole conv stack in
        # one autograd function over csrc/gps_fused.hip (ops/gps_encoder.py)
        from ..ops import gps_encoder

        if self.use_global_attn and ctx.get("gps_lazy") and gps_encoder.eligible(self, ctx):
            return gps_encoder.encode(self, ctx), equiv, ctx
        self._materialize_radial(ctx)
        return None

    def _stack_convs(self):
        out = []
        for c in self.graph_convs:
            c = getattr(c, "conv", c)  # GPS wraps the local conv
            if isinstance(c, PNAConvFused) and c.plus:
                out.append(c)
        return out

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
