"""SchNet stack (reference ``hydragnn/models/SCFStack.py:34-293``).

Continuous-filter convolution (``CFConv``, reference ``:214-293``):

    C_e = 0.5 (cos(pi d_e / cutoff) + 1)
    W_e = nn(GaussRBF(d_e) [ ⊕ e_e ]) * C_e           nn = Lin -> ShiftedSoftplus -> Lin
    x'  = lin2( sum_{e -> i} lin1(x)_{src(e)} * W_e )
    (equivariant, not last layer)  pos' = pos + mean_{e: src(e)=n} clamp(d̂_e coord_mlp(W_e), +-100)

Without edge attributes (and without GPS) the reference rebuilds the interaction
graph from the current positions in every layer (``RadiusInteractionGraph``); here
it is built once per forward when positions are static and per layer only for the
position-updating (equivariant) layers.  Aggregations are CSR segment sums (HIP).
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

from ..ops import segment as seg
from ..ops.geometry import GaussianSmearing, cosine_cutoff, edge_vectors_and_lengths
from ..ops.radius import interaction_graph, interaction_graph_static
from .layers import Linear
from .base import Base


class ShiftedSoftplus(nn.Module):
    def __init__(self):
        super().__init__()
        self.shift = math.log(2.0)

    def forward(self, x):
        return F.softplus(x) - self.shift


class _CFFilter(torch.autograd.Function):
    """W = (ssp(rbf W1^T + b1) W2^T + b2) * C in one HIP launch each way (csrc/schnet.hip).
    The backward kernel emits the row factors of the four weight/bias gradients; they join
    the step's deferred grouped weight-gradient launch (ops/linear.py) when it is open, else
    one grouped launch here."""

    @staticmethod
    def forward(ctx, rbf, C, W1, b1, W2, b2):
        from .. import _native

        Wf, H1 = _native.ops().cf_filter_fwd(rbf, W1, b1, W2, b2, C)
        ctx.save_for_backward(rbf, C, H1, W2)
        ctx.params = (W1, b1, W2, b2)
        return Wf

    @staticmethod
    def backward(ctx, g):
        from .. import _native
        from ..ops import linear as _lin

        rbf, C, H1, W2 = ctx.saved_tensors
        dH2, A1, dH1 = _native.ops().cf_filter_bwd(g, C, H1, W2)
        W1p, b1p, W2p, b2p = ctx.params
        if _lin._can_defer(W1p, b1p) and _lin._can_defer(W2p, b2p):
            _lin._record((dH2, A1, W2p, b2p))
            _lin._record((dH1, rbf, W1p, b1p))
            return None, None, None, None, None, None
        dW1, db1 = torch.empty_like(W1p), torch.empty_like(b1p)
        dW2, db2 = torch.empty_like(W2p), torch.empty_like(b2p)
        _native.ops().linear_wgrad_grouped([dH2, dH1], [A1, rbf], [dW2, dW1], [db2, db1], [0, 0])
        return None, None, dW1, db1, dW2, db2


def _filter_fusable(nn_, h, C):
    from ..ops.pna import fused

    if not (h.is_cuda and h.dtype == torch.float32 and h.dim() == 2 and h.shape[1] <= 64 and fused("cfconv")
            and not h.requires_grad and not C.requires_grad and isinstance(nn_, nn.Sequential) and len(nn_) == 3):
        return False
    l1, act, l2 = nn_[0], nn_[1], nn_[2]
    return (isinstance(l1, nn.Linear) and isinstance(act, ShiftedSoftplus) and isinstance(l2, nn.Linear)
            and l1.bias is not None and l2.bias is not None and l1.in_features == h.shape[1]
            and l1.out_features == l2.in_features == l2.out_features <= 64)


class CFConv(nn.Module):
    def __init__(self, in_channels, out_channels, num_filters, nn_, cutoff, equivariant):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.lin1 = Linear(in_channels, num_filters, bias=False)
        self.lin2 = Linear(num_filters, out_channels)
        self.nn = nn_
        self.cutoff = cutoff
        self.equivariant = equivariant
        if equivariant:
            layer = Linear(num_filters, 1, bias=False)
            nn.init.xavier_uniform_(layer.weight, gain=0.001)
            self.coord_mlp = nn.Sequential(Linear(num_filters, num_filters), nn.ReLU(), layer)
        nn.init.xavier_uniform_(self.lin1.weight)
        nn.init.xavier_uniform_(self.lin2.weight)
        self.lin2.bias.data.fill_(0)

    def forward(self, inv, equiv, ctx):
        pos = equiv
        g = ctx.layer_graph(self, pos)  # (dst_si, src_si, dist, rbf, edge_attr)
        dst_si, src_si, dist, rbf, eattr = g
        C = cosine_cutoff(dist, self.cutoff, masked=False)  # one launch on the GPU
        h = rbf if eattr is None else torch.cat([rbf, eattr], -1)
        if _filter_fusable(self.nn, h, C):
            l1, l2 = self.nn[0], self.nn[2]
            W = _CFFilter.apply(h, C.reshape(-1).contiguous(), l1.weight, l1.bias, l2.weight, l2.bias)
        else:
            W = self.nn(h) * C.view(-1, 1)
        x = self.lin1(inv)
        if self.equivariant:
            coord_diff, _ = edge_vectors_and_lengths(pos, dst_si, src_si, None, normalize=True, eps=1.0)
            trans = (coord_diff * self.coord_mlp(W)).clamp(-100.0, 100.0)
            pos = pos + seg.segment_mean(trans, src_si)
        x = seg.gather_mul_sum(x, W, src_si, dst_si)  # gather * filter -> segment sum, one pass
        return self.lin2(x), pos

    def __repr__(self):
        return f"CFConv({self.in_channels}, {self.out_channels}, equivariant={self.equivariant})"


class SCFStack(Base):
    is_edge_model = True

    @property
    def capturable(self):
        # a statically padded batch rebuilds the in-forward radius graph with fixed capacity
        # (ops.radius.interaction_graph_static: no host sync), equivariant layers included
        return True

    def __init__(self, input_args, conv_args, num_filters, edge_dim, num_gaussians, radius, *args,
                 max_neighbours=None, **kwargs):
        self.radius = radius
        self.max_neighbours = max_neighbours
        self.num_filters = num_filters
        self.edge_dim = edge_dim
        self.num_gaussians = num_gaussians
        super().__init__(input_args, conv_args, *args, **kwargs)

    def _init_conv(self):
        self.distance_expansion = GaussianSmearing(0.0, self.radius, self.num_gaussians)
        n = self.num_conv_layers
        self.graph_convs.append(self._apply_global_attn(
            self.get_conv(self.embed_dim, self.hidden_dim, n == 1, edge_dim=self.edge_embed_dim)))
        self.feature_layers.append(nn.Identity())
        for i in range(n - 1):
            self.graph_convs.append(self._apply_global_attn(
                self.get_conv(self.hidden_dim, self.hidden_dim, i == n - 2, edge_dim=self.edge_embed_dim)))
            self.feature_layers.append(nn.Identity())

    def get_conv(self, input_dim, output_dim, last_layer=False, edge_dim=None):
        mlp_in = self.num_gaussians + edge_dim if edge_dim else self.num_gaussians
        mlp = nn.Sequential(Linear(mlp_in, self.num_filters), ShiftedSoftplus(),
                            Linear(self.num_filters, self.num_filters))
        return CFConv(input_dim, output_dim, self.num_filters, mlp, self.radius,
                      equivariant=self.equivariance and not last_layer)

    def _conv_head_kwargs(self):
        return {"last_layer": False, **super()._conv_head_kwargs()}

    def _embedding(self, data):
        x, pos, ctx = super()._embedding(data)
        with_edges = self.use_edge_attr or (self.use_global_attn and self.is_edge_model)
        if with_edges and self.equivariance:
            raise Exception("For SchNet if using edge attributes or edge encodings for gps, then E(3)-equivariance "
                            "cannot be ensured. Please disable equivariance or edge attributes.")
        stack = self
        cache = {}

        # statically padded (captured) batch: the in-forward radius graph (SCFStack.py:175-190)
        # is rebuilt on the device with a fixed edge capacity, so the step has static shapes
        static_graph = data.get("graph_mask") is not None

        def layer_graph(conv, p):
            if static_graph and not with_edges:
                key = "g" if not conv.equivariant else None
                if key is not None and "g" in cache:
                    return cache["g"]
                dst_si, src_si = interaction_graph_static(p, data, stack.radius, stack.max_neighbours)
                _, d = edge_vectors_and_lengths(p, dst_si, src_si, None)
                d = d.view(-1)
                g = (dst_si, src_si, d, stack.distance_expansion(d), None)
                if not conv.equivariant:
                    cache["g"] = g
                return g
            if with_edges:  # data edges, no PBC shifts (reference overrides shifts with zeros)
                if "g" not in cache:
                    _, d = edge_vectors_and_lengths(p, ctx.dst_si, ctx.src_si, None)
                    d = d.view(-1)
                    cache["g"] = (ctx.dst_si, ctx.src_si, d, stack.distance_expansion(d),
                                  ctx.edge_attr if with_edges else None)
                return cache["g"]
            key = "g" if not conv.equivariant and "static" in cache else None
            if key is not None:
                return cache["g"]
            dst_si, src_si = interaction_graph(p, data.batch, stack.radius, stack.max_neighbours)
            _, d = edge_vectors_and_lengths(p, dst_si, src_si, None)
            d = d.view(-1)
            g = (dst_si, src_si, d, stack.distance_expansion(d), None)
            if not stack.equivariance:
                cache["g"], cache["static"] = g, True
            return g

        ctx.layer_graph = layer_graph
        return x, pos, ctx

    def __str__(self):
        return "SCFStack"
