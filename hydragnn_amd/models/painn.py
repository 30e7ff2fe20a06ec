"""PAINN and PNAEq stacks (reference ``hydragnn/models/PAINNStack.py:27-343`` and
``hydragnn/models/PNAEqStack.py:41-493``).

Both carry a scalar state s [N, F] and a vector state v [N, 3, F] (zero-initialised).
Note the message direction of the reference: edge e = (src, dst) = edge_index[:, e];
node states are gathered at ``dst`` and summed onto ``src`` (``index_add_(0,
edge[:, 0], ...)``), i.e. CSR-by-source segment sums here (deterministic).

PAINN message (``PAINNStack.py:194-263``):
    W_e   = filter(sinc(d_e)) * cos_cutoff(d_e) [* edge_filter(e_e)]            [E, 3F]
    (g_v, g_e, m_s) = split(W_e * scalar_mlp(s)[dst])
    m_v   = v[dst] * g_v + g_e * (d̂_e / d_e)                                     (reference quirk: d̂/d)
    s += sum_src m_s ;  v += sum_src m_v

PNAEq message (``PNAEqStack.py:224-394``): PNA-style pre_nn over cat[s_src, s_dst,
rbf_emb(rbf)(, enc(e))], scalar_mlp, rbf_lin gate, 4 aggregators x 5 scalers
(incl. inverse_linear) at the source, post_nn.

Update (both): U v, V v -> a_vv, a_sv, a_ss = mlp(cat[|V v|, s]);
    v += a_vv * U v ;  s += a_sv * <U v, V v> + a_ss
followed by the reference's size adapters (node_embed_out: Lin-Tanh-Lin,
vec_embed_out: Lin on the channel dim).  Deliberate fix: every Linear acting on the
vector state (U, V, vec_embed_out) is bias-free here; the reference's biases add the
same offset to all three Cartesian components and break rotation equivariance.
"""

import torch
from torch import nn

from ..ops import segment as seg
from ..ops import geometry as _geo
from ..ops.geometry import edge_vectors_and_lengths
from ..ops.pna import degree_scalers, pna_aggregate, pna_avg_deg
from .layers import Linear
from .base import Base


def sinc_expansion(edge_dist, num_radial, cutoff):
    """[E, 1] distances -> [E, num_radial] (one launch on the GPU, ops/geometry.py)."""
    return _geo.sinc_expansion(edge_dist.reshape(-1), num_radial, cutoff)


def cosine_cutoff(edge_dist, cutoff):
    return _geo.cosine_cutoff(edge_dist, cutoff, masked=True)


class rbf_BasisLayer(nn.Module):
    """sinc(n pi d / c) / d * cosine_cutoff(d)  (reference ``PNAEqStack.py:453-493``)."""

    def __init__(self, num_radial, cutoff):
        super().__init__()
        self.num_radial, self.cutoff = num_radial, cutoff

    def forward(self, edge_dist):
        d = edge_dist.unsqueeze(-1)
        return sinc_expansion(d, self.num_radial, self.cutoff) * cosine_cutoff(d, self.cutoff)


class PainnMessage(nn.Module):
    def __init__(self, node_size, num_radial, cutoff, edge_dim):
        super().__init__()
        self.node_size, self.num_radial, self.cutoff, self.edge_dim = node_size, num_radial, cutoff, edge_dim
        F = node_size
        self.scalar_message_mlp = nn.Sequential(Linear(F, F), nn.SiLU(), Linear(F, 3 * F))
        self.filter_layer = Linear(num_radial, 3 * F)
        if edge_dim is not None:
            self.edge_filter = nn.Sequential(Linear(edge_dim, F), nn.SiLU(), Linear(F, 3 * F))

    def _edge_terms(self, ctx):
        """Layer-independent edge terms — sinc basis, cosine cutoff, d̂/d as [E, 3, 1] —
        computed once per forward and shared by every message layer (the reference
        recomputes them per layer, ``PAINNStack.py:228-236``; same values)."""
        key = ("painn_edge", self.num_radial, float(self.cutoff))
        cache = ctx.get("_painn_cache")
        if cache is None:
            cache = {}
            ctx._painn_cache = cache
        if key not in cache:
            d = ctx.edge_dist
            cache[key] = (sinc_expansion(d, self.num_radial, self.cutoff), cosine_cutoff(d, self.cutoff),
                          (ctx.edge_diff / d).unsqueeze(-1))
        return cache[key]

    def forward(self, s, v, ctx):
        F = self.node_size
        rbf, cut, unit = self._edge_terms(ctx)
        W = self.filter_layer(rbf) * cut
        if ctx.edge_attr is not None and self.edge_dim is not None:
            W = W * self.edge_filter(ctx.edge_attr)
        out = W * seg.gather(self.scalar_message_mlp(s), ctx.dst_si)
        # one split (backward: one concat) instead of three slices (a zero-fill + copy each,
        # at every order of differentiation under force training)
        g_v, g_e, m_s = out.split(F, 1)
        m_v = seg.gather(v, ctx.dst_si) * g_v.unsqueeze(1) + g_e.unsqueeze(1) * unit
        s = s + seg.segment_sum(m_s, ctx.src_si)
        v = v + seg.segment_sum(m_v, ctx.src_si)
        return s, v


def safe_vector_norm(v, dim):
    """||v|| with a zero (not NaN) first AND second derivative at v = 0.

    Nodes with no incoming message keep v = 0 (padding atoms of a captured bucket, or
    isolated atoms); ``torch.linalg.vector_norm``'s double backward is 0/0 there, which
    poisons force training (``energy_force_loss`` differentiates twice).  Equal to the
    plain norm wherever v != 0."""
    n2 = (v * v).sum(dim)
    nz = n2 > 0
    return torch.where(nz, torch.sqrt(torch.where(nz, n2, torch.ones_like(n2))), torch.zeros_like(n2))


class PainnUpdate(nn.Module):
    def __init__(self, node_size, last_layer=False, u_name="update_U"):
        super().__init__()
        self._u = u_name
        # U, V act on the vector state: bias-free (as in PaiNN) so the update stays equivariant
        # (the reference's biased Linears shift every Cartesian component alike)
        setattr(self, u_name, Linear(node_size, node_size, bias=False))
        self.update_V = Linear(node_size, node_size, bias=False)
        self.last_layer = last_layer
        out = 2 * node_size if last_layer else 3 * node_size
        self.update_mlp = nn.Sequential(Linear(2 * node_size, node_size), nn.SiLU(), Linear(node_size, out))

    def forward(self, s, v):
        F = s.shape[-1]
        Uv = getattr(self, self._u)(v)
        Vv = self.update_V(v)
        a = self.update_mlp(torch.cat((safe_vector_norm(Vv, 1), s), dim=-1))
        inner = (Uv * Vv).sum(1)
        if self.last_layer:
            a_sv, a_ss = a.split(F, 1)
            return s + a_sv * inner + a_ss, v
        a_vv, a_sv, a_ss = a.split(F, 1)
        return s + a_sv * inner + a_ss, v + a_vv.unsqueeze(1) * Uv


class _EqLayer(nn.Module):
    """message -> update -> node_embed_out (-> vec_embed_out)."""

    def __init__(self, message, update, node_embed_out, vec_embed_out):
        super().__init__()
        self.message = message
        self.update = update
        self.node_embed_out = node_embed_out
        self.vec_embed_out = vec_embed_out

    def forward(self, inv, equiv, ctx):
        s, v = self.message(inv, equiv, ctx)
        s, v = self.update(s, v)
        s = self.node_embed_out(s)
        if self.vec_embed_out is not None:
            v = self.vec_embed_out(v)
        return s, v


class _EqStackBase(Base):
    is_edge_model = True

    def _init_conv(self):
        n = self.num_conv_layers
        self.graph_convs.append(self._apply_global_attn(
            self.get_conv(self.embed_dim, self.hidden_dim, n == 1, edge_dim=self.edge_embed_dim)))
        self.feature_layers.append(nn.Identity())
        for i in range(n - 1):
            self.graph_convs.append(self._apply_global_attn(
                self.get_conv(self.hidden_dim, self.hidden_dim, i == n - 2, edge_dim=self.edge_embed_dim)))
            self.feature_layers.append(nn.Identity())

    def _conv_head_kwargs(self):
        return {"last_layer": False, **super()._conv_head_kwargs()}

    def _adapters(self, input_dim, output_dim, last_layer):
        node_embed_out = nn.Sequential(Linear(input_dim, output_dim), nn.Tanh(), Linear(output_dim, output_dim))
        # bias-free on purpose: the reference's Linear(input_dim, output_dim) adds the same bias
        # to all three Cartesian components of v, which breaks rotation equivariance
        vec_embed_out = Linear(input_dim, output_dim, bias=False) if not last_layer else None
        return node_embed_out, vec_embed_out

    def _geometry(self, data, ctx):
        assert data.pos is not None, f"{self} requires node positions (data.pos) to be set."
        vec, dist = edge_vectors_and_lengths(data.pos, ctx.dst_si, ctx.src_si, data.get("edge_shifts"),
                                             normalize=True)
        return vec, dist

    def _embedding(self, data):
        x, pos, ctx = super()._embedding(data)
        vec, dist = self._geometry(data, ctx)
        ctx.edge_diff, ctx.edge_dist = vec, dist
        self._extra_geometry(ctx, dist)
        v = torch.zeros(x.shape[0], 3, x.shape[1], device=x.device, dtype=x.dtype)
        return x, v, ctx

    def _extra_geometry(self, ctx, dist):
        pass


class PAINNStack(_EqStackBase):
    def __init__(self, input_args, conv_args, edge_dim, num_radial, radius, *args, **kwargs):
        self.edge_dim = edge_dim
        self.num_radial = num_radial
        self.radius = radius
        super().__init__(input_args, conv_args, *args, **kwargs)

    def _fused_encode(self, inv, equiv, ctx):
        """Native twice-differentiable encoder (ops/painn_force.py): geometry, message and
        per-layer node chains as closed op families with explicit first and second
        derivatives (force training without the composite op-by-op graph)."""
        from ..ops import painn_force

        if not painn_force.model_ok(self, ctx):
            return None
        if ctx.get("gps_lazy"):
            return None
        return painn_force.painn_encode(self, inv, ctx)

    def decode(self, x, equiv, ctx):
        # the native encoder fused a single node MLP head into its last node chain
        e = ctx.get("native_node_head")
        if e is not None:
            return [e]
        return super().decode(x, equiv, ctx)

    def get_conv(self, input_dim, output_dim, last_layer=False, edge_dim=None):
        hidden = output_dim if input_dim == 1 else input_dim
        assert hidden > 1, "PainnNet requires more than one hidden dimension between input_dim and output_dim."
        msg = PainnMessage(input_dim, self.num_radial, self.radius, edge_dim)
        upd = PainnUpdate(input_dim, last_layer=last_layer, u_name="update_U")
        return _EqLayer(msg, upd, *self._adapters(input_dim, output_dim, last_layer))

    def __str__(self):
        return "PAINNStack"


class PNAEqMessage(nn.Module):
    def __init__(self, node_size, deg, edge_dim, num_radial,
                 aggregators=("mean", "min", "max", "std"),
                 scalers=("identity", "amplification", "attenuation", "linear", "inverse_linear")):
        super().__init__()
        F = node_size
        self.node_size, self.edge_dim, self.num_radial = F, edge_dim, num_radial
        self.aggregators, self.scalers = tuple(aggregators), tuple(scalers)
        self.register_buffer("deg", torch.as_tensor(deg, dtype=torch.float32))
        self.avg_deg = pna_avg_deg(self.deg)
        self.pre_nns = nn.ModuleList([nn.Sequential(Linear((4 if edge_dim else 3) * F, F))])
        self.post_nns = nn.ModuleList([nn.Sequential(
            Linear((len(aggregators) * len(scalers) + 1) * F, F))])
        self.rbf_emb = nn.Sequential(Linear(num_radial, F), nn.Tanh())
        if edge_dim is not None:
            self.edge_encoder = Linear(edge_dim, F)
        self.rbf_lin = Linear(num_radial, 3 * F, bias=False)
        self.scalar_message_mlp = nn.Sequential(Linear(F, F), nn.Tanh(), Linear(F, F), nn.SiLU(),
                                                Linear(F, 3 * F))

    def _aggregate(self, m, si):
        if m.is_cuda:
            # one HIP pass each way for [mean, min, max, std] x 5 scalers (csrc/segment.hip
            # seg_pna_agg); composite fallback inside for double backward / other sets
            return pna_aggregate(m, si, self.avg_deg, self.aggregators, self.scalers)
        aggs = []
        for a in self.aggregators:
            if a == "mean":
                aggs.append(seg.segment_mean(m, si))
            elif a == "min":
                aggs.append(seg.segment_min(m, si))
            elif a == "max":
                aggs.append(seg.segment_max(m, si))
            elif a == "std":
                aggs.append(seg.segment_std(m, si))
            elif a == "sum":
                aggs.append(seg.segment_sum(m, si))
            else:
                raise ValueError(a)
        out = torch.cat(aggs, -1)
        deg = si.degree(out.dtype).to(out.device)
        return torch.cat([out * sc for sc in degree_scalers(deg, self.avg_deg, self.scalers)], -1)

    def forward(self, s, v, ctx):
        F = self.node_size
        pre = self.pre_nns[0][0]
        W = pre.weight
        # concat-linear decomposition: [s_src | s_dst] blocks at node level
        nb = torch.nn.functional.linear(s, torch.cat([W[:, :F], W[:, F:2 * F]], 0))
        m = seg.gather(nb[:, :F], ctx.src_si) + seg.gather(nb[:, F:], ctx.dst_si) + pre.bias
        m = m + torch.nn.functional.linear(self.rbf_emb(ctx.edge_rbf), W[:, 2 * F:3 * F])
        if ctx.edge_attr is not None and self.edge_dim:
            m = m + torch.nn.functional.linear(self.edge_encoder(ctx.edge_attr), W[:, 3 * F:])
        out = self.scalar_message_mlp(m) * self.rbf_lin(ctx.edge_rbf)
        g_v, g_e, m_s = out[:, :F], out[:, F:2 * F], out[:, 2 * F:]
        m_v = seg.gather(v, ctx.dst_si) * g_v.unsqueeze(1) + g_e.unsqueeze(1) * ctx.edge_diff.unsqueeze(-1)
        agg = self._aggregate(m_s, ctx.src_si)
        ds = self.post_nns[0](torch.cat([s, agg], -1))
        return s + ds, v + seg.segment_sum(m_v, ctx.src_si)


class PNAEqStack(_EqStackBase):
    def __init__(self, input_args, conv_args, deg, edge_dim, num_radial, radius, *args, **kwargs):
        self.x_aggregators = ["mean", "min", "max", "std"]
        self.x_scalers = ["identity", "amplification", "attenuation", "linear", "inverse_linear"]
        self.deg = torch.as_tensor(deg, dtype=torch.float32)
        self.edge_dim = edge_dim
        self.num_radial = num_radial
        self.radius = radius
        super().__init__(input_args, conv_args, *args, **kwargs)
        self.rbf = rbf_BasisLayer(self.num_radial, self.radius)

    def get_conv(self, input_dim, output_dim, last_layer=False, edge_dim=None):
        hidden = output_dim if input_dim == 1 else input_dim
        assert hidden > 1, "PNAEq requires more than one hidden dimension between input_dim and output_dim."
        msg = PNAEqMessage(input_dim, self.deg, edge_dim, self.num_radial, self.x_aggregators, self.x_scalers)
        upd = PainnUpdate(input_dim, last_layer=last_layer, u_name="update_X")
        return _EqLayer(msg, upd, *self._adapters(input_dim, output_dim, last_layer))

    def _extra_geometry(self, ctx, dist):
        ctx.edge_rbf = self.rbf(dist.view(-1))

    def __str__(self):
        return "PNAEqStack"
