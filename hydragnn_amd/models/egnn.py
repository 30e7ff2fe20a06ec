"""EGNN stack (reference ``hydragnn/models/EGCLStack.py:22-298``) — the SC25 GFM model.

E_GCL layer (reference ``EGCLStack.py:175-289``), edge_index = (row, col) = (source,
destination) in PyG order:

    m_e   = edge_mlp(cat[x_row, x_col, |d_e|, e_e])          d_e = pos[col] - pos[row]
    pos'  = pos + mean_{e: row(e)=n} clamp(d_e / (|d_e| + 1) * coord_mlp(m_e), +-100)
    x'    = node_mlp(cat[x, sum_{e: row(e)=n} m_e])

Note the reference aggregates onto ``row`` (the *source* index); this is kept (CSR
by source = ``src_si``, deterministic, atomic-free).

MI355X mapping: the first edge_mlp Linear over the concatenation is decomposed
column-wise — the x_row / x_col blocks run as ONE node-level GEMM [N, 2H] and are
gathered per edge, so the only edge-row GEMM is the H x H second layer.
Parameter names follow the reference (``edge_mlp.0``, ``node_mlp.2``,
``coord_mlp.2``) so state dicts interchange.
"""
import torch
from torch import nn

from .. import _native
from ..ops import segment as seg
from ..ops.geometry import edge_vectors_and_lengths
from ..ops.linear import ACT_RELU, linear
from ..ops.pna import fused
from .layers import Linear
from .base import Base


class _EdgeGatherAct(torch.autograd.Function):
    """act(A[src] + B[dst] + r w + b (+ e-term)) in one pass (csrc/conv_misc.hip): r [E, K]
    scalar edge features (the radial length, plus narrow edge attributes) with their weight
    rows w [K, H]; backward: one pass for dz / dr, CSR segment sums for dA / dB, one K-row
    GEMM for dw."""

    @staticmethod
    def forward(ctx, ab, r, w, b, et, src_si, dst_si, act):
        out = _native.ops().edge_gather_act_fwd(ab, src_si.index, dst_si.index, r, w, b, et, act)
        ctx.save_for_backward(ab, r, w, b, et)
        ctx.cfg = (src_si, dst_si, act)
        return out

    @staticmethod
    def backward(ctx, g):
        ab, r, w, b, et = ctx.saved_tensors
        src_si, dst_si, act = ctx.cfg
        dz, dr = _native.ops().edge_gather_act_bwd(g, ab, src_si.index, dst_si.index, r, w, b, et, act)
        dab = torch.cat([seg.segment_sum(dz, src_si), seg.segment_sum(dz, dst_si)], 1)
        K = w.numel() // dz.shape[1]
        dw = (r.view(-1, K).t() @ dz).view_as(w)  # [K, E] x [E, H] (the dz^T r form ran at 4 workgroups)
        return dab, dr.view_as(r), dw, dz.sum(0), (dz if et is not None else None), None, None, None


_ACT_CODE = {nn.ReLU: 1, nn.SiLU: 2}


def split_concat_linear(lin, widths):
    """Column blocks of ``lin.weight`` for an input that is a concatenation of ``widths``."""
    out, o = [], 0
    for w in widths:
        out.append(lin.weight[:, o:o + w])
        o += w
    return out


class E_GCL(nn.Module):
    def __init__(self, input_channels, output_channels, hidden_channels, edge_attr_dim=0, nodes_attr_dim=0,
                 act_fn=None, recurrent=False, coords_weight=1.0, attention=False, clamp=False, norm_diff=True,
                 tanh=True, equivariant=False):
        super().__init__()
        act_fn = act_fn if act_fn is not None else nn.ReLU()
        self.input_channels = input_channels
        self.coords_weight = coords_weight
        self.recurrent = recurrent
        self.attention = attention
        self.norm_diff = norm_diff
        self.tanh = tanh
        self.equivariant = equivariant
        self.edge_attr_dim = edge_attr_dim or 0
        self.edge_mlp = nn.Sequential(
            Linear(2 * input_channels + 1 + self.edge_attr_dim, hidden_channels), act_fn,
            Linear(hidden_channels, hidden_channels), act_fn)
        self.node_mlp = nn.Sequential(
            Linear(hidden_channels + input_channels + nodes_attr_dim, hidden_channels), act_fn,
            Linear(hidden_channels, output_channels))
        self.clamp = clamp
        if equivariant:
            layer = Linear(hidden_channels, 1, bias=False)
            nn.init.xavier_uniform_(layer.weight, gain=0.001)
            mods = [Linear(hidden_channels, hidden_channels), act_fn, layer]
            if tanh:
                mods.append(nn.Tanh())
            self.coord_mlp = nn.Sequential(*mods)
        if attention:
            self.att_mlp = nn.Sequential(Linear(hidden_channels, 1), nn.Sigmoid())
        self.act_fn = act_fn

    def edge_model(self, x, radial, edge_attr, dst_si, src_si):
        F = x.shape[1]
        l0 = self.edge_mlp[0]
        ws = [F, F, 1] + ([self.edge_attr_dim] if edge_attr is not None and self.edge_attr_dim else [])
        Wb = split_concat_linear(l0, ws)
        # [x_row | x_col] blocks at node level (one GEMM), gathered per edge
        ab = linear(x, torch.cat([Wb[0], Wb[1]], 0))
        act_code = _ACT_CODE.get(type(self.edge_mlp[1]))
        if x.is_cuda and x.dtype == torch.float32 and fused("egnn") and act_code is not None:
            r, w, et = radial.reshape(-1, 1), Wb[2].t(), None
            if len(ws) == 4 and ws[3] <= 3:
                # narrow edge attributes join the radial column inside the pass (no [E, H] term)
                r, w = torch.cat([r, edge_attr.reshape(-1, ws[3])], 1), torch.cat([w, Wb[3].t()], 0)
            elif len(ws) == 4:
                et = linear(edge_attr, Wb[3]).contiguous()
            h = _EdgeGatherAct.apply(ab.contiguous(), r.contiguous(), w.contiguous(), l0.bias, et, src_si, dst_si,
                                     act_code)
        else:
            h = seg.gather(ab[:, :l0.out_features], src_si) + seg.gather(ab[:, l0.out_features:], dst_si)
            h = h + radial * Wb[2].view(1, -1) + l0.bias
            if len(ws) == 4:
                h = h + linear(edge_attr, Wb[3])
            h = self.edge_mlp[1](h)
        l2, a2 = self.edge_mlp[2], self.edge_mlp[3]
        if isinstance(a2, nn.ReLU) and l2.bias is not None:
            out = linear(h, l2.weight, l2.bias, act=ACT_RELU)  # ReLU in the GEMM epilogue (tall maps)
        else:
            out = a2(l2(h))
        if self.attention:
            out = out * self.att_mlp(out)
        return out

    def node_model(self, x, m, src_si):
        agg = seg.segment_sum(m, src_si)
        out = self.node_mlp(torch.cat([x, agg], 1))
        if self.recurrent:
            out = x + out
        return out

    def coord_model(self, pos, coord_diff, m, src_si):
        c0, a0 = self.coord_mlp[0], self.coord_mlp[1]
        if isinstance(a0, nn.ReLU) and c0.bias is not None:
            phi = self.coord_mlp[2:](linear(m, c0.weight, c0.bias, act=ACT_RELU))  # ReLU in the epilogue
        else:
            phi = self.coord_mlp(m)
        trans = (coord_diff * phi).clamp(-100.0, 100.0)
        return pos + seg.segment_mean(trans, src_si) * self.coords_weight

    def forward(self, inv, equiv, ctx):
        pos = equiv
        coord_diff, radial = edge_vectors_and_lengths(pos, ctx.dst_si, ctx.src_si, None, normalize=self.norm_diff,
                                                      eps=1.0)
        m = self.edge_model(inv, radial, ctx.edge_attr, ctx.dst_si, ctx.src_si)
        if self.equivariant:
            pos = self.coord_model(pos, coord_diff, m, ctx.src_si)
        x = self.node_model(inv, m, ctx.src_si)
        return x, pos

    def __repr__(self):
        return f"E_GCL({self.input_channels}, equivariant={self.equivariant})"


class EGCLStack(Base):
    is_edge_model = True

    def __init__(self, input_args, conv_args, edge_attr_dim, *args, max_neighbours=None, **kwargs):
        self.edge_dim = 0 if edge_attr_dim is None else edge_attr_dim
        super().__init__(input_args, conv_args, *args, **kwargs)

    def _init_conv(self):
        n = self.num_conv_layers
        self.graph_convs.append(self._apply_global_attn(
            self.get_conv(self.embed_dim, self.hidden_dim, n == 1, edge_dim=self.edge_embed_dim)))
        self.feature_layers.append(nn.Identity())
        for i in range(n - 1):
            self.graph_convs.append(self._apply_global_attn(
                self.get_conv(self.hidden_dim, self.hidden_dim, i == n - 2, edge_dim=self.edge_embed_dim)))
            self.feature_layers.append(nn.Identity())

    def get_conv(self, input_dim, output_dim, last_layer=False, edge_dim=None):
        if not edge_dim:
            edge_dim = self.edge_dim
        return E_GCL(input_dim, output_dim, self.hidden_dim, edge_attr_dim=edge_dim,
                     equivariant=self.equivariance and not last_layer)

    def _conv_head_kwargs(self):
        return {"last_layer": False, "edge_dim": self.edge_embed_dim}

    def _fused_encode(self, inv, equiv, ctx):
        # bf16 precision on the GPU: the whole wide E_GCL stack on the MFMA engine
        # (ops/egnn_wide.py over csrc/bgemm.hip + csrc/egnn.hip)
        from ..ops import egnn_wide

        if self.training is not None and egnn_wide.eligible(self, ctx):
            x, pos = egnn_wide.encode(self, ctx)
            keep = ctx.data.get("node_mask")
            if keep is not None:
                x = x * keep.view(-1, 1).to(x.dtype)
            return x, pos, ctx
        return None

    def _embedding(self, data):
        x, pos, ctx = super()._embedding(data)
        if not self.use_global_attn and not self.edge_dim:
            ctx.edge_attr = None
        return x, pos, ctx

    def __str__(self):
        return "EGCLStack"
