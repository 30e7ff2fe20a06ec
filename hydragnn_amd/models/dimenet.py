"""DimeNet++ stack (reference ``hydragnn/models/DIMEStack.py:34-305``; PyG
``InteractionPPBlock`` / ``OutputPPBlock`` / ``SphericalBasisLayer`` semantics).

Per layer:  x <- lin(x);  m_ji = act(lin(cat[x_i, x_j, act(lin_rbf rbf_ji)(, act(edge_lin e))]))
            (HydraEmbeddingBlock, i = destination, j = source)
            m_ji <- InteractionPP(m, rbf, sbf, triplets)
            x_i  <- OutputPP: lin(act(lins(lin_up(sum_{j} lin_rbf(rbf_ji) * m_ji))))

Triplets (k -> j -> i, k != i) come straight from the destination CSR: the
in-edges of j are one contiguous segment, so for edge e_ji the candidates k->j
are ``rowptr[j]..rowptr[j+1]`` — no sparse-tensor indexing.  Triplets are emitted
grouped by e_ji, so the k->j => j->i message reduction is a sorted (atomic-free)
segment sum.  The spherical basis uses spherical Bessel functions j_l(z_ln r)
(zeros from scipy, evaluated in float64 by upward recurrence) times zonal
harmonics Y_l^0(angle) = sqrt((2l+1)/4pi) P_l(cos angle), enveloped as in PyG.
"""
import math
import os

import numpy as np
import torch
from torch import nn

from ..ops import segment as seg
from ..ops.geometry import BesselBasis, Envelope, edge_vectors_and_lengths
from ..ops.linear import linear_cols
from .layers import Linear
from .base import Base


# ----------------------------------------------------------------------------- bases
def _sph_jn_np(l, x):
    from scipy.special import spherical_jn

    return spherical_jn(l, x)


def bessel_zeros(n, k):
    """First k positive zeros of j_l for l < n (n x k array)."""
    from scipy.optimize import brentq

    zeros = np.zeros((n, k))
    zeros[0] = np.arange(1, k + 1) * np.pi
    pts = np.arange(1, k + n) * np.pi
    racines = np.zeros(k + n - 1)
    for l in range(1, n):
        for j in range(k + n - 1 - l):
            racines[j] = brentq(lambda x: _sph_jn_np(l, x), pts[j], pts[j + 1])
        pts = racines.copy()
        zeros[l][:k] = racines[:k]
    return zeros


def _sph_jn_torch(lmax, x):
    """[j_0(x) .. j_lmax(x)] by upward recurrence (float64 for stability)."""
    x = x.to(torch.float64)
    s, c = torch.sin(x), torch.cos(x)
    out = [s / x]
    if lmax >= 1:
        out.append(s / (x * x) - c / x)
    for l in range(1, lmax):
        out.append((2 * l + 1) / x * out[l] - out[l - 1])
    return out


def _legendre(lmax, t):
    p = [torch.ones_like(t)]
    if lmax >= 1:
        p.append(t)
    for l in range(1, lmax):
        p.append(((2 * l + 1) * t * p[l] - l * p[l - 1]) / (l + 1))
    return p


class _TripletSBF(torch.autograd.Function):
    """Triplet angle + spherical basis in one HIP pass each way (csrc/dimenet.hip):
    sbf[t] from vec[e_ji], vec[e_kj]; backward returns d vec (analytic)."""

    @staticmethod
    def forward(ctx, vec, kj, ji, layer, limit=None):
        from .. import _native

        ctx.save_for_backward(vec, kj, ji)
        ctx.layer, ctx.limit = layer, limit
        return _native.ops().dimenet_sbf_fwd(vec, kj, ji, layer.zeros, layer.norm, layer.cutoff, layer.exponent, limit)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        vec, kj, ji = ctx.saved_tensors
        L = ctx.layer
        dvec = _native.ops().dimenet_sbf_bwd(g.contiguous(), vec, kj, ji, L.zeros, L.norm, L.cutoff, L.exponent,
                                             ctx.limit)
        return dvec, None, None, None, None


class SphericalBasisLayer(nn.Module):
    def __init__(self, num_spherical, num_radial, cutoff=5.0, envelope_exponent=5):
        super().__init__()
        assert num_radial <= 64
        self.num_spherical, self.num_radial = num_spherical, num_radial
        self.cutoff = float(cutoff)
        self.exponent = int(envelope_exponent)
        self.envelope = Envelope(envelope_exponent)
        z = bessel_zeros(num_spherical, num_radial)
        norm = np.zeros_like(z)
        for l in range(num_spherical):
            norm[l] = 1.0 / np.sqrt(0.5 * _sph_jn_np(l + 1, z[l]) ** 2)
        self.register_buffer("zeros", torch.tensor(z, dtype=torch.float64), persistent=False)
        self.register_buffer("norm", torch.tensor(norm, dtype=torch.float64), persistent=False)

    def forward(self, dist, angle, idx_kj):
        n, k = self.num_spherical, self.num_radial
        d = (dist / self.cutoff).to(torch.float64)
        rbf = []
        for l in range(n):
            x = d.view(-1, 1) * self.zeros[l].view(1, -1)  # [E, k]
            rbf.append(self.norm[l].view(1, -1) * _sph_jn_torch(l, x)[l])
        rbf = torch.stack(rbf, 1).to(dist.dtype)  # [E, n, k]
        rbf = self.envelope(dist / self.cutoff).view(-1, 1, 1) * rbf
        t = torch.cos(angle.to(torch.float64))
        P = _legendre(n - 1, t)
        cbf = torch.stack([math.sqrt((2 * l + 1) / (4 * math.pi)) * P[l] for l in range(n)], 1).to(dist.dtype)
        return (seg.gather(rbf.reshape(-1, n * k), idx_kj).view(-1, n, k) * cbf.view(-1, n, 1)).reshape(-1, n * k)

    def native_ok(self, vec):
        from ..ops.pna import fused

        return vec.is_cuda and vec.dtype == torch.float32 and fused("sbf") and self.num_spherical <= 8 and \
            self.num_radial <= 8

    def from_vectors(self, vec, kj_si, ji_si):
        """sbf directly from edge vectors (the GPU path: angle + basis in one kernel).  A
        static triplet list (``triplets_static``) carries its real count as the indices'
        ``limit``: the basis rows of the padding triplets are zero."""
        return _TripletSBF.apply(vec.contiguous(), kj_si.index, ji_si.index, self, ji_si.limit)


# ----------------------------------------------------------------------------- triplets
def triplets_csr(dst_si, src_si, num_nodes):
    """(idx_kj, idx_ji) for all k->j->i with k != i, grouped by e_ji (ascending)."""
    dev = dst_si.rowptr.device
    if dst_si.rowptr.is_cuda:  # HIP count/scan/fill builder (csrc/graph.hip), same order as below
        from .. import _native

        ei = torch.stack([src_si.index.long(), dst_si.index.long()], 0)
        return _native.ops().triplets(ei, dst_si.rowptr.to(torch.int32))
    src = src_si.index.long()
    dst = dst_si.index.long()
    rowptr = dst_si.rowptr.long()
    E = src.numel()
    deg_j = rowptr[src + 1] - rowptr[src]  # in-degree of j for every edge j->i
    e_ji = torch.repeat_interleave(torch.arange(E, device=dev), deg_j)
    start = torch.repeat_interleave(rowptr[src], deg_j)
    off = torch.arange(e_ji.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(deg_j, 0) - deg_j, deg_j)
    e_kj = start + off
    keep = src[e_kj] != dst[e_ji]  # k != i
    return e_kj[keep], e_ji[keep]


def _note_overflow(total, Tcap):
    """Record a device triplet count above the static capacity (the fill kernels clamp to
    ``Tcap``, so such a batch would train on a truncated triplet set): folded into a
    persistent device flag (``ops/devcheck.py``) that the epoch loop turns into an error."""
    from ..ops import devcheck

    f = devcheck.flag(total.device, "triplet_cap")
    torch.maximum(f, total.sub(Tcap), out=f)
    devcheck.debug_check("triplet_cap", total.device)


def check_triplet_overflow():
    from ..ops import devcheck

    devcheck.check_all()


def triplets_static(dst_si, src_si, node_mask, Tcap):
    """Triplets of a statically padded batch with FIXED capacity ``Tcap`` and no host
    synchronisation (capturable; csrc/graph.hip ``triplets_static_*``).  Only edges into
    valid nodes emit triplets (padding edges join padding nodes), in the order of
    ``triplets_csr``; slots [T, Tcap) are dummy triplets of the last edge, sorted last in
    both views.  Returns (kj_si, ji_si) whose ``limit`` (device int32 scalar) is T: segment
    sums stop there and the basis kernels zero the padding rows."""
    src, dst, rowptr = src_si.index, dst_si.index, dst_si.rowptr
    E = src.numel()
    mask = None if node_mask is None else node_mask.view(-1).bool()
    if src.is_cuda:
        from .. import _native

        counts = _native.ops().triplets_static_count(src, dst, rowptr, mask)
        tptr = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0, dtype=torch.int32)])
        kj, ji = _native.ops().triplets_static_fill(src, dst, rowptr, mask, tptr, int(Tcap))
        kview = None
        if src_si.perm is not None and os.environ.get("HYDRA_TRIPLET_KJ_SORT", "0") != "1":
            # kj CSR view without a sort (csrc/graph.hip triplets_static_kj)
            kview = _native.ops().triplets_static_kj(src, dst, rowptr, src_si.rowptr, src_si.perm, mask, tptr,
                                                     int(Tcap))
    else:  # CPU twin (padded_step tests): the eager order, then the dummy tail
        kview = None
        kj_v, ji_v = triplets_csr(dst_si, src_si, rowptr.numel() - 1)
        if mask is not None:
            keep = mask[dst.long()[ji_v]]
            kj_v, ji_v = kj_v[keep], ji_v[keep]
        T = kj_v.numel()
        if T > Tcap:
            raise RuntimeError(f"triplets_static: {T} triplets exceed the capacity {Tcap}")
        kj = torch.full((Tcap,), E - 1, dtype=torch.int32)
        ji = torch.full((Tcap,), E - 1, dtype=torch.int32)
        kj[:T], ji[:T] = kj_v.int(), ji_v.int()
        tptr = torch.zeros(E + 1, dtype=torch.int32)
        tptr[1:] = torch.cumsum(torch.bincount(ji_v.long(), minlength=E), 0).int()
    if src.is_cuda:
        _note_overflow(tptr[E:E + 1], int(Tcap))
    limit = tptr[E:E + 1].clamp(max=int(Tcap))
    jrp = tptr.clamp(max=int(Tcap))
    jrp[E:].fill_(int(Tcap))  # the dummy tail belongs to the last edge
    if kview is not None:
        krp, perm = kview
    else:
        vals, perm = torch.sort(kj, stable=True)
        krp = torch.searchsorted(vals, torch.arange(E + 1, dtype=torch.int32, device=kj.device), out_int32=True)
    return (seg.SegIndex(kj, krp, perm.to(torch.int32), E, limit), seg.SegIndex(ji, jrp, None, E, limit))


# ----------------------------------------------------------------------------- blocks
def _glorot_orthogonal(w, scale=2.0):
    nn.init.orthogonal_(w)
    s = scale / ((w.size(0) + w.size(1)) * w.var())
    w.data *= s.sqrt()


class _ResMLP(torch.autograd.Function):
    """y = x + silu(lin2(silu(lin1(x)))) in one HIP launch each way (csrc/resmlp.hip); the
    backward kernel emits the weight gradients' row factors, which join the deferred grouped
    weight-gradient launch (ops/linear.py) when it is open."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        from .. import _native

        y, H1, H2 = _native.ops().res_mlp_fwd(x, W1, b1, W2, b2)
        ctx.save_for_backward(x, H1, H2, W1, W2)
        ctx.params = (W1, b1, W2, b2)
        return y

    @staticmethod
    def backward(ctx, g):
        from .. import _native
        from ..ops import linear as _lin

        x, H1, H2, W1, W2 = ctx.saved_tensors
        dx, dH2, A1, dH1 = _native.ops().res_mlp_bwd(g, H1, H2, W1, W2)
        W1p, b1p, W2p, b2p = ctx.params
        if _lin._can_defer(W1p, b1p) and _lin._can_defer(W2p, b2p):
            _lin._record((dH2, A1, W2p, b2p))
            _lin._record((dH1, x, W1p, b1p))
            return dx, None, None, None, None
        dW1, db1 = torch.empty_like(W1p), torch.empty_like(b1p)
        dW2, db2 = torch.empty_like(W2p), torch.empty_like(b2p)
        _native.ops().linear_wgrad_grouped([dH2, dH1], [A1, x], [dW2, dW1], [db2, db1], [0, 0])
        return dx, dW1, db1, dW2, db2


class _SiluLinear(torch.autograd.Function):
    """y = silu(x W^T + b) * mul + add in one HIP launch each way (csrc/resmlp.hip lin_act);
    the weight gradient's row factors join the deferred grouped weight-gradient launch."""

    @staticmethod
    def forward(ctx, x, W, b, mul, add):
        from .. import _native

        y, Z = _native.ops().lin_act_fwd(x, W, b, mul, add)
        ctx.save_for_backward(x, Z, W, mul)
        ctx.params = (W, b)
        ctx.has_add = add is not None
        return y

    @staticmethod
    def backward(ctx, g):
        from .. import _native
        from ..ops import linear as _lin

        x, Z, W, mul = ctx.saved_tensors
        want_dmul = mul is not None and ctx.needs_input_grad[3]
        dx, dZ, dmul = _native.ops().lin_act_bwd(g, Z, W, mul, want_dmul)
        Wp, bp = ctx.params
        dadd = g if (ctx.has_add and ctx.needs_input_grad[4]) else None
        dmul = dmul if want_dmul else None
        if _lin._can_defer(Wp, bp):
            _lin._record((dZ, x, Wp, bp))
            return dx, None, None, dmul, dadd
        dW = torch.empty_like(Wp)
        db = torch.empty_like(bp) if bp is not None else torch.empty(0, device=g.device, dtype=g.dtype)
        _native.ops().linear_wgrad_grouped([dZ], [x], [dW], [db], [0])
        return dx, dW, (db if bp is not None else None), dmul, dadd


def silu_lin(lin, act, x, mul=None, add=None):
    """``act(lin(x)) * mul + add`` (mul / add optional): one fused HIP launch each way for
    SiLU on GPU fp32 edge-sized rows (widths <= 64), the module chain otherwise."""
    from ..ops.pna import fused

    W = lin.weight
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[0] >= 1024 and x.shape[1] <= 64 and
            W.shape[0] <= 64 and isinstance(act, nn.SiLU) and fused("resmlp") and torch.is_grad_enabled() and
            (mul is None or mul.shape == (x.shape[0], W.shape[0])) and
            (add is None or add.shape == (x.shape[0], W.shape[0]))):
        return _SiluLinear.apply(x.contiguous(), W, lin.bias, None if mul is None else mul.contiguous(),
                                 None if add is None else add.contiguous())
    y = act(lin(x))
    if mul is not None:
        y = y * mul
    if add is not None:
        y = y + add
    return y


class ResidualLayer(nn.Module):
    def __init__(self, hidden, act):
        super().__init__()
        self.act = act
        self.lin1 = Linear(hidden, hidden)
        self.lin2 = Linear(hidden, hidden)
        for l in (self.lin1, self.lin2):
            _glorot_orthogonal(l.weight)
            l.bias.data.fill_(0)

    def forward(self, x):
        from ..ops.pna import fused

        if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] <= 64 and x.shape[0] >= 1024
                and isinstance(self.act, nn.SiLU) and fused("resmlp") and torch.is_grad_enabled()):
            return _ResMLP.apply(x.contiguous(), self.lin1.weight, self.lin1.bias, self.lin2.weight, self.lin2.bias)
        return x + self.act(self.lin2(self.act(self.lin1(x))))


class HydraEmbeddingBlock(nn.Module):
    def __init__(self, num_radial, hidden_channels, act, edge_dim=None):
        super().__init__()
        self.act = act
        self.lin_rbf = Linear(num_radial, hidden_channels)
        if edge_dim is not None:
            self.edge_lin = Linear(edge_dim, hidden_channels)
            self.lin = Linear(4 * hidden_channels, hidden_channels)
        else:
            self.lin = Linear(3 * hidden_channels, hidden_channels)

    def forward(self, x, rbf, dst_si, src_si, edge_attr=None):
        H = x.shape[1]
        W = self.lin.weight
        # concat-linear split: the node blocks [x_i | x_j] at node level, then gathered; every
        # column block's weight gradient joins the deferred grouped launch (ops.linear.linear_cols)
        h = seg.gather(linear_cols(x, W, 0), dst_si) + seg.gather(linear_cols(x, W, H), src_si) + self.lin.bias
        h = h + linear_cols(self.act(self.lin_rbf(rbf)), W, 2 * H)
        if edge_attr is not None and hasattr(self, "edge_lin"):
            h = h + linear_cols(self.act(self.edge_lin(edge_attr)), W, 3 * H)
        return self.act(h)


class _LowRankGMS(torch.autograd.Function):
    """``gather_mul_sum(x_kj, s8 @ W2^T, kj_si, ji_si)`` without the [T, I] triplet filter
    (csrc/dimenet.hip lr_gather_mul_sum / lr_filter_grad): the filter is recomputed per
    column from the 8-wide basis row.  First order (composite mode keeps the torch chain)."""

    @staticmethod
    def forward(ctx, x, s8, W2, gsi, ssi):
        from .. import _native

        ctx.save_for_backward(x, s8, W2)
        ctx.gsi, ctx.ssi = gsi, ssi
        return _native.ops().lr_gather_mul_sum(x.contiguous(), s8.contiguous(), W2, gsi.index, ssi.rowptr,
                                               ssi.perm, ssi.num_segments, ssi.limit)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        x, s8, W2 = ctx.saved_tensors
        gsi, ssi = ctx.gsi, ctx.ssi
        ops = _native.ops()
        g = g.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            # dx[k] = sum_{t: kj(t) = k} g[ji(t)] * w[t]: the same kernel over the kj CSR
            dx = ops.lr_gather_mul_sum(g, s8, W2, ssi.index, gsi.rowptr, gsi.perm, x.shape[0], gsi.limit)
        ds8 = dW2 = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            ds8, dW2 = ops.lr_filter_grad(x, gsi.index, g, ssi.index, s8, W2, ssi.limit)
        return dx, ds8, dW2, None, None


def _lowrank_ok(x, s8, W2):
    from ..ops.pna import fused

    return (x.is_cuda and x.dtype == torch.float32 and s8.dtype == torch.float32 and x.dim() == 2
            and x.shape[1] % 4 == 0 and x.shape[1] <= 64 and s8.shape[1] == 8 and fused("dimenet_lr")
            and _LOWRANK)


# HYDRA_DIMENET_LOWRANK=0: materialise the [T, I] filter (lin_sbf2) and use gather_mul_sum
_LOWRANK = os.environ.get("HYDRA_DIMENET_LOWRANK", "1") == "1"


class InteractionPPBlock(nn.Module):
    def __init__(self, hidden_channels, int_emb_size, basis_emb_size, num_spherical, num_radial, num_before_skip,
                 num_after_skip, act):
        super().__init__()
        self.act = act
        self.lin_rbf1 = Linear(num_radial, basis_emb_size, bias=False)
        self.lin_rbf2 = Linear(basis_emb_size, hidden_channels, bias=False)
        self.lin_sbf1 = Linear(num_spherical * num_radial, basis_emb_size, bias=False)
        self.lin_sbf2 = Linear(basis_emb_size, int_emb_size, bias=False)
        self.lin_kj = Linear(hidden_channels, hidden_channels)
        self.lin_ji = Linear(hidden_channels, hidden_channels)
        self.lin_down = Linear(hidden_channels, int_emb_size, bias=False)
        self.lin_up = Linear(int_emb_size, hidden_channels, bias=False)
        self.layers_before_skip = nn.ModuleList([ResidualLayer(hidden_channels, act) for _ in range(num_before_skip)])
        self.lin = Linear(hidden_channels, hidden_channels)
        self.layers_after_skip = nn.ModuleList([ResidualLayer(hidden_channels, act) for _ in range(num_after_skip)])
        for l in (self.lin_rbf1, self.lin_rbf2, self.lin_sbf1, self.lin_sbf2, self.lin_kj, self.lin_ji,
                  self.lin_down, self.lin_up, self.lin):
            _glorot_orthogonal(l.weight)
            if l.bias is not None:
                l.bias.data.fill_(0)

    def forward(self, x, rbf, sbf, kj_si, ji_si):
        # every act(lin(.)) (* / +) step is one fused launch each way (silu_lin)
        x_ji = silu_lin(self.lin_ji, self.act, x)
        x_kj = silu_lin(self.lin_kj, self.act, x, mul=self.lin_rbf2(self.lin_rbf1(rbf)))
        x_kj = silu_lin(self.lin_down, self.act, x_kj)
        s8 = self.lin_sbf1(sbf)
        if _lowrank_ok(x_kj, s8, self.lin_sbf2.weight):
            # the [T, I] filter s8 W2^T is recomputed per column inside the pass (never stored)
            x_kj = _LowRankGMS.apply(x_kj, s8, self.lin_sbf2.weight, kj_si, ji_si)
        else:
            x_kj = seg.gather_mul_sum(x_kj, self.lin_sbf2(s8), kj_si, ji_si)  # gather * sbf -> sum
        h = silu_lin(self.lin_up, self.act, x_kj, add=x_ji)
        for layer in self.layers_before_skip:
            h = layer(h)
        h = silu_lin(self.lin, self.act, h, add=x)
        for layer in self.layers_after_skip:
            h = layer(h)
        return h


class OutputPPBlock(nn.Module):
    def __init__(self, num_radial, hidden_channels, out_emb_channels, out_channels, num_layers, act):
        super().__init__()
        self.act = act
        self.lin_rbf = Linear(num_radial, hidden_channels, bias=False)
        self.lin_up = Linear(hidden_channels, out_emb_channels, bias=False)
        self.lins = nn.ModuleList([Linear(out_emb_channels, out_emb_channels) for _ in range(num_layers)])
        self.lin = Linear(out_emb_channels, out_channels, bias=False)
        _glorot_orthogonal(self.lin_rbf.weight)
        _glorot_orthogonal(self.lin_up.weight)
        for l in self.lins:
            _glorot_orthogonal(l.weight)
            l.bias.data.fill_(0)
        _glorot_orthogonal(self.lin.weight)

    def forward(self, m, rbf, dst_si):
        x = seg.segment_sum(self.lin_rbf(rbf) * m, dst_si)
        x = self.lin_up(x)
        for l in self.lins:
            x = self.act(l(x))
        return self.lin(x)


class DimeNetLayer(nn.Module):
    def __init__(self, lin, emb, inter, dec):
        super().__init__()
        self.lin, self.emb, self.inter, self.dec = lin, emb, inter, dec

    def forward(self, inv, equiv, ctx):
        x = self.lin(inv)
        m = self.emb(x, ctx.rbf, ctx.dst_si, ctx.src_si, ctx.edge_attr)
        m = self.inter(m, ctx.rbf, ctx.sbf, ctx.kj_si, ctx.ji_si)
        return self.dec(m, ctx.rbf, ctx.dst_si), equiv


class DIMEStack(Base):
    is_edge_model = True
    # a statically padded batch carries the store's triplet capacity: the triplets are then
    # built on the device with fixed shapes (triplets_static), so the step is capturable
    capturable = True

    def __init__(self, input_args, conv_args, basis_emb_size, envelope_exponent, int_emb_size, out_emb_size,
                 num_after_skip, num_before_skip, num_radial, num_spherical, edge_dim, radius, *args,
                 max_neighbours=None, **kwargs):
        self.basis_emb_size = basis_emb_size
        self.int_emb_size = int_emb_size
        self.out_emb_size = out_emb_size
        self.num_radial = num_radial
        self.num_spherical = num_spherical
        self.num_before_skip = num_before_skip
        self.num_after_skip = num_after_skip
        self.edge_dim = edge_dim
        self.radius = radius
        super().__init__(input_args, conv_args, *args, **kwargs)
        self.rbf = BesselBasis(num_radial, radius, envelope_exponent)
        self.sbf = SphericalBasisLayer(num_spherical, num_radial, radius, envelope_exponent)

    def _init_conv(self):
        self.graph_convs.append(self._apply_global_attn(
            self.get_conv(self.embed_dim, self.hidden_dim, edge_dim=self.edge_embed_dim)))
        self.feature_layers.append(nn.Identity())
        for _ in range(self.num_conv_layers - 1):
            self.graph_convs.append(self._apply_global_attn(
                self.get_conv(self.hidden_dim, self.hidden_dim, edge_dim=self.edge_embed_dim)))
            self.feature_layers.append(nn.Identity())

    def get_conv(self, input_dim, output_dim, edge_dim=None):
        hidden = output_dim if input_dim == 1 else input_dim
        assert hidden > 1, "DimeNet requires more than one hidden dimension between input_dim and output_dim."
        act = nn.SiLU()
        lin = Linear(input_dim, hidden)
        emb = HydraEmbeddingBlock(self.num_radial, hidden, act, edge_dim=edge_dim)
        inter = InteractionPPBlock(hidden, self.int_emb_size, self.basis_emb_size, self.num_spherical,
                                   self.num_radial, self.num_before_skip, self.num_after_skip, act)
        dec = OutputPPBlock(self.num_radial, hidden, self.out_emb_size, output_dim, 1, act)
        return DimeNetLayer(lin, emb, inter, dec)

    def _embedding(self, data):
        x, pos, ctx = super()._embedding(data)
        assert data.pos is not None, "DimeNet requires node positions (data.pos) to be set."
        N = data.num_nodes
        E = ctx.dst_si.index.numel()
        tcap = data.get("triplet_cap")  # padded batch: the store's capacity (host int, lazy)
        tcap = tcap() if callable(tcap) else tcap
        if tcap is not None and E > 0:
            ctx.kj_si, ctx.ji_si = triplets_static(ctx.dst_si, ctx.src_si, data.get("node_mask"), tcap)
        else:
            idx_kj, idx_ji = triplets_csr(ctx.dst_si, ctx.src_si, N)
            ctx.kj_si = seg.SegIndex.from_index(idx_kj, E, sorted_=False)
            ctx.ji_si = seg.SegIndex.from_index(idx_ji, E, sorted_=True)
        vec, dist = edge_vectors_and_lengths(data.pos, ctx.dst_si, ctx.src_si, data.get("edge_shifts"))
        d = dist.view(-1)
        ctx.rbf = self.rbf(d)
        if self.sbf.native_ok(vec):
            ctx.sbf = self.sbf.from_vectors(vec, ctx.kj_si, ctx.ji_si)
            return x, pos, ctx
        pos_ji = seg.gather(vec, ctx.ji_si)
        pos_ki = seg.gather(vec, ctx.kj_si) + pos_ji
        a = (pos_ji * pos_ki).sum(-1)
        b = torch.linalg.cross(pos_ji, pos_ki).norm(dim=-1)
        angle = torch.atan2(b, a)
        ctx.sbf = self.sbf(d, angle, ctx.kj_si)
        if ctx.kj_si.limit is not None:  # padding triplets: zero basis rows
            live = torch.arange(ctx.sbf.shape[0], device=d.device) < ctx.kj_si.limit
            ctx.sbf = ctx.sbf * live.view(-1, 1).to(ctx.sbf.dtype)
        return x, pos, ctx

    def __str__(self):
        return "DIMEStack"
