"""MACE stack (reference ``hydragnn/models/MACEStack.py:75-546`` and
``hydragnn/utils/model/mace_utils/modules/blocks.py``) on the in-house O(3) toolkit
(``ops/o3.py``; e3nn is not available, basis/sign parity with e3nn is unpinned,
equivariance is tested directly).

Per layer (``RealAgnosticAttResidualInteractionBlock`` + ``EquivariantProductBasisBlock``):

    sc   = skip_linear(h)
    m_i  = linear( sum_{j->i} TP_uvu(linear_up(h)_j, [e_ij ⊕] Y(r̂_ij); FCN([R(r_ij), down(h)_j, down(h)_i])) ) / avg_neighbours
    h'   = linear(SymmetricContraction_{correlation}(m_i; element_i)) + sc
    h'   = sizing(h')   -> split into scalars (inv) and l > 0 blocks (equiv)

and a read-out after the embedding and after every layer whose predictions are
*summed* (linear read-outs, a non-linear one after the last layer).  Messages are
reduced with the CSR segment sum over destinations (deterministic, HIP on GPU).
"""
import math
import os
import warnings

import torch
from torch import nn
from torch.nn import ModuleDict, ModuleList, Sequential

from .. import _native
from ..ops import o3
from ..ops import branch_mlp as _bmlp
from ..ops import segment as seg
from ..ops.pna import fused
from ..ops.geometry import edge_vectors_and_lengths
from .base import Base
from .layers import Linear

NUM_ELEMENTS = 118


# ----------------------------------------------------------------------------- radial
class MACEBesselBasis(nn.Module):
    """sqrt(2/r_max) sin(n pi r / r_max) / r (reference ``radial.py:23-63``)."""

    def __init__(self, r_max, num_basis=8, trainable=False):
        super().__init__()
        w = math.pi / r_max * torch.linspace(1.0, num_basis, num_basis)
        if trainable:
            self.bessel_weights = nn.Parameter(w)
        else:
            self.register_buffer("bessel_weights", w)
        self.prefactor = math.sqrt(2.0 / r_max)

    def forward(self, x):
        return self.prefactor * torch.sin(self.bessel_weights * x) / x


class GaussianBasis(nn.Module):
    def __init__(self, r_max, num_basis=128, trainable=False):
        super().__init__()
        gw = torch.linspace(0.0, r_max, num_basis)
        if trainable:
            self.gaussian_weights = nn.Parameter(gw)
        else:
            self.register_buffer("gaussian_weights", gw)
        self.coeff = -0.5 / (r_max / (num_basis - 1)) ** 2

    def forward(self, x):
        return torch.exp(self.coeff * (x - self.gaussian_weights) ** 2)


class ChebychevBasis(nn.Module):
    def __init__(self, r_max, num_basis=8):
        super().__init__()
        self.r_max, self.num_basis = r_max, num_basis
        self.register_buffer("n", torch.arange(1, num_basis + 1).float())

    def forward(self, x):
        t = x.expand(-1, self.num_basis)
        return torch.special.chebyshev_polynomial_t(t, self.n)


class PolynomialCutoff(nn.Module):
    def __init__(self, r_max, p=6):
        super().__init__()
        self.r_max, self.p = float(r_max), float(p)

    def forward(self, x):
        p, u = self.p, x / self.r_max
        env = (1.0 - (p + 1.0) * (p + 2.0) / 2.0 * u ** p + p * (p + 2.0) * u ** (p + 1)
               - p * (p + 1.0) / 2.0 * u ** (p + 2))
        return env * (x < self.r_max)


class _MaceRadial(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, w, rc, p):
        ctx.save_for_backward(r, w)
        ctx.cfg = (float(rc), float(p))
        return _native.ops().mace_radial_fwd(r, w, *ctx.cfg)

    @staticmethod
    def backward(ctx, g):
        r, w = ctx.saved_tensors
        dr = _native.ops().mace_radial_bwd(g, r, w, *ctx.cfg) if ctx.needs_input_grad[0] else None
        return dr, None, None, None


class RadialEmbeddingBlock(nn.Module):
    def __init__(self, r_max, num_bessel, num_polynomial_cutoff, radial_type="bessel", distance_transform=None):
        super().__init__()
        if radial_type in (None, "bessel"):
            self.bessel_fn = MACEBesselBasis(r_max, num_bessel)
        elif radial_type == "gaussian":
            self.bessel_fn = GaussianBasis(r_max, num_bessel)
        elif radial_type == "chebyshev":
            self.bessel_fn = ChebychevBasis(r_max, num_bessel)
        else:
            raise ValueError(f"unknown radial_type {radial_type}")
        from ..ops.covalent import AgnesiTransform, SoftTransform

        if distance_transform in (None, "None"):
            self.distance_transform = None
        elif distance_transform == "Agnesi":
            self.distance_transform = AgnesiTransform()
        elif distance_transform == "Soft":
            self.distance_transform = SoftTransform()
        else:
            raise ValueError(f"unknown distance_transform {distance_transform}")
        self.cutoff_fn = PolynomialCutoff(r_max, num_polynomial_cutoff)
        self.out_dim = num_bessel

    def forward(self, edge_lengths, z_src=None, z_dst=None):
        """(reference ``blocks.py:148-162``): the cutoff acts on the raw length, the basis on
        the (optionally) transformed one."""
        bf = self.bessel_fn
        if (self.distance_transform is None and isinstance(bf, MACEBesselBasis) and edge_lengths.is_cuda
                and edge_lengths.dtype == torch.float32 and not bf.bessel_weights.requires_grad and fused("radial")):
            # basis x cutoff in one HIP launch (csrc/radial.hip mace_radial_fwd), first order
            return _MaceRadial.apply(edge_lengths.reshape(-1), bf.bessel_weights, self.cutoff_fn.r_max,
                                     self.cutoff_fn.p)
        cutoff = self.cutoff_fn(edge_lengths)
        if self.distance_transform is not None:
            edge_lengths = self.distance_transform(edge_lengths, z_src, z_dst)
        return self.bessel_fn(edge_lengths) * cutoff


# ----------------------------------------------------------------------------- blocks
_PERM_CACHE = {}


def _to_channels(x, irreps):
    """flat e3nn layout (blocks of [H, 2l+1], equal H) -> [N, H, sum(2l+1)].

    The map is a fixed column permutation: on the GPU ONE column gather (backward: one
    index-add) instead of per-block reshapes + concat (whose backward copies every
    non-contiguous block gradient)."""
    N = x.shape[0]
    if x.is_cuda and len(irreps.blocks) > 1:
        key = (tuple(irreps.blocks), x.device)
        perm = _PERM_CACHE.get(key)
        if perm is None:
            H = irreps.blocks[0][0]
            cols = []
            for u in range(H):
                for (a, b), (m, l, _) in zip(irreps.slices(), irreps.blocks):
                    d = 2 * l + 1
                    cols += [a + u * d + c for c in range(d)]
            perm = torch.tensor(cols, dtype=torch.long, device=x.device)
            _PERM_CACHE[key] = perm
        return x.index_select(1, perm).view(N, irreps.blocks[0][0], -1)
    parts = torch.split(x, [b - a for a, b in irreps.slices()], 1) if len(irreps.blocks) > 1 else [x]
    out = [t.reshape(N, m, 2 * l + 1) for t, (m, l, _) in zip(parts, irreps.blocks)]
    return torch.cat(out, -1) if len(out) > 1 else out[0]


class InteractionBlock(nn.Module):
    """RealAgnosticAttResidualInteractionBlock (reference ``blocks.py:286-388``)."""

    def __init__(self, node_feats_irreps, edge_attrs_irreps, num_edge_feats, target_irreps, hidden_irreps,
                 avg_num_neighbors):
        super().__init__()
        self.node_feats_irreps, self.edge_attrs_irreps = node_feats_irreps, edge_attrs_irreps
        self.target_irreps, self.hidden_irreps = target_irreps, hidden_irreps
        self.avg_num_neighbors = avg_num_neighbors
        n_down = hidden_irreps.count(0, 1)
        self.linear_up = o3.O3Linear(node_feats_irreps, node_feats_irreps)
        irreps_mid, ins = o3.tp_uvu_instructions(node_feats_irreps, edge_attrs_irreps, target_irreps)
        self.conv_tp = o3.TensorProductUVU(node_feats_irreps, edge_attrs_irreps, irreps_mid, ins)
        self.linear_down = o3.O3Linear(node_feats_irreps, o3.Irreps([(n_down, 0, 1)]))
        self.conv_tp_weights = o3.FullyConnectedNet([num_edge_feats + 2 * n_down] + 3 * [n_down]
                                                    + [self.conv_tp.weight_numel])
        self.linear = o3.O3Linear(irreps_mid.simplify(), target_irreps)
        # the radial MLP's last 1/sqrt(fan_in) and the 1/avg_num_neighbors normalisation are
        # constants on a chain that is linear in them (w -> TP -> segment sum -> linear):
        # folded into the output linear's path scales instead of two elementwise passes
        self.conv_tp_weights.defer_last_scale = True
        self.linear.scale_paths(self.conv_tp_weights.last_scale() / avg_num_neighbors)
        self.skip_linear = o3.O3Linear(node_feats_irreps, hidden_irreps)

    def forward(self, h, edge_attrs, edge_feats, dst_si, src_si):
        # three linears over the same rows: natively their input gradients are one chain of
        # launches with the partial sum in each epilogue (no autograd add per extra consumer)
        sc, up, down = o3.linear_multi([self.skip_linear, self.linear_up, self.linear_down], h)
        # radial FCN over cat[edge_feats, down[src], down[dst]]: first layer split at node level
        w = self.conv_tp_weights.forward_split(edge_feats, down, src_si, dst_si)
        # gather -> uvu tensor product -> segment sum, fused on the GPU (one launch each way)
        msg = self.linear(self.conv_tp.conv(up, edge_attrs, w, src_si, dst_si))  # scales folded (init)
        return _to_channels(msg, self.target_irreps), sc


class EquivariantProductBasisBlock(nn.Module):
    def __init__(self, lmax_in, target_irreps, correlation, num_features, num_elements, use_sc=True):
        super().__init__()
        self.use_sc = use_sc
        self.symmetric_contractions = o3.SymmetricContraction(lmax_in, target_irreps, correlation, num_features,
                                                              num_elements)
        self.linear = o3.O3Linear(target_irreps, target_irreps)

    def forward(self, x, sc, elem):
        # the skip connection is added in the linear's epilogue (natively: no add pass)
        return self.linear(self.symmetric_contractions(x, elem), residual=sc if self.use_sc else None)


def _joined(inv, equiv):
    """``cat([inv, equiv], 1)`` — or, when the two are the adjacent column blocks of one
    [N, F] tensor (the previous layer's output, split for the read-out), that tensor itself:
    no copy forward, no split / concat pair backward (autograd sums the read-out's gradient
    of the ``inv`` view and this layer's gradient of the whole)."""
    b = inv._base
    if (b is not None and equiv._base is b and b.dim() == 2 and inv.dim() == 2 and equiv.dim() == 2 and
            b.is_contiguous() and inv.storage_offset() == b.storage_offset() and
            inv.shape[1] + equiv.shape[1] == b.shape[1] and equiv.storage_offset() == b.storage_offset() + inv.shape[1]
            and inv.shape[0] == b.shape[0] == equiv.shape[0]):
        return b
    return torch.cat([inv, equiv], 1)


class MACELayer(nn.Module):
    def __init__(self, inter, prod, sizing, n_scalars_out):
        super().__init__()
        self.inter, self.prod, self.sizing = inter, prod, sizing
        self.n_scalars_out = n_scalars_out

    def forward(self, inv, equiv, ctx):
        h = _joined(inv, equiv)
        m, sc = self.inter(h, ctx.edge_attributes, ctx.edge_features, ctx.dst_si, ctx.src_si)
        h = self.sizing(self.prod(m, sc, ctx.elem))
        # one split (backward: one concat) instead of two slices (a zero-fill + copy each)
        inv, equiv = h.split([self.n_scalars_out, h.shape[1] - self.n_scalars_out], 1)
        return inv, equiv


class _ScalarLinear(nn.Module):
    """o3.Linear(irreps -> n x 0e): only the scalar block contributes (no bias)."""

    def __init__(self, irreps_in, n_out):
        super().__init__()
        self.lin = o3.O3Linear(irreps_in, o3.Irreps([(n_out, 0, 1)]))

    def forward(self, x):
        return self.lin(x)


class _PerNodeMLP(nn.Module):
    """``mlp_per_node`` MACE read-out (reference ``blocks.py:770-900``, Linear/NonLinear
    MLPNode with ``num_mlp = num_nodes``): graphs of a fixed size, one MLP per node slot.
    The first layer is the slot's o3.Linear to scalars, i.e. a linear map of the scalar
    channels (the only block an irreps -> n x 0e map can use); every layer runs for all
    slots at once as one batched product over stacked weights [slots, in, out] instead
    of the reference's per-slot Python loop with index lists."""

    def __init__(self, input_irreps, dims, act, num_nodes):
        super().__init__()
        assert num_nodes is not None and num_nodes > 0, "num_nodes must be positive integer for MLP"
        self.num_nodes = num_nodes
        self.n_scalar = input_irreps.count(0, 1)
        self.act = act
        self.weights = nn.ParameterList()
        self.biases = nn.ParameterList()
        fan = [self.n_scalar] + list(dims)
        for i in range(len(dims)):
            w = torch.empty(num_nodes, fan[i], fan[i + 1])
            for k in range(num_nodes):
                nn.init.kaiming_uniform_(w[k].T, a=5 ** 0.5)
            self.weights.append(nn.Parameter(w))
            # the o3.Linear first layer has no bias
            self.biases.append(nn.Parameter(torch.zeros(num_nodes, fan[i + 1]), requires_grad=i > 0))

    def forward(self, x):
        nn_ = self.num_nodes
        G = x.shape[0] // nn_
        xs = x if x.shape[1] == self.n_scalar else x[:, :self.n_scalar]
        h = xs.reshape(G, nn_, -1).transpose(0, 1)  # [slots, G, F]
        # o3.Linear normalisation of the scalar block: 1/sqrt(fan_in)
        h = torch.baddbmm(self.biases[0].unsqueeze(1), h, self.weights[0]) / self.n_scalar ** 0.5
        for i in range(1, len(self.weights)):
            h = torch.baddbmm(self.biases[i].unsqueeze(1), self.act(h), self.weights[i])
        return h.transpose(0, 1).reshape(G * nn_, -1)


def _bmlp_ok():
    from ..ops.pna import fused

    return fused("linear") and os.environ.get("HYDRA_BRANCH_MLP", "1") == "1"


class MultiheadDecoderBlock(nn.Module):
    """Linear (intermediate) or non-linear (last) MACE read-out over all heads
    (reference ``blocks.py:417-767``)."""

    def __init__(self, nonlinear, input_irreps, config_heads, head_dims, head_type, num_heads, act, num_nodes):
        super().__init__()
        self.nonlinear = nonlinear
        self.head_dims, self.head_type, self.num_heads = head_dims, head_type, num_heads
        self.config_heads = config_heads
        self.input_scalar_dim = input_irreps.count(0, 1)
        self.graph_shared = ModuleDict({})
        self.heads_NN = ModuleList()
        self.num_branches = len(config_heads["graph"]) if "graph" in config_heads else (
            len(config_heads["node"]) if "node" in config_heads else 1)
        if nonlinear and "graph" in config_heads:
            for b in config_heads["graph"]:
                a = b["architecture"]
                ds = a["dim_sharedlayers"]
                layers = [Linear(self.input_scalar_dim, ds), act]
                for _ in range(a["num_sharedlayers"] - 1):
                    layers += [Linear(ds, ds), act]
                self.graph_shared[b["type"]] = Sequential(*layers)
        for ih in range(num_heads):
            hn = ModuleDict({})
            if head_type[ih] == "graph":
                for b in config_heads["graph"]:
                    a = b["architecture"]
                    if nonlinear:
                        dh = a["dim_headlayers"]
                        layers = [Linear(a["dim_sharedlayers"], dh[0]), act]
                        for il in range(a["num_headlayers"] - 1):
                            layers += [Linear(dh[il], dh[il + 1]), act]
                        layers.append(Linear(dh[-1], head_dims[ih]))
                    else:
                        layers = [Linear(self.input_scalar_dim, head_dims[ih])]
                    hn[b["type"]] = Sequential(*layers)
            elif head_type[ih] == "node":
                for b in config_heads["node"]:
                    a = b["architecture"]
                    if a["type"] == "conv":
                        raise ValueError("Node-level convolutional layers are not supported in MACE")
                    if a["type"] == "mlp_per_node":
                        dims = (list(a["dim_headlayers"]) if nonlinear else []) + [head_dims[ih]]
                        hn[b["type"]] = _PerNodeMLP(input_irreps, dims, act, num_nodes)
                        continue
                    if nonlinear:
                        dh = a["dim_headlayers"]
                        layers = [_ScalarLinear(input_irreps, dh[0]), act]
                        for il in range(len(dh) - 1):
                            layers += [Linear(dh[il], dh[il + 1]), act]
                        layers.append(Linear(dh[-1], head_dims[ih]))
                    else:
                        layers = [_ScalarLinear(input_irreps, head_dims[ih])]
                    hn[b["type"]] = Sequential(*layers)
            else:
                raise ValueError("Unknown head type" + head_type[ih])
            self.heads_NN.append(hn)

    def _chain_steps(self, mods):
        """Sequential head modules -> [(W [out, in], bias | None, act | None)], or None when
        a module is not a plain linear map / activation (e.g. ``mlp_per_node``)."""
        steps = []
        for m in mods:
            if isinstance(m, nn.Linear):
                steps.append([m.weight, m.bias, None, 1.0, (m.weight, 0)])
            elif isinstance(m, _ScalarLinear):
                lin = m.lin
                if len(lin.paths) != 1 or lin.paths[0][0] != 0 or lin.irreps_in.blocks[0][1] != 0:
                    return None
                # raw weight view; the (branch-independent) path normalisation is applied once
                # to the stacked product instead of once per branch weight
                _, _, _, mi, mo, a = lin.paths[0]
                steps.append([lin.weight.view(mi, mo).t(), None, None, a, (lin.weight, 1)])
                continue
            elif steps and steps[-1][2] is None and not isinstance(m, (nn.Sequential, _PerNodeMLP)):
                steps[-1][2] = m
            else:
                return None
        return steps

    @staticmethod
    def _row_select(ctx, rid, tag):
        """(gather index [R, 1, 1] int64, valid-row mask [R, 1]) of a row -> branch id vector,
        built once per forward and shared by every read-out (padding rows: id -1 -> 0, masked)."""
        cache = ctx.get("_mace_rowsel")
        if cache is None:
            cache = {}
            ctx._mace_rowsel = cache
        key = (tag, rid.shape[0])
        if key not in cache:
            cache[key] = (rid.clamp(min=0).view(-1, 1, 1), (rid >= 0).to(torch.float32).view(-1, 1))
        return cache[key]

    @staticmethod
    def _rid32(ctx, rid, tag):
        """int32 row -> branch ids (padding rows -1), built once per forward per row kind."""
        cache = ctx.get("_mace_rid32")
        if cache is None:
            cache = {}
            ctx._mace_rid32 = cache
        key = (tag, rid.shape[0])
        if key not in cache:
            cache[key] = rid.to(torch.int32).contiguous()
        return cache[key]

    def _stacked_dense(self, names, gfeat, sc, dn, dn_node, ctx=None, acc=None):
        """Dense multi-branch decode with the branches STACKED: per layer one GEMM over all
        branches (the first layer's weights concatenated along the output, later layers one
        batched product), then one per-row gather of the row's own branch.  Same values as
        evaluating every branch head on every row and selecting with ``torch.where`` (the
        reference decode ``blocks.py:417-767`` per branch), at a launch count independent of
        the branch count.  None when the heads are not plain MLP chains."""
        nb = len(names)
        if [int(b.split("-")[1]) for b in names] != list(range(nb)):
            return None
        outs = []
        for ih, (hd, hn, t) in enumerate(zip(self.head_dims, self.heads_NN, self.head_type)):
            chains = []
            for bt in names:
                mods = list(hn[bt]) if isinstance(hn[bt], nn.Sequential) else None
                if mods is None:
                    return None
                if t == "graph" and self.nonlinear:
                    mods = list(self.graph_shared[bt]) + mods
                st = self._chain_steps(mods)
                if st is None:
                    return None
                chains.append(st)
            shapes = [[(tuple(s[0].shape), s[1] is None, type(s[2]), s[3]) for s in c] for c in chains]
            if any(s != shapes[0] for s in shapes):
                return None
            x, rid = (gfeat, dn) if t == "graph" else (sc, dn_node)
            R = x.shape[0]
            if ctx is not None and _bmlp_ok():
                # every row through its own branch's chain: one launch each way (ops/branch_mlp.py)
                bch = [[(st[4][0], st[4][1], st[1], st[2], st[3]) for st in c] for c in chains]
                if _bmlp.eligible(x, bch):
                    a = acc[ih] if acc is not None else None
                    if a is not None and not (a.shape == (R, hd) and a.dtype == x.dtype):
                        a = None
                    o = _bmlp.branch_mlp(x, self._rid32(ctx, rid, t), bch, hd, acc=a)
                    outs.append(o if (a is not None or acc is None) else o + acc[ih])
                    continue
            h = None  # [nb, features, R]: weights multiply from the LEFT, so the weight
            # gradients come out in the parameters' own layout (no per-parameter copies)
            for li in range(len(chains[0])):
                Ws = [c[li][0] for c in chains]
                bs = [c[li][1] for c in chains]
                act, scale = chains[0][li][2], chains[0][li][3]
                out_dim = Ws[0].shape[0]
                if li == 0:  # shared input: one GEMM against the branch-concatenated weights
                    xs = x * scale if scale != 1.0 else x
                    y = torch.nn.functional.linear(xs, torch.cat(Ws, 0), None if bs[0] is None else torch.cat(bs, 0))
                    h = y.t().view(nb, out_dim, R)
                else:
                    hs = h * scale if scale != 1.0 else h
                    W = torch.stack(Ws, 0)
                    h = torch.bmm(W, hs) if bs[0] is None else torch.baddbmm(torch.stack(bs, 0).unsqueeze(2), W, hs)
                if act is not None:
                    h = act(h)
            h = h[:, :hd, :].permute(2, 0, 1)  # [R, nb, hd]
            if ctx is not None:
                idx, valid = self._row_select(ctx, rid, t)
                sel = h.gather(1, idx.expand(R, 1, hd)).squeeze(1)
                outs.append(sel * valid.to(sel.dtype) if acc is None else acc[ih] + sel * valid.to(sel.dtype))
            else:
                sel = h.gather(1, rid.clamp(min=0).view(R, 1, 1).expand(R, 1, hd)).squeeze(1)
                sel = torch.where((rid >= 0).unsqueeze(1), sel, torch.zeros((), dtype=sel.dtype, device=sel.device))
                outs.append(sel if acc is None else acc[ih] + sel)
        return outs

    def forward(self, node_features, ctx, ids, acc=None):
        """Read-out of every head; ``acc`` (the previous layers' summed read-outs): the result
        is ``acc + read-out`` (fused into the branch kernel on the captured path)."""
        if acc is not None:
            out = self._forward(node_features, ctx, ids, acc)
            if isinstance(out, tuple):  # (outputs, fused) from the stacked path
                return out[0]
            return [a + b for a, b in zip(acc, out)]
        return self._forward(node_features, ctx, ids, None)

    def _forward(self, node_features, ctx, ids, acc):
        gsi = ctx.graph_si
        # the read-outs only use the scalar channels; the stack hands over just those
        sc = node_features if node_features.shape[1] == self.input_scalar_dim else \
            node_features[:, :self.input_scalar_dim]
        # padded batch: the limit skips the padding graph's (long, all-zero) segment
        gfeat = sc.mean(0, keepdim=True) if gsi is None else \
            seg.segment_mean(sc, gsi, limit=ctx.data.get("num_valid"))
        data = ctx.data
        outs = []
        granges, nranges = data.get("branch_graph_ranges"), data.get("branch_node_ranges")
        if self.num_branches > 1 and ids is None:
            # statically padded (captured) batch: every branch densely, selected per row
            dn = data.dataset_name.view(-1)
            dn_node = ctx.get("_mace_dn_node")
            if dn_node is None:  # once per forward (shared by every read-out)
                dn_node = ctx._mace_dn_node = dn.index_select(0, data.batch)
            names = sorted(self.heads_NN[0].keys(), key=lambda k: int(k.split("-")[1]))
            stacked = self._stacked_dense(names, gfeat, sc, dn, dn_node, ctx, acc=acc)
            if stacked is not None:
                return (stacked, True) if acc is not None else stacked
            for hd, hn, t in zip(self.head_dims, self.heads_NN, self.head_type):
                feats, rid = (gfeat, dn) if t == "graph" else (node_features, dn_node)
                out = feats.new_zeros(feats.shape[0], hd)
                for bt in names:
                    x = self.graph_shared[bt](feats) if (t == "graph" and self.nonlinear) else feats
                    out = torch.where((rid == int(bt.split("-")[1])).unsqueeze(1), hn[bt](x)[:, :hd], out)
                outs.append(out)
            return outs
        if self.num_branches > 1 and granges is not None and len(granges) > 1:
            # store batches are grouped by branch: contiguous slices, no masks / host syncs
            for hd, hn, t in zip(self.head_dims, self.heads_NN, self.head_type):
                feats, rng, total = (gfeat, granges, gfeat.shape[0]) if t == "graph" else \
                    (node_features, nranges, node_features.shape[0])
                parts = []
                for ID, a, b in rng:
                    bt = f"branch-{ID}"
                    x = feats[a:b]
                    if t == "graph" and self.nonlinear:
                        x = self.graph_shared[bt](x)
                    parts.append(hn[bt](x)[:, :hd])
                if rng[-1][2] < total:
                    parts.append(feats.new_zeros(total - rng[-1][2], hd))
                outs.append(torch.cat(parts, 0))
            return outs
        for hd, hn, t in zip(self.head_dims, self.heads_NN, self.head_type):
            if t == "graph":
                if self.num_branches == 1 or len(ids) <= 1:
                    bt = f"branch-{ids[0] if ids else 0}" if self.num_branches > 1 else "branch-0"
                    x = self.graph_shared[bt](gfeat) if self.nonlinear else gfeat
                    outs.append(hn[bt](x)[:, :hd])
                else:
                    dn = data.dataset_name.view(-1)
                    head = gfeat.new_zeros(gfeat.shape[0], hd)
                    for ID in ids:
                        mask = dn == ID
                        bt = f"branch-{ID}"
                        x = gfeat[mask]
                        x = self.graph_shared[bt](x) if self.nonlinear else x
                        head = head.index_put((mask,), hn[bt](x)[:, :hd])
                    outs.append(head)
            else:
                if self.num_branches == 1 or len(ids) <= 1:
                    bt = f"branch-{ids[0] if ids else 0}" if self.num_branches > 1 else "branch-0"
                    outs.append(hn[bt](node_features)[:, :hd])
                else:
                    dn = data.dataset_name.view(-1)
                    head = node_features.new_zeros(node_features.shape[0], hd)
                    for ID in ids:
                        mask = (dn == ID)[data.batch]
                        head = head.index_put((mask,), hn[f"branch-{ID}"](node_features[mask])[:, :hd])
                    outs.append(head)
        return outs


# ----------------------------------------------------------------------------- stack
def process_node_attributes(x, num_elements=NUM_ELEMENTS):
    """Atomic numbers (data.x) -> one-hot [N, 118] (reference ``MACEStack.py:485-520``)."""
    z = x.squeeze()
    if z.dim() == 0:
        z = z.view(1)
    assert z.dim() == 1, "MACE only supports raw atomic numbers as node_attributes (1D data.x)."
    capturing = z.is_cuda and torch.cuda.is_current_stream_capturing()
    if not capturing:  # host-side checks would synchronise inside a hipGraph capture
        if not bool(torch.all(z == z.round())):
            warnings.warn("MACE only supports raw atomic numbers as node_attributes. Your data.x contains floats.")
        if not bool(torch.all((z >= 1) & (z <= num_elements))):
            warnings.warn("MACE only supports raw atomic numbers as node_attributes. Your data.x is not in 1-118.")
    z = z.clamp(1, num_elements)
    idx = (z - 1).long()
    return torch.nn.functional.one_hot(idx, num_classes=num_elements).float(), idx


class MACEStack(Base):
    is_edge_model = True


    def branch_param_groups(self):
        """Per-branch read-out parameters of every layer's decoder (graph shared MLP + each
        head's branch module), in branch id order: the usage groups of the captured step, so a
        branch absent from a batch keeps torch's skip-if-no-grad semantics (its heads get a
        zero gradient from the dense / branch-keyed decode, and FusedAdamW skips them)."""
        if self.num_branches <= 1:
            return []
        names = sorted(self.multihead_decoders[0].heads_NN[0].keys(), key=lambda k: int(k.split("-")[1]))
        groups = []
        for bt in names:
            ps = []
            for dec in self.multihead_decoders:
                if bt in dec.graph_shared:
                    ps += list(dec.graph_shared[bt].parameters())
                for hn in dec.heads_NN:
                    if bt in hn:
                        ps += list(hn[bt].parameters())
            groups.append([p for p in ps if p.requires_grad])
        return groups

    def __init__(self, input_args, conv_args, r_max, radial_type, distance_transform, num_bessel, edge_dim, max_ell,
                 node_max_ell, avg_num_neighbors, num_polynomial_cutoff, correlation, *args, **kwargs):
        self.max_ell = max_ell
        self.node_max_ell = node_max_ell
        self.edge_dim = edge_dim
        self.avg_num_neighbors = avg_num_neighbors
        self.num_elements = NUM_ELEMENTS
        self.num_polynomial_cutoff = 5 if num_polynomial_cutoff is None else num_polynomial_cutoff
        corr = 2 if correlation is None else correlation
        self.correlation = corr if isinstance(corr, (list, tuple)) else [corr]
        self.radial_type = "bessel" if radial_type is None else radial_type
        self.num_bessel = num_bessel
        self.r_max = r_max
        super().__init__(input_args, conv_args, *args, **kwargs)
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, self.num_polynomial_cutoff, self.radial_type,
                                                     distance_transform)
        self.node_embedding = o3.O3Linear(o3.Irreps([(self.num_elements, 0, 1)]),
                                          o3.Irreps([(self.hidden_dim, 0, 1)]))

    # decoders are built per layer; Base's multi-head decoder is not used
    def _multihead(self):
        self.num_branches = len(self.config_heads["graph"]) if "graph" in self.config_heads else 1

    def _init_conv(self):
        H = self.hidden_dim
        self.sh_irreps = o3.Irreps.sh(self.max_ell)
        if self.use_edge_attr:
            # every edge-attribute scalar is its own 1x0e block (not merged with Y_0 into one
            # multi-channel 0e block): the uvu product is the same function class (one weight
            # per (u, v) either way), and single-channel blocks keep the fused HIP convolution
            # (csrc/equivariant.hip) applicable
            self.edge_attrs_irreps = o3.Irreps([(1, 0, 1)] * self.edge_dim) + self.sh_irreps
        else:
            self.edge_attrs_irreps = self.sh_irreps
        hidden = o3.Irreps.natural(H, self.node_max_ell)
        final = o3.Irreps.natural(H, 0)
        self.multihead_decoders = ModuleList()
        n = self.num_conv_layers
        dec = lambda nonlin, irr: MultiheadDecoderBlock(nonlin, irr, self.config_heads, self.head_dims,  # noqa: E731
                                                         self.head_type, self.num_heads, self.activation_function,
                                                         self.num_nodes)
        self.multihead_decoders.append(dec(n == 1, o3.Irreps([(self.num_elements, 0, 1)])))
        for i in range(n):
            last = i == n - 1
            self.graph_convs.append(self._apply_global_attn(self.get_conv(H, H, first_layer=i == 0, last_layer=last,
                                                                          layer=i)))
            self.feature_layers.append(nn.Identity())
            self.multihead_decoders.append(dec(last, final if last else hidden))

    def get_conv(self, input_dim, output_dim, first_layer=False, last_layer=False, layer=0):
        hidden_dim = output_dim if input_dim == 1 else input_dim
        node_feats = o3.Irreps.natural(input_dim, 0 if first_layer else self.node_max_ell)
        hidden = o3.Irreps.natural(hidden_dim, self.node_max_ell)
        interaction = o3.Irreps.natural(hidden_dim, self.max_ell)
        output = o3.Irreps.natural(output_dim, self.node_max_ell)
        if last_layer:
            hidden = o3.Irreps.natural(hidden_dim, 0)
            output = o3.Irreps.natural(output_dim, 0)
        # under GPS the edge features are the hidden-width relative-PE encoding (reference
        # MACEStack.py:455-462); size the radial MLP input for it (the reference would not run)
        n_edge = self.hidden_dim if (self.use_global_attn and self.is_edge_model) else self.num_bessel
        inter = InteractionBlock(node_feats, self.edge_attrs_irreps, n_edge, interaction, hidden,
                                 self.avg_num_neighbors)
        # per-layer correlation order (reference MACEStack.py: ``correlation`` may be a list, one
        # entry per interaction layer; a scalar applies to all)
        corr = self.correlation[min(layer, len(self.correlation) - 1)]
        prod = EquivariantProductBasisBlock(self.max_ell, hidden, corr, hidden_dim, self.num_elements, use_sc=True)
        sizing = o3.O3Linear(hidden, output)
        return MACELayer(inter, prod, sizing, output.count(0, 1))

    def _embedding(self, data):
        ctx = self._base_ctx(data)
        assert data.pos is not None, "MACE requires node positions (data.pos) to be set."
        pos = data.pos
        # centre positions per graph (reference MACEStack.py:411-419)
        if ctx.graph_si is None:
            pos = pos - pos.mean(0, keepdim=True)
        else:
            # (padded batch: the padding graph's rows are skipped by the limit; its nodes keep
            # their raw positions, a common shift that leaves every padding distance unchanged)
            pos = pos - seg.gather(seg.segment_mean(pos, ctx.graph_si, limit=data.get("num_valid")),
                                   ctx.graph_si)
        vec, dist = edge_vectors_and_lengths(pos, ctx.dst_si, ctx.src_si, data.get("edge_shifts"))
        node_attrs, elem = process_node_attributes(data.x)
        # element-indexed weight tables are gathered, not multiplied by the one-hot: the node
        # embedding and every symmetric contraction use the element SegIndex (the one-hot
        # only feeds the first linear read-out, as in the reference)
        ctx.node_attributes, ctx.elem = node_attrs, o3.element_index(elem, self.num_elements)
        node_feats = self.node_embedding.lookup(ctx.elem)
        ea = o3.spherical_harmonics(self.max_ell, vec)
        if self.use_edge_attr:
            ea = torch.cat([data.edge_attr, ea], 1)
        ctx.edge_attributes = ea
        z = elem + 1  # one-hot index -> atomic number (covalent-radius table index)
        if self.radial_embedding.distance_transform is not None:
            ctx.edge_features = self.radial_embedding(dist, z[ctx.src_si.index64], z[ctx.dst_si.index64])
        else:
            ctx.edge_features = self.radial_embedding(dist)
        if self.use_global_attn:
            x = self.pos_emb(data.pe)
            if self.input_dim:
                x = self.node_lin(torch.cat((node_feats, x), 1))
            if self.is_edge_model:
                e = self.rel_pos_emb(data.rel_pe)
                if self.use_edge_attr:
                    # the reference concatenates the radial features here, which only fits when
                    # num_bessel == hidden_dim; encode the edge attributes like every other stack
                    e = self.edge_lin(torch.cat((self.edge_emb(data.edge_attr), e), 1))
                ctx.edge_features = e
            return x[:, :self.hidden_dim], x[:, self.hidden_dim:], ctx
        return node_feats[:, :self.hidden_dim], node_feats[:, self.hidden_dim:], ctx

    def forward(self, data):
        inv, equiv, ctx = self._embedding(data)
        ids = self._branch_ids(data) if self.num_branches > 1 else [0]
        if self.num_branches > 1 and data.get("dataset_name") is not None:
            self._note_branch_presence(data.dataset_name.view(-1))  # captured step's usage flags
        outputs = self.multihead_decoders[0](ctx.node_attributes, ctx, ids)
        for conv, readout in zip(self.graph_convs, self.multihead_decoders[1:]):
            inv, equiv = self._run_conv(conv, inv, equiv, ctx)
            outputs = readout(inv, ctx, ids, acc=outputs)  # scalar block only; + the running sum
        return outputs

    def __str__(self):
        return "MACEStack"
