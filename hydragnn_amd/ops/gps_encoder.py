"""Fused GPS(PNAPlus) encoder: the whole conv stack as ONE autograd function over the
kernels of ``csrc/gps_fused.hip`` (plus the PNA, attention, edge-linear and weight-prep
kernels it shares with the unfused path).

Reference computation per layer (``globalAtt/gps.py:103-152`` around
``PNAPlusStack.py:228-279``, then ``Base.py:466``)::

    h_att = BN2(drop(MHA(x)) + x)
    h_loc = BN1(drop(lin(post_nn(PNA(x)))) + x)
    out   = h_loc + h_att
    z3    = drop(W2 drop(relu(W1 out + b1)) + b2) + out
    x'    = relu(BN4(BN3(z3)))            (rows >= num_valid -> 0)

Stream schedule (all captured into the step graph as parallel branches):

* prologue: every layer's weight prep (one launch); on a third stream the edge chain
  (edge embedding, radial basis + every layer's radial embedding, every layer's edge term
  C = r Wr^T + e Wd^T + bc in one launch) beside the node embedding and the first layer;
* forward per layer: node GEMM [AB | qkv] (+ previous layer's BN3/BN4 finalise + apply in
  its prologue), {side stream: attention, o-proj + BN2 stats}, PNA aggregate (joins the
  edge chain once), post/lin GEMM chain + BN1 stats, {join} BN1/BN2 apply + MLP chain + BN3
  stats;
* backward per layer: mlp, {side: BN2 + o-proj dgrad whose epilogue packs the attention
  operands, attention}, BN1 + lin/post dgrad, [third stream: the previous layer's weight
  gradients, one grouped launch pair, beside this layer's attention], PNA, [third stream:
  edge dgrad (the first layer's on a fourth)], {join} node dgrad + previous pair statistics;
  the first layer's and the embeddings' weight gradients close the backward on the main
  stream.

BN4 o BN3 is a single per-column affine map: BN4's batch statistics are derived from
BN3's (mean4 = beta3, var4 = gamma3^2 var3 / (var3 + eps3)), and its backward is closed-
form (``csrc/gps_fused.hip``, "BN3 -> BN4 pair").  Mathematically identical to the
reference; numerically equal to fp32 rounding.

Used in GPU training mode when every layer matches the pattern (``eligible``); CPU,
eval, double-backward (composite mode) and any other configuration run the module path.
``HYDRA_UNFUSED=gpsfused`` switches it off.
"""
import os

import torch

from .. import _native
from . import pna as _mode
from . import streams as _streams
from ..parallel import gradslots as _gradslots

NREP = 8
SITES = 11  # fwd BN1 (2) + BN2 (2) + BN3 (2) + bwd pair (2) + bwd BN1/BN2 (3)
NSAVED = 7


def _bn(m):
    return m.module if hasattr(m, "module") else m


def _bn_ok(m, F):
    b = _bn(m)
    return (isinstance(b, torch.nn.BatchNorm1d) and b.affine and b.momentum is not None and b.training
            and b.num_features == F)


def pre_eligible(model, data):
    """Cheap checks before the embedding runs (the fused path absorbs the GPS embedding)."""
    x = data.get("x")
    return (model.training and x is not None and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
            and model.input_dim and 1 <= x.shape[1] <= 16 and data.get("pe") is not None
            and data.pe.shape[1] <= 16 and model.is_edge_model and model.use_edge_attr
            and data.get("edge_attr") is not None and data.edge_attr.dim() == 2 and data.edge_attr.shape[1] <= 16
            and data.get("rel_pe") is not None and data.rel_pe.shape[1] <= 16
            and not (data.x.requires_grad or data.pe.requires_grad or data.edge_attr.requires_grad)
            and _mode.fused("gpsfused") and model.hidden_dim in (32, 64))


def eligible(model, ctx):
    """True when the fused encoder reproduces ``Base.encode`` for this model and batch."""
    from ..models.gps import GPSConv, MultiheadAttention
    from ..models.pnaplus import PNAConvFused

    if not (_mode.fused("gpsfused") and _mode.fused("attn") and _mode.fused("pna") and model.training):
        return False
    F = model.hidden_dim
    if F not in (32, 64) or model.conv_checkpointing:
        return False
    if not isinstance(model.activation_function, torch.nn.ReLU):
        return False
    from .radial import MAX_K, MAX_L

    dist, geom = ctx.get("dist"), ctx.get("geom")
    if dist is None:
        if geom is None or geom[0].requires_grad or geom[0].dtype != torch.float32 or not geom[0].is_cuda:
            return False
        if ctx.src_si is None or ctx.src_si.index.dtype != torch.int32 or ctx.dst_si.index.dtype != torch.int32:
            return False
    elif dist.requires_grad or not dist.is_cuda:
        return False  # the radial basis is computed inside the encoder (no force training)
    if ctx.get("rbf_basis") is None:
        return False
    if ctx.rbf_basis.freq.numel() > MAX_K or len(model.graph_convs) > MAX_L or not _mode.fused("radial"):
        return False

    if ctx.dst_si is None or ctx.dst_si.perm is not None or ctx.get("attn_seg_id") is None:
        return False
    for conv, bn in zip(model.graph_convs, model.feature_layers):
        if not isinstance(conv, GPSConv) or not isinstance(conv.attn, MultiheadAttention):
            return False
        c = conv.conv
        if not (isinstance(c, PNAConvFused) and c.plus and c.edge_dim is not None):
            return False
        if c.F_in != F or c.F_out != F or not hasattr(c, "edge_encoder"):
            return False
        if not isinstance(conv.mlp[1], torch.nn.ReLU):
            return False
        if any(n is None or not _bn_ok(n, F) for n in (conv.norm1, conv.norm2, conv.norm3)) or not _bn_ok(bn, F):
            return False
        D = F // conv.heads
        if D not in (4, 8, 16, 32, 64) or conv.attn.in_proj_bias is None:
            return False
    return True


def _layer_params(conv, bn4):
    c = conv.conv
    at = conv.attn
    n1, n2, n3, n4 = _bn(conv.norm1), _bn(conv.norm2), _bn(conv.norm3), _bn(bn4)
    lin1, _, _, lin2, _ = conv.mlp
    return [at.in_proj_weight, at.in_proj_bias, at.out_proj.weight, at.out_proj.bias,
            c.pre_nns[0][0].weight, c.pre_nns[0][0].bias, c.edge_encoder.weight, c.edge_encoder.bias,
            c.post_nns[0][0].weight, c.post_nns[0][0].bias, c.lin.weight, c.lin.bias,
            n1.weight, n1.bias, n2.weight, n2.bias, n3.weight, n3.bias, n4.weight, n4.bias,
            lin1.weight, lin1.bias, lin2.weight, lin2.bias,
            c.rbf_emb[0].weight, c.rbf_emb[0].bias, c.rbf_lin.weight]


NP = 27


class _Cfg:
    pass


def encode(model, ctx):
    """Run the fused encoder: returns x_L (the input of the decoder heads)."""
    from . import rng as _rng
    from .attention import _SPLITS, _max_span

    data = ctx.data
    x0 = data.x
    cfg = _Cfg()
    convs = list(model.graph_convs)
    cfg.L = len(convs)
    cfg.F = model.hidden_dim
    cfg.bns = [(_bn(c.norm1), _bn(c.norm2), _bn(c.norm3), _bn(b)) for c, b in zip(convs, model.feature_layers)]
    cfg.salts = [list(c._salts) for c in convs]
    cfg.p = float(convs[0].dropout) if model.training else 0.0
    cfg.rng = _rng.counter(x0.device) if cfg.p > 0 else None
    cfg.heads = convs[0].heads
    cfg.scale = 1.0 / float(cfg.F // cfg.heads) ** 0.5
    cfg.sid, cfg.sptr = ctx.attn_seg_id, ctx.attn_seg_ptr
    cfg.span = _max_span(x0.shape[0], cfg.sptr)
    cfg.splits = _SPLITS
    cfg.dst, cfg.src = ctx.dst_si, ctx.src_si
    cfg.avg = [(float(c.conv.avg_deg["log"]), float(c.conv.avg_deg["lin"])) for c in convs]
    nv = ctx.get("num_valid")
    if nv is not None:
        from .norm import _as_nv

        nv = _as_nv(nv, x0.device)
    cfg.nv = nv
    cfg.side = _streams.enabled(x0)
    # 8-wide heads: MFMA attention (csrc/attention8.hip) on operands the node kernel packs
    cfg.a8 = cfg.F // cfg.heads == 8 and _mode.fused("attn8")
    # precision "bf16": the attention products on bf16 MFMA (fp32 accumulate, fp32 softmax)
    from .linear import get_precision

    cfg.bf16 = cfg.a8 and cfg.splits <= 0 and get_precision() == "bf16"

    basis = ctx.rbf_basis
    cfg.cutoff, cfg.exponent = float(basis.cutoff), int(basis.envelope.p - 1)
    flat = []
    for c, b in zip(convs, model.feature_layers):
        flat += _layer_params(c, b)
    emb = [model.node_emb.weight, model.pos_emb.weight, model.node_lin.weight,
           model.edge_emb.weight, model.rel_pos_emb.weight, model.edge_lin.weight]
    ins = [data.x.float().contiguous(), data.pe.contiguous(), ctx.edge_attr_raw.contiguous(), data.rel_pe.contiguous()]
    gsi = ctx.get("graph_si")
    cfg.gptr = gsi.rowptr if (gsi is not None and gsi.rowptr.dtype == torch.int32
                              and gsi.index.dtype == torch.int32 and gsi.rowptr.is_cuda) else None
    cfg.gidx = gsi.index if cfg.gptr is not None else None
    if ctx.get("dist") is None:  # distances computed inside the radial launch
        pos, shifts = ctx.geom
        cfg.geom = (pos.contiguous(), cfg.dst.index, cfg.src.index,
                    shifts.float().contiguous() if shifts is not None else None)
        dist = None
    else:
        cfg.geom = None
        dist = ctx.dist.contiguous()
    xL, pooled = _GPSEncoder.apply(cfg, dist, basis.freq, *ins, *emb, *flat)
    if cfg.gptr is not None:
        ctx.pooled = pooled  # per-graph mean of x_L (Base.decode), pooled inside the final launch
    return xL


class _Side:
    """Fork/join of the attention branch onto the cached side stream (capture-safe)."""

    def __init__(self, dev, on):
        self.on = on
        if on:
            self.main = torch.cuda.current_stream(dev)
            self.side = _streams.side_stream(dev)

    def __enter__(self):
        if self.on:
            self.side.wait_stream(self.main)
            self._c = torch.cuda.stream(self.side)
            self._c.__enter__()
        return self

    def __exit__(self, *exc):
        if self.on:
            self._c.__exit__(*exc)
        return False

    def used(self, *ts):  # main-stream tensors read on the side stream
        if self.on:
            for t in ts:
                if t is not None:
                    t.record_stream(self.side)

    def join(self, *ts):  # side-stream results read on the main stream
        if self.on:
            self.main.wait_stream(self.side)
            for t in ts:
                if t is not None:
                    t.record_stream(self.main)


def _bn_state(b):
    track = b.track_running_stats and b.running_mean is not None
    return ((b.running_mean if track else None), (b.running_var if track else None),
            (b.num_batches_tracked if track and b.num_batches_tracked is not None else None),
            float(b.momentum), float(b.eps))


class _GPSEncoder(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, dist, freq, xin, pe, eattr, rpe, Wne, Wpe, Wnl, Wee, Wrp, Wel, *flat):
        ops = _native.ops()
        L, F = cfg.L, cfg.F
        prm = [flat[NP * l: NP * (l + 1)] for l in range(L)]
        dev = xin.device
        nv, rng, p = cfg.nv, cfg.rng, cfg.p
        # the PNAPlus edge term C = r Wr^T + e Wd^T + bc depends on no node state: every layer's
        # is computed up front (one launch) instead of inside the local branch of its layer
        # (the critical path of the layer's two-stream fork; concurrent with the attention
        # kernels the per-layer edge launch took ~3x its standalone time)
        hoist = os.environ.get("HYDRA_EDGE_HOIST", "1") == "1"
        if hoist:
            pw = ops.pna_wprep_fwd_multi([q[4] for q in prm], [q[5] for q in prm], [q[6] for q in prm],
                                         [q[7] for q in prm])
            preps = [pw[4 * l: 4 * l + 4] for l in range(L)]
        # the edge chain (edge embedding -> radial basis / per-layer embeddings -> edge terms)
        # feeds only the local branches: on a third stream it overlaps the node embedding, the
        # first node launch and the first attention; the main stream joins it just before the
        # first PNA aggregation
        eside = hoist and cfg.side and os.environ.get("HYDRA_EDGE_SIDE", "1") == "1"
        geo = cfg.geom if cfg.geom is not None else (None, None, None, None)
        if eside:
            emain = torch.cuda.current_stream(dev)
            estream = _streams.side_stream(dev, 2)
            estream.wait_stream(emain)
            ectx = torch.cuda.stream(estream)
            ectx.__enter__()
        # edge embedding, then edge distances + Bessel basis + every layer's radial embedding /
        # gate in one launch (the basis and its frequency derivative are kept for the weight
        # gradients), then every layer's edge term
        e = ops.gf_embed_fwd(eattr, rpe, Wee, Wrp, Wel, None)
        ro = ops.radial_fwd_multi(dist, freq, [q[24] for q in prm], [q[25] for q in prm], [q[26] for q in prm],
                                  cfg.cutoff, cfg.exponent, bool(freq.requires_grad), *geo)
        rbf, drdf, Rl, Gl = ro[0], ro[1], ro[2:2 + L], ro[2 + L:2 + 2 * L]
        Cs = ops.gf_edge_fwd_multi(list(Rl), e, [q[1] for q in preps], [q[2] for q in preps],
                                   [q[3] for q in preps]) if hoist else None
        if eside:
            ectx.__exit__(None, None, None)
        edge_pending = eside
        # GPS node input embedding (rows >= num_valid -> 0)
        x0 = ops.gf_embed_fwd(xin, pe, Wne, Wpe, Wnl, cfg.nv)
        # BN statistics sites: 3 fixed-point 64-bit words per statistic (deterministic integer
        # atomics, csrc/gps_fused.hip col_sum_add); zeroed by the first node launch
        # the attention + PNA forward as one launch (fp32 quad-block attention, F = 64);
        # HYDRA_GPS_ONE_LAUNCH=0: the two-stream form
        one_launch = (cfg.a8 and not cfg.bf16 and cfg.splits <= 0 and F == 64
                      and os.environ.get("HYDRA_ATTN8_QUAD", "1") != "0"
                      and os.environ.get("HYDRA_GPS_ONE_LAUNCH", "1") == "1")
        acc = torch.empty(L, 3 * NREP * SITES * F, device=dev, dtype=torch.float64)
        saved = torch.empty(L, NSAVED, F, device=dev, dtype=torch.float32)
        st = []
        z3 = None
        for l in range(L):
            (Win, bin_, Wo, bo, Wpre, bpre, Wenc, benc, Wpost, bpost, Wlin, blin,
             g1, b1n, g2, b2n, g3, b3n, g4, b4n, W1, b1, W2, b2, _, _, _) = prm[l]
            r, G = Rl[l], Gl[l]
            s0, s1, s2, s3 = cfg.salts[l]
            Wab, Wr, Wd, bc = preps[l] if hoist else ops.pna_wprep_fwd(Wpre, bpre, Wenc, benc)
            if l == 0:
                outs = ops.gf_node_fwd(x0, Wab, Win, bin_, nv, None, None, [], None, None, None, None, None,
                                       None, 0.0, 0.0, 0.0, 0.0, acc, cfg.a8)
            else:
                _, _, n3p, n4p = cfg.bns[l - 1]
                rm3, rv3, nb3, m3, e3 = _bn_state(n3p)
                rm4, rv4, nb4, m4, e4 = _bn_state(n4p)
                pp = prm[l - 1]
                outs = ops.gf_node_fwd(z3, Wab, Win, bin_, nv, acc[l - 1], saved[l - 1],
                                       [pp[16], pp[17], pp[18], pp[19]], rm3, rv3, nb3, rm4, rv4, nb4,
                                       m3, e3, m4, e4, None, cfg.a8)
            x, AB = outs[0], outs[1]
            pk = outs[2:] if cfg.a8 else None
            qkv = None if cfg.a8 else outs[2]
            if one_launch:
                # attention + PNA aggregation as ONE launch on this stream (no fork / join:
                # each hipGraph fork or join edge cost ~7 us on the layer's critical path)
                if edge_pending:
                    emain.wait_stream(estream)
                    for t in [e, rbf, drdf, *Rl, *Gl, *Cs]:
                        if t is not None:
                            t.record_stream(emain)
                    edge_pending = False
                C = Cs[l] if hoist else ops.gf_edge_fwd(r, e, Wr, Wd, bc)
                O, LSE, Z, amin, amax = ops.attn8_pna_fwd(pk[0], pk[2], pk[5], cfg.sid, cfg.sptr, x.shape[0],
                                                          cfg.scale, x, AB, C, G, cfg.src.index, cfg.dst.rowptr,
                                                          cfg.avg[l][0], cfg.avg[l][1])
                z2, pl, z1 = ops.gf_oproj_post_fwd(O, Wo, bo, Z, Wpost, bpost, Wlin, blin, x, acc[l], rng, s1, s0,
                                                   p, nv)
                n1, n2, _, _ = cfg.bns[l]
                rm1, rv1, nb1, m1, e1 = _bn_state(n1)
                rm2, rv2, nb2, m2, e2 = _bn_state(n2)
                out, md, z3 = ops.gf_mlp_fwd(z1, z2, acc[l], saved[l], [g1, b1n, g2, b2n], rm1, rv1, nb1, rm2, rv2,
                                             nb2, m1, e1, m2, e2, W1, b1, W2, b2, rng, s2, s3, p, nv)
                st.append(dict(x=x, AB=AB, qkv=qkv, pk=pk, O=O, LSE=LSE, z2=z2, C=C, Z=Z, amin=amin, amax=amax,
                               p=pl, z1=z1, out=out, md=md, z3=z3, Wab=Wab, Wr=Wr, Wd=Wd))
                continue
            side = _Side(dev, cfg.side)
            with side:
                side.used(x, *(pk if cfg.a8 else [qkv]))
                if cfg.a8:
                    O, LSE = ops.attn8_fwd(pk[0], pk[2], pk[5], cfg.sid, cfg.sptr, x.shape[0], cfg.scale, cfg.splits,
                                           cfg.bf16)
                else:
                    O, LSE = ops.attn_fwd(qkv, cfg.sid, cfg.sptr, cfg.heads, cfg.scale, cfg.span, cfg.splits)
                z2 = ops.gf_oproj_fwd(O, Wo, bo, x, acc[l], rng, s1, p, nv)
            if edge_pending:  # join the edge chain (its outputs live on in the main stream)
                emain.wait_stream(estream)
                for t in [e, rbf, drdf, *Rl, *Gl, *Cs]:
                    if t is not None:
                        t.record_stream(emain)
                edge_pending = False
            C = Cs[l] if hoist else ops.gf_edge_fwd(r, e, Wr, Wd, bc)
            Z, amin, amax = ops.pna_fwd(x, AB, C, G, cfg.src.index, cfg.dst.rowptr, cfg.avg[l][0], cfg.avg[l][1])
            pl, z1 = ops.gf_post_fwd(Z, Wpost, bpost, Wlin, blin, x, acc[l], rng, s0, p, nv)
            side.join(O, LSE, z2)
            n1, n2, _, _ = cfg.bns[l]
            rm1, rv1, nb1, m1, e1 = _bn_state(n1)
            rm2, rv2, nb2, m2, e2 = _bn_state(n2)
            out, md, z3 = ops.gf_mlp_fwd(z1, z2, acc[l], saved[l], [g1, b1n, g2, b2n], rm1, rv1, nb1, rm2, rv2, nb2,
                                         m1, e1, m2, e2, W1, b1, W2, b2, rng, s2, s3, p, nv)
            st.append(dict(x=x, AB=AB, qkv=qkv, pk=pk, O=O, LSE=LSE, z2=z2, C=C, Z=Z, amin=amin, amax=amax, p=pl, z1=z1,
                           out=out, md=md, z3=z3, Wab=Wab, Wr=Wr, Wd=Wd))
        _, _, n3, n4 = cfg.bns[L - 1]
        rm3, rv3, nb3, m3, e3 = _bn_state(n3)
        rm4, rv4, nb4, m4, e4 = _bn_state(n4)
        pp = prm[L - 1]
        xL, pooled = ops.gf_final_fwd(z3, acc[L - 1], saved[L - 1], [pp[16], pp[17], pp[18], pp[19]], rm3, rv3, nb3,
                                      rm4, rv4, nb4, m3, e3, m4, e4, nv, cfg.gptr)
        ctx.set_materialize_grads(False)
        ctx.cfg = cfg
        ctx.st = st
        ctx.acc, ctx.saved = acc, saved
        ctx.radial = (rbf, drdf, Rl, Gl)
        ctx.emb = e
        ctx.freq_grad = bool(freq.requires_grad)
        # the parameter objects themselves (gradient slots are keyed by parameter)
        ctx.pobj = (freq, (Wne, Wpe, Wnl, Wee, Wrp, Wel), flat)
        ctx.save_for_backward(xin, pe, eattr, rpe, Wne, Wpe, Wnl, Wee, Wrp, Wel, xL, *flat)
        return xL, pooled

    @staticmethod
    def backward(ctx, dxL, dpool):
        ops = _native.ops()
        cfg = ctx.cfg
        L, F = cfg.L, cfg.F
        xin, pe, eattr, rpe, Wne, Wpe, Wnl, Wee, Wrp, Wel, xL, *flat = ctx.saved_tensors
        prm = [flat[NP * l: NP * (l + 1)] for l in range(L)]
        rbf, drdf, Rl, Gl = ctx.radial
        e = ctx.emb
        K = rbf.shape[1]
        acc, saved, st = ctx.acc, ctx.saved, ctx.st
        nv, rng, p = cfg.nv, cfg.rng, cfg.p
        dev = xin.device
        if dpool is not None and cfg.gptr is None:
            dpool = None
        g = ops.gf_pair_stats_bwd(dxL, xL, st[L - 1]["z3"], saved[L - 1], acc[L - 1], nv, dpool, cfg.gidx, cfg.gptr)
        empty = torch.empty(0, device=dev, dtype=torch.float32)
        dys, xs, dws, dbs = [], [], [], []
        # parameter gradients go straight into the training step's flat-buffer slots when it
        # provides them (parallel/gradslots.py): autograd then hands back the slot views and
        # the step packs nothing
        pfreq, pemb, pflat = ctx.pobj
        ctx.pobj = None
        pobj = [pflat[NP * l: NP * (l + 1)] for l in range(L)]

        def gsl(*ps):
            return _gradslots.slots(list(ps))

        def item(dy, x, W, with_bias, pW=None, pb=None):
            shape = W if isinstance(W, tuple) else W.shape
            sl = gsl(pW, pb) if (pW is not None and pb is not None) else (gsl(pW) if pW is not None else None)
            dW = sl[0] if sl is not None else torch.empty(shape, device=dev, dtype=torch.float32)
            if with_bias:
                db = sl[1] if (sl is not None and pb is not None) else torch.empty(shape[0], device=dev,
                                                                                 dtype=torch.float32)
            else:
                db = None
            dys.append(dy)
            xs.append(x)
            dws.append(dW)
            dbs.append(db if db is not None else empty)
            return dW, db

        grads = [None] * len(flat)
        de = None
        drbf = None
        dx0 = None
        wg = []  # per layer: (dWab, (dWr, dbc), dWd)
        # layer l's weight gradients are launched on a third stream during layer l-1's
        # backward (the last layer's, plus the embeddings', stay on the main stream at the end)
        wside = cfg.side and os.environ.get("HYDRA_WGRAD_OVERLAP", "1") == "1"
        if wside:
            wmain = torch.cuda.current_stream(dev)
            wstream = _streams.side_stream(dev, 2)
        lo = 0
        edge_ev = None
        # HYDRA_EARLY_WGRAD=1: layer 0's ready weight gradients on the edge stream during its
        # attention backward
        # (default off: at layer 0 the local chain is the longer branch, so the early launch
        # could not start before it ended and only split the tail into two launch pairs;
        # measured 0.905-0.914 vs 0.921-0.923 ms/step with it on MI355X)
        early0 = wside and os.environ.get("HYDRA_EARLY_WGRAD", "0") == "1"
        # HYDRA_L0_WGRAD_SIDE=1: layer 0's joined-branch weight gradients on a side stream beside
        # its node backward (see below; off by default: measured 0.912-0.923 vs 0.900-0.913
        # ms/step on MI355X, the fork / join and the shared CUs cost more than the overlap)
        late0 = wside and os.environ.get("HYDRA_GPS_ATTN_MAIN", "0") != "1" and \
            os.environ.get("HYDRA_L0_WGRAD_SIDE", "0") == "1"
        l0_ev = None
        early_done = False
        gw0 = dfreq_w = te = None
        # HYDRA_GPS_ATTN_MAIN=1: the attention branch on the main stream and the local chain on
        # the side stream (measured 0.990 vs 0.917 ms/step on MI355X: the runtime's queue
        # mapping then put the attention beside the weight-gradient launches); default: the
        # attention branch on the side stream
        attn_main = cfg.side and os.environ.get("HYDRA_GPS_ATTN_MAIN", "0") == "1"
        for l in reversed(range(L)):
            s = st[l]
            (Win, bin_, Wo, bo, Wpre, bpre, Wenc, benc, Wpost, bpost, Wlin, blin,
             g1, b1n, g2, b2n, g3, b3n, g4, b4n, W1, b1, W2, b2, Wemb, bemb, Wrl) = prm[l]
            s0, s1, s2, s3 = cfg.salts[l]
            n1, n2, n3, n4 = cfg.bns[l]
            P = pobj[l]
            dg, dpre, dout, dw3, db3, dw4, db4 = ops.gf_mlp_bwd(g, s["z3"], acc[l], saved[l], g3, g4, float(n3.eps),
                                                               float(n4.eps), s["md"], W2, W1, s["z1"], s["z2"], rng,
                                                               s2, s3, p, nv, gsl(P[16], P[17], P[18], P[19]))
            att_ev = [None]

            def attn_branch():
                if cfg.a8 and cfg.splits <= 0:
                    # the attention backward's operands (-delta, dO in the pair / quad layouts)
                    # come out of the output-projection backward's epilogue: no packing launch
                    pk = s["pk"]
                    dz2, da, _, dw2n, db2n, nd, dOp, dOq = ops.gf_att_bwd(dout, s["z2"], acc[l], saved[l], g2, Wo, rng,
                                                                          s1, p, nv, s["O"], gsl(P[14], P[15]))
                    att_ev[0] = torch.cuda.Event()
                    att_ev[0].record()  # da ready (the early weight gradients of layer 0 wait on it)
                    dqkv = ops.attn8_bwd_packed(nd, dOp, dOq, s["LSE"], pk[0], pk[1], pk[2], pk[3], pk[4], cfg.sid,
                                                cfg.sptr, s["x"].shape[0], cfg.scale, cfg.bf16)
                    dO = None
                elif cfg.a8:
                    dz2, da, dO, dw2n, db2n = ops.gf_att_bwd(dout, s["z2"], acc[l], saved[l], g2, Wo, rng, s1, p, nv,
                                                             None, gsl(P[14], P[15]))
                    pk = s["pk"]
                    dqkv = ops.attn8_bwd(dO, s["O"], s["LSE"], pk[0], pk[1], pk[2], pk[3], pk[4], cfg.sid, cfg.sptr,
                                         cfg.scale, cfg.splits)
                else:
                    dz2, da, dO, dw2n, db2n = ops.gf_att_bwd(dout, s["z2"], acc[l], saved[l], g2, Wo, rng, s1, p, nv,
                                                             None, gsl(P[14], P[15]))
                    dqkv = ops.attn_bwd(dO, s["qkv"], s["O"], s["LSE"], cfg.sid, cfg.sptr, cfg.heads, cfg.scale,
                                        cfg.span, cfg.splits)
                return dz2, da, dO, dqkv, dw2n, db2n

            def loc_bwd():
                return ops.gf_loc_bwd(dout, s["z1"], acc[l], saved[l], g1, Wlin, Wpost, rng, s0, p, nv,
                                      gsl(P[12], P[13]))

            def pna_branch():
                dE, dG, dAB = ops.pna_bwd(dZ, s["Z"], s["AB"], s["C"], Gl[l], cfg.src.index, cfg.dst.rowptr,
                                          s["amin"], s["amax"], cfg.avg[l][0], cfg.avg[l][1])
                ops.seg_sum_out(dE, cfg.src.rowptr, cfg.src.perm, dAB[:, F:])
                return dE, dG, dAB

            def wgrad_prev():
                nonlocal lo
                if wside and lo < len(dys):
                    # the previous layer's weight gradients: enqueued here so they run beside this
                    # layer's attention backward (long, matrix-core bound) rather than beside the
                    # short node / MLP / delta kernels that lead into it (the critical path)
                    wstream.wait_stream(wmain)
                    with torch.cuda.stream(wstream):
                        ops.linear_wgrad_grouped(dys[lo:], xs[lo:], dws[lo:], dbs[lo:], [0] * (len(dys) - lo))
                    lo = len(dys)

            def edge_launch(after):
                # dr (masked by the radial ReLU), de += dC Wd, drbf += dr Wemb + dG Wlin: one launch.
                # Nothing of the layer chain reads them (only weight gradients and the embedding /
                # radial backward at the end): with the weight-gradient stream it runs there, off
                # the local branch's critical path.  ``after``: the event of the local chain
                nonlocal de, drbf, edge_ev
                if wside and l > 0:
                    wstream.wait_event(after)
                    with torch.cuda.stream(wstream):
                        dr, de, drbf = ops.gf_edge_bwd(dE, s["Wr"], s["Wd"], Rl[l], de, dG, Wemb, Wrl, drbf, K)
                    edge_ev = torch.cuda.Event()
                    edge_ev.record(wstream)
                elif wside:
                    # the first layer's: the weight-gradient stream is still busy with layer 1's
                    # weight gradients, so a fourth stream runs it beside the attention backward,
                    # behind the previous edge launch (accumulated de / drbf) through an event
                    e3 = _streams.side_stream(dev, 3)
                    e3.wait_event(after)
                    if edge_ev is not None:
                        e3.wait_event(edge_ev)
                    with torch.cuda.stream(e3):
                        dr, de, drbf = ops.gf_edge_bwd(dE, s["Wr"], s["Wd"], Rl[l], de, dG, Wemb, Wrl, drbf, K)
                    edge_ev = torch.cuda.Event()
                    edge_ev.record(e3)
                else:
                    dr, de, drbf = ops.gf_edge_bwd(dE, s["Wr"], s["Wd"], Rl[l], de, dG, Wemb, Wrl, drbf, K)
                return dr

            if attn_main:
                # the attention branch (the long one) stays on the main stream: a hipGraph fork
                # delays the branch it starts and a join the node that waits (~7 us each, see
                # tools/graph_fork_cost.py), so the local chain (loc -> PNA -> dB segment sum,
                # shorter) takes the side stream and its join is ready when attention ends
                loc = _Side(dev, True)
                with loc:
                    loc.used(dout)
                    dz1, dq, dp, dZ, dw1n, db1n = loc_bwd()
                    dE, dG, dAB = pna_branch()
                    lev = torch.cuda.Event()
                    lev.record(loc.side)
                wgrad_prev()
                dz2, da, dO, dqkv, dw2n, db2n = attn_branch()
                if wside:
                    dr = edge_launch(lev)
                loc.join(dz1, dq, dp, dZ, dw1n, db1n, dE, dG, dAB)
                if not wside:
                    dr = edge_launch(None)
            else:
                side = _Side(dev, cfg.side)
                with side:
                    side.used(dout)
                    dz2, da, dO, dqkv, dw2n, db2n = attn_branch()
                dz1, dq, dp, dZ, dw1n, db1n = loc_bwd()
                wgrad_prev()
                dE, dG, dAB = pna_branch()
                mev = None
                if wside:
                    mev = torch.cuda.Event()
                    mev.record(wmain)
                dr = edge_launch(mev)
                if early0 and l == 0 and att_ev[0] is not None:
                    # layer 0's weight gradients whose factors are ready (all but Win's dqkv and the
                    # node embedding's dx0), the edge embeddings' and dfreq: one grouped launch on
                    # the first layer's edge stream, beside the attention backward, instead of on
                    # the main stream after the last node launch (the step's tail)
                    gw0 = {}
                    gw0["Wemb"] = item(dr, rbf, Wemb, True, P[24], P[25])
                    gw0["Wrl"] = item(dG, rbf, Wrl, False, P[26])
                    gw0["Wo"] = item(da, s["O"], Wo, True, P[2], P[3])
                    gw0["Wab"] = item(dAB, s["x"], s["Wab"], False)
                    gw0["Wr"] = item(dE, Rl[l], s["Wr"], True)
                    gw0["Wd"] = item(dE, e, s["Wd"], False)
                    gw0["Wpost"] = item(dp, s["Z"], Wpost, True, P[8], P[9])
                    gw0["Wlin"] = item(dq, s["p"], Wlin, True, P[10], P[11])
                    gw0["W1"] = item(dpre, s["out"], W1, True, P[20], P[21])
                    gw0["W2"] = item(dg, s["md"], W2, True, P[22], P[23])
                    dfreq_w = item(drbf, drdf, (K, K), False)[0] if ctx.freq_grad else None
                    te = [item(de, eattr, (F, eattr.shape[1]), False)[0], item(de, rpe, (F, rpe.shape[1]), False)[0]]
                    e3 = _streams.side_stream(dev, 3)  # holds the layer's edge launch (de / drbf final)
                    e3.wait_event(att_ev[0])
                    with torch.cuda.stream(e3):
                        ops.linear_wgrad_grouped(dys[lo:], xs[lo:], dws[lo:], dbs[lo:], [0] * (len(dys) - lo))
                    lo = len(dys)
                    edge_ev = torch.cuda.Event()
                    edge_ev.record(e3)
                    early_done = True
                # (fanning the dQ and dK/dV passes out onto two more streams measured slower on
                # MI355X: the attention passes are throughput-bound once they overlap the local
                # branch, 209 vs 200 us per layer)
                side.join(dz2, da, dO, dqkv, dw2n, db2n)
            if l == 0 and late0 and not early_done:
                # layer 0's weight gradients whose factors are final once both branches joined
                # (all but the edge embedding's, whose dr comes from the edge launch): one grouped
                # launch on a fifth stream beside the node backward and the layer's edge
                # backward, so the step's tail keeps only the small embedding problems
                gl0 = {}
                gl0["Wrl"] = item(dG, rbf, Wrl, False, P[26])
                gl0["Win"] = item(dqkv, s["x"], Win, True, P[0], P[1])
                gl0["Wo"] = item(da, s["O"], Wo, True, P[2], P[3])
                gl0["Wab"] = item(dAB, s["x"], s["Wab"], False)
                gl0["Wr"] = item(dE, Rl[l], s["Wr"], True)
                gl0["Wd"] = item(dE, e, s["Wd"], False)
                gl0["Wpost"] = item(dp, s["Z"], Wpost, True, P[8], P[9])
                gl0["Wlin"] = item(dq, s["p"], Wlin, True, P[10], P[11])
                gl0["W1"] = item(dpre, s["out"], W1, True, P[20], P[21])
                gl0["W2"] = item(dg, s["md"], W2, True, P[22], P[23])
                s5 = _streams.side_stream(dev, 5)
                s5.wait_stream(wmain)
                with torch.cuda.stream(s5):
                    ops.linear_wgrad_grouped(dys[lo:], xs[lo:], dws[lo:], dbs[lo:], [0] * (len(dys) - lo))
                lo = len(dys)
                l0_ev = torch.cuda.Event()
                l0_ev.record(s5)
            if l > 0:
                sp = st[l - 1]
                g = ops.gf_node_bwd(dAB, dqkv, s["Wab"], Win, dZ, dz1, dz2, s["x"], sp["z3"], saved[l - 1], acc[l - 1],
                                    nv)
            else:
                dx0 = ops.gf_node_bwd(dAB, dqkv, s["Wab"], Win, dZ, dz1, dz2, s["x"], None, None, None, nv)
            base = NP * l
            if early_done and l == 0:
                gw = gw0
                gw["Win"] = item(dqkv, s["x"], Win, True, P[0], P[1])
            elif l0_ev is not None and l == 0:
                gw = gl0
                gw["Wemb"] = item(dr, rbf, Wemb, True, P[24], P[25])
            else:
                gw = {}
                gw["Wemb"] = item(dr, rbf, Wemb, True, P[24], P[25])
                gw["Wrl"] = item(dG, rbf, Wrl, False, P[26])
                gw["Win"] = item(dqkv, s["x"], Win, True, P[0], P[1])
                gw["Wo"] = item(da, s["O"], Wo, True, P[2], P[3])
                gw["Wab"] = item(dAB, s["x"], s["Wab"], False)
                gw["Wr"] = item(dE, Rl[l], s["Wr"], True)
                gw["Wd"] = item(dE, e, s["Wd"], False)
                gw["Wpost"] = item(dp, s["Z"], Wpost, True, P[8], P[9])
                gw["Wlin"] = item(dq, s["p"], Wlin, True, P[10], P[11])
                gw["W1"] = item(dpre, s["out"], W1, True, P[20], P[21])
                gw["W2"] = item(dg, s["md"], W2, True, P[22], P[23])
            wg.append((l, gw))
            grads[base + 12], grads[base + 13] = dw1n, db1n
            grads[base + 14], grads[base + 15] = dw2n, db2n
            grads[base + 16], grads[base + 17] = dw3, db3
            grads[base + 18], grads[base + 19] = dw4, db4
        if wside:
            # the edge backward's outputs (and the overlapped weight gradients) join the main stream
            wmain.wait_stream(wstream)
            if l0_ev is not None:
                wmain.wait_event(l0_ev)
            if edge_ev is not None:
                wmain.wait_event(edge_ev)
            for t in (dr, de, drbf):
                if t is not None:
                    t.record_stream(wmain)
        if not early_done:
            dfreq_w = item(drbf, drdf, (K, K), False)[0] if ctx.freq_grad else None
        # embeddings: only the narrow products dy^T [A | B] (see csrc/gps_fused.hip, EmbFwd)
        tn = [item(dx0, xin, (F, xin.shape[1]), False)[0], item(dx0, pe, (F, pe.shape[1]), False)[0]]
        if not early_done:
            te = [item(de, eattr, (F, eattr.shape[1]), False)[0], item(de, rpe, (F, rpe.shape[1]), False)[0]]
        # every weight gradient of the stack (incl. the radial basis and its frequencies): one
        # grouped launch pair
        ops.linear_wgrad_grouped(dys[lo:], xs[lo:], dws[lo:], dbs[lo:], [0] * (len(dys) - lo))
        # weight-prep backward of every layer, embedding weights and dfreq: one launch
        wp, fp = [], []
        for l, gw in wg:
            wp += [gw["Wab"][0], gw["Wr"][0], gw["Wd"][0], gw["Wr"][1], prm[l][4], prm[l][6], prm[l][7]]
            fp += list(pobj[l][4:8])  # dWpre, dbpre, dWenc, dbenc
        fp += list(pemb) + ([pfreq] if dfreq_w is not None else [])
        fin = ops.gf_finish(wp, [tn[0], tn[1], Wne, Wpe, Wnl, te[0], te[1], Wee, Wrp, Wel], dfreq_w,
                            _gradslots.slots(fp))
        dfreq = fin[4 * L + 6] if dfreq_w is not None else None
        emb_g = fin[4 * L: 4 * L + 6]  # node dWa, dWb, dWl, edge dWa, dWb, dWl
        for k, (l, gw) in enumerate(wg):
            base = NP * l
            grads[base + 24], grads[base + 25] = gw["Wemb"]
            grads[base + 26] = gw["Wrl"][0]
            grads[base + 0], grads[base + 1] = gw["Win"]
            grads[base + 2], grads[base + 3] = gw["Wo"]
            grads[base + 4], grads[base + 5], grads[base + 6], grads[base + 7] = fin[4 * k: 4 * k + 4]
            grads[base + 8], grads[base + 9] = gw["Wpost"]
            grads[base + 10], grads[base + 11] = gw["Wlin"]
            grads[base + 20], grads[base + 21] = gw["W1"]
            grads[base + 22], grads[base + 23] = gw["W2"]
        ctx.st = None
        ctx.radial = None
        ctx.emb = None
        return (None, None, dfreq, None, None, None, None, *emb_g, *grads)
