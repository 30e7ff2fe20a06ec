"""bf16 MFMA path for wide EGNN encoders (the SC25 EGNN-866 GFM; reference
``hydragnn/models/EGCLStack.py:175-289`` E_GCL + ``Base.py:466`` activation).

One autograd function runs the whole E_GCL stack.  Per layer (H = hidden, Hp = H padded
to 128 with the ones lane at column H, F = input width, Kx = pad128(F)):

  forward  AB   = x [Wa;Wb]^T                    NT  [N, Kx] x [2Hp, Kx]    fp32 out
           h1   = relu(AB[src] + AB[dst] + ...)   egnn_gather_fwd            bf16 [E, Hp]
           m    = relu(h1 W2^T + b2)              NT  (edge GEMM)            bf16 [E, Hp]
           c1   = relu(m Wc1^T + bc1), s = c1 wc2 NT + row-dot epilogue     (equivariant)
           agg, pos' = CSR-by-source sums          egnn_csr_rows / egnn_pos_fwd
           n1   = relu([x | agg] Wn1^T + bn1)     NT, K-concatenated A       bf16 [N, Hp]
           x'   = relu(n1 Wn2^T + bn2)            NT                         bf16 (+fp32 last)
  backward the dual chain: relu'-gated casts, NT data gradients with gather-add and
           relu' epilogues, TN split-row weight gradients (bias gradients from the ones
           lane), coordinate / position kernels (egnn.hip).

Every weight is imaged to padded bf16 (and transposed) in ONE batched launch per forward;
all activations between GEMMs are padded bf16 (fp32 accumulation everywhere).  Eligible:
GPU, ``precision("bf16")``, ReLU convs without attention / recurrence / checkpointing.
"""
import torch

from .. import _native
from ..parallel import gradslots as _gradslots
from . import bgemm as bg


ENABLED = True  # module switch (tests compare against the module-by-module bf16 path)
DEBUG = None  # dict: backward records the position gradient entering each layer (tests)


def eligible(model, ctx):
    from ..models.egnn import E_GCL
    from .linear import get_precision
    from .pna import fused

    if not ENABLED or get_precision() != "bf16" or not fused("egnn") or model.use_global_attn or model.conv_checkpointing:
        return False
    if not isinstance(model.activation_function, torch.nn.ReLU):
        return False
    data = ctx.data
    if data.x is None or not data.x.is_cuda or ctx.src_si is None or ctx.dst_si is None:
        return False
    if ctx.dst_si.perm is not None:  # edges must be stored sorted by destination
        return False
    ea = ctx.get("edge_attr")
    if ea is not None and (ea.dim() != 2 or ea.shape[1] > 3):
        return False
    for conv, fl in zip(model.graph_convs, model.feature_layers):
        if not isinstance(conv, E_GCL) or not isinstance(fl, torch.nn.Identity):
            return False
        if conv.attention or conv.recurrent or not isinstance(conv.act_fn, torch.nn.ReLU) or not conv.norm_diff:
            return False
        if conv.equivariant and not conv.tanh:
            return False
        if conv.edge_mlp[0].out_features < 128:
            return False
    return True


def _layer_params(conv):
    ps = [conv.edge_mlp[0].weight, conv.edge_mlp[0].bias, conv.edge_mlp[2].weight, conv.edge_mlp[2].bias,
          conv.node_mlp[0].weight, conv.node_mlp[0].bias, conv.node_mlp[2].weight, conv.node_mlp[2].bias]
    if conv.equivariant:
        ps += [conv.coord_mlp[0].weight, conv.coord_mlp[0].bias, conv.coord_mlp[2].weight]
    return ps


class _Plan:
    def __init__(self, model, ctx, ea):
        self.convs = list(model.graph_convs)
        self.src, self.dst = ctx.src_si, ctx.dst_si
        self.nea = 0 if ea is None else ea.shape[1]
        self.layers = []
        for conv in self.convs:
            H = conv.edge_mlp[0].out_features
            F = conv.input_channels
            self.layers.append(dict(F=F, H=H, Hp=bg.pad128(H), Kx=bg.pad128(F), Ho=conv.node_mlp[2].out_features,
                                    eq=conv.equivariant, cw=float(conv.coords_weight),
                                    np=len(_layer_params(conv))))


def _images(plan, params, dev):
    """Padded bf16 images (and transposes) of every layer's GEMM weights, one launch."""
    srcs, d, dt, imgs = [], [], [], []
    e = torch.empty(0, device=dev, dtype=torch.bfloat16)

    def job(src, dst, dstT):
        srcs.append(src)
        d.append(dst)
        dt.append(dstT)

    off = 0
    for L in plan.layers:
        F, H, Hp, Kx, Ho = L["F"], L["H"], L["Hp"], L["Kx"], L["Ho"]
        Hop = bg.pad128(Ho)
        p = params[off:off + L["np"]]
        off += L["np"]
        W0, W2, Wn1, Wn2 = p[0], p[2], p[4], p[6]
        im = {}
        im["ab"] = torch.empty((2 * Hp, Kx), device=dev, dtype=torch.bfloat16)
        im["abT"] = torch.empty((Kx, 2 * Hp), device=dev, dtype=torch.bfloat16)
        job(W0[:, :F], im["ab"][:Hp], im["abT"][:, :Hp])
        job(W0[:, F:2 * F], im["ab"][Hp:], im["abT"][:, Hp:])
        im["w2"] = torch.empty((Hp, Hp), device=dev, dtype=torch.bfloat16)
        im["w2T"] = torch.empty((Hp, Hp), device=dev, dtype=torch.bfloat16)
        job(W2, im["w2"], im["w2T"])
        im["n1"] = torch.empty((Hp, Kx + Hp), device=dev, dtype=torch.bfloat16)
        im["n1T"] = torch.empty((Kx + Hp, Hp), device=dev, dtype=torch.bfloat16)
        job(Wn1[:, :F], im["n1"][:, :Kx], im["n1T"][:Kx])
        job(Wn1[:, F:], im["n1"][:, Kx:], im["n1T"][Kx:])
        im["n2"] = torch.empty((Hop, Hp), device=dev, dtype=torch.bfloat16)
        im["n2T"] = torch.empty((Hp, Hop), device=dev, dtype=torch.bfloat16)
        job(Wn2, im["n2"], im["n2T"])
        if L["eq"]:
            Wc1 = p[8]
            im["c1"] = torch.empty((Hp, Hp), device=dev, dtype=torch.bfloat16)
            im["c1T"] = torch.empty((Hp, Hp), device=dev, dtype=torch.bfloat16)
            job(Wc1, im["c1"], im["c1T"])
        imgs.append(im)
    _native.ops().bg_cast_weights(srcs, [x if x.numel() else e for x in d], [x if x.numel() else e for x in dt])
    return imgs


class _EGNNWide(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, x, pos, ea, *params):
        ops = _native.ops()
        dev = x.device
        N, E = x.shape[0], plan.src.index.numel()
        src, dst = plan.src, plan.dst
        imgs = _images(plan, params, dev)
        xb = bg.cast_pad(x, plan.layers[0]["Kx"])
        pos_l = pos.contiguous().float()
        saved = []
        off = 0
        x_out = None
        for li, L in enumerate(plan.layers):
            F, H, Hp, Kx, Ho = L["F"], L["H"], L["Hp"], L["Kx"], L["Ho"]
            p = params[off:off + L["np"]]
            off += L["np"]
            im = imgs[li]
            AB = torch.empty((N, 2 * Hp), device=dev, dtype=torch.float32)
            bg.nt(xb, im["ab"], Kx, 2 * Hp, outf=AB)
            h1 = torch.empty((E, Hp), device=dev, dtype=torch.bfloat16)
            geo = torch.empty((E, 4), device=dev, dtype=torch.float32)
            sc = torch.empty((E, 128), device=dev, dtype=torch.bfloat16)
            ops.egnn_gather_fwd(AB, src.index, dst.index, pos_l, ea, p[0], 2 * F, p[1], h1, geo, sc)
            del AB
            m = torch.empty((E, Hp), device=dev, dtype=torch.bfloat16)
            bg.nt(h1, im["w2"], Hp, H, bias=p[3], act=1, outb=m, ones_col=H)
            s = c1 = None
            if L["eq"]:
                s = torch.zeros(E, device=dev, dtype=torch.float32)
                c1 = torch.empty((E, Hp), device=dev, dtype=torch.bfloat16)
                bg.nt(m, im["c1"], Hp, H, bias=p[9], act=1, outb=c1, rowvec=p[10].reshape(-1), rowdot=s)
            agg = torch.empty((N, Hp), device=dev, dtype=torch.bfloat16)
            pos_n = torch.empty_like(pos_l) if L["eq"] else pos_l
            ops.egnn_csr_rows(m, src.rowptr, src.perm, 0, None, None, 0, agg)
            if L["eq"]:
                ops.egnn_pos_fwd(pos_l, geo, s, src.rowptr, src.perm, L["cw"], pos_n)
            n1 = torch.empty((N, Hp), device=dev, dtype=torch.bfloat16)
            bg.nt(xb, im["n1"], Kx + Hp, H, A2=agg, k1=Kx, bias=p[5], act=1, outb=n1, ones_col=H)
            last = li == len(plan.layers) - 1
            xn = torch.empty((N, bg.pad128(Ho)), device=dev, dtype=torch.bfloat16)
            if last:
                x_out = torch.empty((N, Ho), device=dev, dtype=torch.float32)
            bg.nt(n1, im["n2"], Hp, Ho, bias=p[7], act=1, outb=xn, ones_col=Ho, outf=x_out)
            saved.append(dict(xb=xb, h1=h1, geo=geo, sc=sc, m=m, s=s, c1=c1, agg=agg, n1=n1, xn=xn))
            if DEBUG is not None:
                DEBUG[("s", li)], DEBUG[("geo", li)] = s, geo
            xb, pos_l = xn, pos_n
        ctx.plan, ctx.imgs, ctx.saved, ctx.params = plan, imgs, saved, params
        ctx.mark_non_differentiable(pos_l)
        return x_out, pos_l

    @staticmethod
    def backward(ctx, dx_out, dpos_out):
        ops = _native.ops()
        plan, imgs, saved, params = ctx.plan, ctx.imgs, ctx.saved, ctx.params
        dev = dx_out.device
        src, dst = plan.src, plan.dst
        E = src.index.numel()
        N = dx_out.shape[0]
        grads = [None] * len(params)
        offs, o = [], 0
        for L in plan.layers:
            offs.append(o)
            o += L["np"]
        dx = dx_out.contiguous()
        dpos = None  # the decoder does not read the equivariant state (positions)
        for li in range(len(plan.layers) - 1, -1, -1):
            L, im, S = plan.layers[li], imgs[li], saved[li]
            F, H, Hp, Kx, Ho = L["F"], L["H"], L["Hp"], L["Kx"], L["Ho"]
            Hop = bg.pad128(Ho)
            p = params[offs[li]:offs[li] + L["np"]]
            # gradient slots of the step's flat buffer (parallel/gradslots.py): the layer's
            # weight gradients are written there and handed to the bucketed all-reduce as soon
            # as the layer is done, so the buckets of the last layers reduce while the earlier
            # layers' backward still runs (returned through autograd they all arrived at the end)
            sl = _gradslots.slots(p) if all(isinstance(t, torch.nn.Parameter) for t in p) else None
            g = list(sl) if sl is not None else [torch.empty_like(t) for t in p]
            given = set()

            def give(*ks, p=p, sl=sl, given=given):
                # hand finished slot gradients to the bucketed all-reduce, sub-block by
                # sub-block as the layer's backward produces them
                if sl is None:
                    return
                ks = [k for k in ks if k < len(p) and k not in given]
                given.update(ks)
                if ks:
                    _gradslots.provide([p[k] for k in ks])
            # node MLP
            dn2 = bg.cast_pad(dx, Hop, gate=S["xn"], ones=False)
            bg.wgrad(dn2, S["n1"], Hop, Hp, [(g[6], 0, g[7], H)])
            give(6, 7)
            dn1 = torch.empty((N, Hp), device=dev, dtype=torch.bfloat16)
            bg.nt(dn2, im["n2T"], Hop, H, gate=S["n1"], outb=dn1)
            bg.wgrad(dn1, S["xb"], Hp, Kx + Hp, [(g[4][:, :F], 0, g[5], F), (g[4][:, F:], 0, None, -1, Kx)],
                     X2=S["agg"], kc1=Kx)
            give(4, 5)
            dxa = torch.empty((N, Kx + Hp), device=dev, dtype=torch.float32)
            bg.nt(dn1, im["n1T"], Hp, Kx + Hp, outf=dxa)
            dagg = dxa[:, Kx:Kx + H]
            # coordinate MLP + edge MLP second layer
            dZ2 = torch.empty((E, Hp), device=dev, dtype=torch.bfloat16)
            dcd = None
            if L["eq"]:
                dpo = dpos if dpos is not None else torch.zeros((N, 3), device=dev, dtype=torch.float32)
                dc1 = torch.empty((E, Hp), device=dev, dtype=torch.bfloat16)
                dcd = torch.empty((E, 3), device=dev, dtype=torch.float32)
                part = torch.empty(((E + 31) // 32) * Hp, device=dev, dtype=torch.float32)
                nblk = ops.egnn_coord_bwd(dpo, src.index, src.rowptr, S["geo"], S["s"], S["c1"],
                                          p[10].reshape(-1), L["cw"], dc1, dcd, part)
                ops.bg_slab_reduce(part, nblk, 1, Hp, 0, 0, 1, H, g[10], 0.0, -1, None)
                bg.wgrad(dc1, S["m"], Hp, Hp, [(g[8], 0, g[9], H)])
                give(8, 9, 10)
                bg.nt(dc1, im["c1T"], Hp, H, addg=dagg, addg_idx=src.index, gate=S["m"], outb=dZ2)
                if DEBUG is not None:
                    DEBUG[("dc1", li)] = dc1
                del dc1
            else:
                ops.egnn_gather_gate(dagg, src.index, S["m"], H, dZ2)
            bg.wgrad(dZ2, S["h1"], Hp, Hp, [(g[2], 0, g[3], H)])
            give(2, 3)
            dh1 = torch.empty((E, Hp), device=dev, dtype=torch.bfloat16)
            dr = None  # d loss / d|d_e| (the radial input of edge_mlp[0]), from the fp32 epilogue
            if li > 0:
                dr = torch.zeros(E, device=dev, dtype=torch.float32)
                bg.nt(dZ2, im["w2T"], Hp, H, gate=S["h1"], outb=dh1, rowvec=p[0][:, 2 * F].contiguous(), rowdot=dr)
            else:
                bg.nt(dZ2, im["w2T"], Hp, H, gate=S["h1"], outb=dh1)
            del dZ2
            # edge MLP first layer: node-level blocks are by-source / by-destination CSR sums
            dAB = torch.empty((N, 2 * Hp), device=dev, dtype=torch.bfloat16)
            ops.egnn_csr_rows(dh1, src.rowptr, src.perm, 0, dst.rowptr, None, Hp, dAB)
            ns = plan.nea + 1
            bg.wgrad(dh1, S["sc"], Hp, 128, [(g[0][:, 2 * F:2 * F + ns], 0, g[1], ns)])
            del dh1
            bg.wgrad(dAB, S["xb"], 2 * Hp, Kx, [(g[0][:, :F], 0, None, -1), (g[0][:, F:2 * F], Hp, None, -1)])
            give(0, 1)
            if li > 0:  # the input features and positions are data
                dx = dxa[:, :F]
                bg.nt(dAB, im["abT"], 2 * Hp, F, outf=dx, beta=1.0)
                dpos_in = torch.empty((N, 3), device=dev, dtype=torch.float32)
                ops.egnn_pos_bwd(dpos, S["geo"], dr, dcd, src.rowptr, src.perm, dst.rowptr, dpos_in)
                dpos = dpos_in
                if DEBUG is not None:
                    DEBUG[li] = dpos_in.clone()
            if sl is not None:
                give(*range(len(p)))  # anything not handed over above
            else:
                for j in range(L["np"]):
                    grads[offs[li] + j] = g[j]
        ctx.saved = ctx.imgs = None
        return (None, None, None, None, *grads)


def encode(model, ctx):
    """Run the stack; returns (x [N, H] fp32, pos')."""
    data = ctx.data
    ea = ctx.get("edge_attr")
    if ea is not None:
        ea = ea.float().contiguous()
    plan = _Plan(model, ctx, ea)
    params = []
    for conv in plan.convs:
        params += _layer_params(conv)
    x = data.x.float()
    return _EGNNWide.apply(plan, x, data.pos, ea, *params)
