"""Native twice-differentiable PAINN (reference ``hydragnn/models/PAINNStack.py:194-319``)
for force training (``Base.energy_force_loss``, ``Base.py:582-636``).

A force step differentiates the energy twice: forces = -dE/dpos with ``create_graph``, then
the loss gradient w.r.t. the parameters through that backward graph.  Op by op (the torch
composite) a PAINN step is ~1,300 launches.  Here the model is three op families, each a
closed set of native ops with explicit first AND second derivatives:

* ``EdgeGeom``: pos -> per-edge basis [sinc(n pi d / c)/d * cut(d) | cut(d)] and d̂/d
  (``PAINNStack.py:228-236``; the reference's d̂/d quirk kept).  Backward: one node-parallel
  pass over both CSR views (incoming edges add, outgoing subtract); its backward: the
  per-edge Jacobian-vector product plus the second-derivative term w.r.t. pos.
* ``Msg``: the PAINN message + CSR-by-source segment sums, residual included
  (``PAINNStack.py:194-263``): W_e = [W_f | b_f] basis_e, o = W_e * phi[dst], s += sum o_s,
  v += sum v[dst] o_v + o_e d̂/d.  Backward: one dst-CSR pass; its backward (the VJP's VJP,
  derived in ``_msg_vvjp``): one src-CSR pass + one dst-CSR pass.
* node chains (``ops.rowprog``): update + adapters + activation/mask + the next layer's
  scalar-message MLP as ONE row program per layer; first and second derivative programs
  are generated from it (dual + reverse).

In the force pass (``input_grads_only``) the first backward skips the weight-gradient
work: forces need only input gradients, and the parameter gradients come from the second
backward.  Weight-gradient outputs of the first-order backward ops are marked
non-differentiable (a third derivative through them is not supported).

CPU: every op runs its torch twin (the same formulas as the kernels, vectorised);
``tests/test_painn_force.py`` checks them with fp64 ``gradcheck`` / ``gradgradcheck``.
"""
import contextlib
import math

import torch

from . import rowprog as rp

_state = {"inputs_only": False}


@contextlib.contextmanager
def input_grads_only(enabled=True):
    """First backward of a force step: input gradients only (no weight gradients)."""
    prev = _state["inputs_only"]
    _state["inputs_only"] = enabled
    try:
        yield
    finally:
        _state["inputs_only"] = prev


def _scatter(n, idx, val):
    out = torch.zeros((n,) + tuple(val.shape[1:]), dtype=val.dtype, device=val.device)
    return out.index_add_(0, idx, val)


# ============================================================================ edge geometry
def _radial(L, R, a, cutoff, eps):
    """f [E, R+1], f' and f'' w.r.t. L; q, q', q'' of q(L) = 1 / ((L + eps) L)."""
    inside = (L < cutoff).to(L.dtype)
    k = torch.arange(1, R + 1, device=L.device, dtype=L.dtype) * a
    Lc = L.unsqueeze(1)
    sn, cs = torch.sin(k * Lc), torch.cos(k * Lc)
    g = sn / Lc
    g1 = k * cs / Lc - sn / Lc ** 2
    g2 = -k * k * sn / Lc - 2 * k * cs / Lc ** 2 + 2 * sn / Lc ** 3
    cut = 0.5 * (torch.cos(a * L) + 1) * inside
    cut1 = -0.5 * a * torch.sin(a * L) * inside
    cut2 = -0.5 * a * a * torch.cos(a * L) * inside
    c0, c1, c2 = cut.unsqueeze(1), cut1.unsqueeze(1), cut2.unsqueeze(1)
    f = torch.cat([g * c0, c0], 1)
    f1 = torch.cat([g1 * c0 + g * c1, c1], 1)
    f2 = torch.cat([g2 * c0 + 2 * g1 * c1 + g * c2, c2], 1)
    D = L * L + eps * L
    q = 1.0 / D
    dD = 2 * L + eps
    q1 = -dD / D ** 2
    q2 = (-2 * D + 2 * dD * dD) / D ** 3
    return f, f1, f2, q, q1, q2


def _geom_vec(pos, dst, src, shifts):
    vec = pos[dst] - pos[src]
    if shifts is not None:
        vec = vec + shifts
    return vec


class _GeomCfg:
    __slots__ = ("R", "a", "cutoff", "eps", "dst", "src", "N", "dst_si", "src_si", "shifts")

    def csr_args(self):
        d, s_ = self.dst_si, self.src_si
        return (d.index, s_.index, d.rowptr, d.perm, s_.rowptr, s_.perm)


def _geom_fwd(cfg, pos):
    vec = _geom_vec(pos, cfg.dst, cfg.src, cfg.shifts)
    L = vec.norm(dim=1)
    f, _, _, q, _, _ = _radial(L, cfg.R, cfg.a, cfg.cutoff, cfg.eps)
    return f, vec * q.unsqueeze(1)


def _geom_vjp(cfg, pos, gB, gU):
    vec = _geom_vec(pos, cfg.dst, cfg.src, cfg.shifts)
    L = vec.norm(dim=1)
    f, f1, _, q, q1, _ = _radial(L, cfg.R, cfg.a, cfg.cutoff, cfg.eps)
    A = (gB * f1).sum(1)
    u = (gU * vec).sum(1)
    gv = ((A + u * q1) / L).unsqueeze(1) * vec + gU * q.unsqueeze(1)
    return _scatter(cfg.N, cfg.dst, gv) - _scatter(cfg.N, cfg.src, gv)


def _geom_vvjp(cfg, pos, gB, gU, hpos, need_g, need_pos):
    """Backward of _geom_vjp: (grad gB, grad gU, grad pos) for the upstream hpos."""
    vec = _geom_vec(pos, cfg.dst, cfg.src, cfg.shifts)
    L = vec.norm(dim=1)
    f, f1, f2, q, q1, q2 = _radial(L, cfg.R, cfg.a, cfg.cutoff, cfg.eps)
    hv = hpos[cfg.dst] - hpos[cfg.src]
    t = (vec * hv).sum(1)
    hB = hU = gp = None
    if need_g:
        hB = f1 * (t / L).unsqueeze(1)
        hU = hv * q.unsqueeze(1) + vec * (q1 * t / L).unsqueeze(1)
    if need_pos:
        A = (gB * f1).sum(1)
        A1 = (gB * f2).sum(1)
        u = (gU * vec).sum(1)
        w = (gU * hv).sum(1)
        c_vec = (A1 + u * q2) * t / L ** 2 - (A + u * q1) * t / L ** 3 + q1 * w / L
        gvec = c_vec.unsqueeze(1) * vec + (q1 * t / L).unsqueeze(1) * gU + ((A + u * q1) / L).unsqueeze(1) * hv
        gp = _scatter(cfg.N, cfg.dst, gvec) - _scatter(cfg.N, cfg.src, gvec)
    return hB, hU, gp


def _ops():
    from .. import _native

    return _native.ops()


def _c(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


class _Geom(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pos, cfg):
        ctx.cfg = cfg
        ctx.save_for_backward(pos)
        if _device(pos):
            d, s_ = cfg.csr_args()[:2]
            B, U = _ops().painn_geom_fwd(_c(pos), _c(cfg.shifts), d, s_, cfg.R, cfg.a, cfg.cutoff, cfg.eps)
            return B, U
        return _geom_fwd(cfg, pos)

    @staticmethod
    def backward(ctx, gB, gU):
        (pos,) = ctx.saved_tensors
        E = ctx.cfg.dst.numel()
        if gB is None:
            gB = torch.zeros(E, ctx.cfg.R + 1, dtype=pos.dtype, device=pos.device)
        if gU is None:
            gU = torch.zeros(E, 3, dtype=pos.dtype, device=pos.device)
        return _GeomBwd.apply(gB, gU, pos, ctx.cfg), None


class _GeomBwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gB, gU, pos, cfg):
        ctx.cfg = cfg
        ctx.save_for_backward(gB, gU, pos)
        if _device(pos):
            return _ops().painn_geom_vjp(_c(pos), _c(cfg.shifts), *cfg.csr_args(), _c(gB), _c(gU), cfg.R, cfg.a,
                                         cfg.cutoff, cfg.eps)
        return _geom_vjp(cfg, pos, gB, gU)

    @staticmethod
    def backward(ctx, hpos):
        gB, gU, pos = ctx.saved_tensors
        cfg = ctx.cfg
        need_g = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        need_pos = ctx.needs_input_grad[2]
        if _device(pos):
            hB, hU, gp = _ops().painn_geom_vvjp(_c(pos), _c(cfg.shifts), *cfg.csr_args(), _c(gB), _c(gU), _c(hpos),
                                                cfg.R, cfg.a, cfg.cutoff, cfg.eps, need_g, need_pos)
            return (hB if need_g else None), (hU if need_g else None), (gp if need_pos else None), None
        hB, hU, gp = _geom_vvjp(cfg, pos, gB, gU, hpos, need_g, need_pos)
        return hB, hU, gp, None


def edge_geometry(pos, dst_si, src_si, num_radial, cutoff, shifts=None, eps=1e-9):
    """(basis [E, R+1] = [sinc_n(d) * cut(d) | cut(d)], d̂ / d [E, 3]) for PAINN."""
    cfg = _GeomCfg()
    cfg.R, cfg.a, cfg.cutoff, cfg.eps = int(num_radial), math.pi / float(cutoff), float(cutoff), float(eps)
    cfg.dst, cfg.src = dst_si.index64, src_si.index64
    cfg.dst_si, cfg.src_si = dst_si, src_si
    cfg.N = pos.shape[0]
    cfg.shifts = shifts
    return _Geom.apply(pos, cfg)


# ============================================================================ message
class _MsgCfg:
    __slots__ = ("dst", "src", "N", "F", "R", "dst_si", "src_si")

    def csr_args(self):
        d, s_ = self.dst_si, self.src_si
        return (d.index, s_.index, d.rowptr, d.perm, s_.rowptr, s_.perm)


def _msg_w(Bas, W, b):
    R = W.shape[1]
    return Bas[:, :R] @ W.t() + Bas[:, R:R + 1] * b.view(1, -1)


def _msg_fwd(cfg, s, v, phi, Bas, Un, W, b):
    F = cfg.F
    w = _msg_w(Bas, W, b)
    o = w * phi[cfg.dst]
    ov, oe, os_ = o[:, :F], o[:, F:2 * F], o[:, 2 * F:]
    mv = v[cfg.dst] * ov.unsqueeze(1) + oe.unsqueeze(1) * Un.unsqueeze(2)
    return s + _scatter(cfg.N, cfg.src, os_), v + _scatter(cfg.N, cfg.src, mv)


def _msg_vjp(cfg, Gs, Gv, v, phi, Bas, Un, W, b, need_w):
    """-> (g_v total, g_phi, g_Bas, g_Un, g_W, g_b); g_s = Gs (identity, returned by the caller)."""
    F, R = cfg.F, cfg.R
    dst, src = cfg.dst, cfg.src
    w = _msg_w(Bas, W, b)
    P = phi[dst]
    o = w * P
    Gs_e, Gv_e = Gs[src], Gv[src]
    Vj = v[dst]
    go = torch.cat([(Gv_e * Vj).sum(1), (Gv_e * Un.unsqueeze(2)).sum(1), Gs_e], 1)
    g_phi = _scatter(cfg.N, dst, go * w)
    g_v = Gv + _scatter(cfg.N, dst, Gv_e * o[:, :F].unsqueeze(1))
    gw = go * P
    g_Bas = torch.cat([gw @ W, (gw * b.view(1, -1)).sum(1, keepdim=True)], 1)
    g_Un = (Gv_e * o[:, F:2 * F].unsqueeze(1)).sum(2)
    g_W = g_b = None
    if need_w:
        g_W = gw.t() @ Bas[:, :R]
        g_b = (gw * Bas[:, R:R + 1]).sum(0)
    return g_v, g_phi, g_Bas, g_Un, g_W, g_b


def _msg_vvjp(cfg, Gs, Gv, v, phi, Bas, Un, W, b, Hv, Hphi, HBas, HUn, HW, Hb, need):
    """Backward of _msg_vjp for the upstream (Hv, Hphi, HBas, HUn, HW, Hb) (None = zero).
    need: flags for (Gs, Gv, v, phi, Bas, Un, W, b).  Derivation: with a = [sum_c Gv_c Hv[dst]_c,
    sum_c Gv_c HUn_c, 0], bb = [sum_c Gv_c v[dst]_c, sum_c Gv_c Un_c, Gs] (bb = the VJP's go),
    w' = W HBas + HW Bas and o' = w' P + w HP, the VJP's contraction with the upstream is
    Hv.Gv + sum_e a.o + bb.o'; its gradients are taken term by term."""
    F, R = cfg.F, cfg.R
    dst, src = cfg.dst, cfg.src
    E = Bas.shape[0]
    z3 = lambda: torch.zeros(E, 3 * F, dtype=Bas.dtype, device=Bas.device)  # noqa: E731
    w = _msg_w(Bas, W, b)
    P = phi[dst]
    HP = Hphi[dst] if Hphi is not None else None
    o = w * P
    wp = _msg_w(HBas, W, b) if HBas is not None else z3()
    if HW is not None or Hb is not None:
        wp = wp + _msg_w(Bas, HW if HW is not None else torch.zeros_like(W), Hb if Hb is not None else torch.zeros_like(b))
    op = wp * P + (w * HP if HP is not None else 0)
    Gs_e, Gv_e = Gs[src], Gv[src]
    Vj = v[dst]
    HVj = Hv[dst] if Hv is not None else None
    out = [None] * 8
    # (1) gradients w.r.t. the VJP's upstream (Gs, Gv): J applied to the tangent
    if need[0]:
        out[0] = _scatter(cfg.N, src, op[:, 2 * F:])
    if need[1]:
        t = Vj * op[:, :F].unsqueeze(1) + op[:, F:2 * F].unsqueeze(1) * Un.unsqueeze(2)
        if HVj is not None:
            t = t + HVj * o[:, :F].unsqueeze(1)
        if HUn is not None:
            t = t + o[:, F:2 * F].unsqueeze(1) * HUn.unsqueeze(2)
        gGv = _scatter(cfg.N, src, t)
        out[1] = gGv + Hv if Hv is not None else gGv
    # (2) second-order terms
    a = torch.cat([(Gv_e * HVj).sum(1) if HVj is not None else torch.zeros_like(Gs_e),
                   (Gv_e * HUn.unsqueeze(2)).sum(1) if HUn is not None else torch.zeros_like(Gs_e),
                   torch.zeros_like(Gs_e)], 1)
    bb = torch.cat([(Gv_e * Vj).sum(1), (Gv_e * Un.unsqueeze(2)).sum(1), Gs_e], 1)
    if need[2]:
        out[2] = _scatter(cfg.N, dst, Gv_e * op[:, :F].unsqueeze(1))
    if need[3]:
        out[3] = _scatter(cfg.N, dst, a * w + bb * wp)
    gw2 = a * P + (bb * HP if HP is not None else 0)
    bP = bb * P
    if need[4]:
        gB = torch.cat([gw2 @ W, (gw2 * b.view(1, -1)).sum(1, keepdim=True)], 1)
        if HW is not None:
            gB[:, :R] += bP @ HW
        if Hb is not None:
            gB[:, R] += (bP * Hb.view(1, -1)).sum(1)
        out[4] = gB
    if need[5]:
        out[5] = (Gv_e * op[:, F:2 * F].unsqueeze(1)).sum(2)
    if need[6] or need[7]:
        gW = gw2.t() @ Bas[:, :R]
        gb = (gw2 * Bas[:, R:R + 1]).sum(0)
        if HBas is not None:
            gW = gW + bP.t() @ HBas[:, :R]
            gb = gb + (bP * HBas[:, R:R + 1]).sum(0)
        out[6], out[7] = gW, gb
    return out


class _Msg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, v, phi, Bas, Un, W, b, cfg):
        ctx.cfg = cfg
        ctx.save_for_backward(v, phi, Bas, Un, W, b)
        if _device(s):
            s1, v1 = _ops().painn_msg_fwd(_c(s), _c(v), _c(phi), _c(Bas), _c(Un), _c(W), _c(b), *cfg.csr_args())
            return s1, v1
        return _msg_fwd(cfg, s, v, phi, Bas, Un, W, b)

    @staticmethod
    def backward(ctx, Gs, Gv):
        v, phi, Bas, Un, W, b = ctx.saved_tensors
        if Gs is None:
            Gs = torch.zeros_like(phi[:, :ctx.cfg.F])
        if Gv is None:
            Gv = torch.zeros_like(v)
        need_w = not _state["inputs_only"] and (ctx.needs_input_grad[5] or ctx.needs_input_grad[6])
        g_v, g_phi, g_Bas, g_Un, g_W, g_b = _MsgBwd.apply(Gs, Gv, v, phi, Bas, Un, W, b, ctx.cfg, need_w)
        return Gs, g_v, g_phi, g_Bas, g_Un, g_W, g_b, None


class _MsgBwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Gs, Gv, v, phi, Bas, Un, W, b, cfg, need_w):
        ctx.cfg = cfg
        ctx.save_for_backward(Gs, Gv, v, phi, Bas, Un, W, b)
        if _device(v):
            out = _ops().painn_msg_vjp(_c(Gs), _c(Gv), _c(v), _c(phi), _c(Bas), _c(Un), _c(W), _c(b),
                                       *cfg.csr_args(), need_w)
            out = list(out)
            if not need_w:
                out[4] = out[5] = None
        else:
            out = _msg_vjp(cfg, Gs, Gv, v, phi, Bas, Un, W, b, need_w)
        if need_w:
            ctx.mark_non_differentiable(out[4], out[5])
        return tuple(out)

    @staticmethod
    def backward(ctx, Hv, Hphi, HBas, HUn, HW, Hb):
        Gs, Gv, v, phi, Bas, Un, W, b = ctx.saved_tensors
        need = ctx.needs_input_grad[:8]
        if _device(v):
            g = _ops().painn_msg_vvjp(_c(Gs), _c(Gv), _c(v), _c(phi), _c(Bas), _c(Un), _c(W), _c(b),
                                      *ctx.cfg.csr_args(), _c(Hv), _c(Hphi), _c(HBas), _c(HUn),
                                      [int(x) for x in need])
            g = [t if n else None for t, n in zip(g, need)]
        else:
            g = _msg_vvjp(ctx.cfg, Gs, Gv, v, phi, Bas, Un, W, b, Hv, Hphi, HBas, HUn, None, None, need)
        return (*g, None, None)


def painn_message(s, v, phi, Bas, Un, W, b, dst_si, src_si):
    """s + sum_src o_s, v + sum_src (v[dst] o_v + o_e d̂/d) with o = ([W | b] basis) * phi[dst]."""
    cfg = _MsgCfg()
    cfg.dst, cfg.src = dst_si.index64, src_si.index64
    cfg.dst_si, cfg.src_si = dst_si, src_si
    cfg.N, cfg.F, cfg.R = s.shape[0], s.shape[1], W.shape[1]
    return _Msg.apply(s, v, phi, Bas, Un, W, b, cfg)


# ============================================================================ node chains
class ChainProg:
    """A compiled node chain: forward program + generated VJP / VVJP programs."""

    def __init__(self, prog, ins, outs, weights):
        self.prog, self.ins, self.outs, self.weights = prog, list(ins), list(outs), list(weights)
        self.dev = {}  # (mode, device) -> _DevMode
        # first order: reverse of the forward program
        self.gouts = [rp.Val(o.w, o.nc, name=f"g{o.name}") for o in self.outs]
        vjp, self.vjp_res, self.vjp_wg = rp.reverse(prog, dict(zip(self.outs, self.gouts)), self.ins)
        vjp_in, self.vjp_in_res, _ = rp.reverse(prog, dict(zip(self.outs, self.gouts)), self.ins, want_weights=False)
        # backward programs recompute the forward values they read (cheap row-local work)
        wg_reads = [r[3] for r in self.vjp_wg if r[0] == "w"] + [r[4] for r in self.vjp_wg if r[0] == "w"] + \
            [r[2] for r in self.vjp_wg if r[0] == "b"]
        self.vjp = rp.concat_pruned(prog.ins, vjp.ins, keep_out=wg_reads)
        self.vjp_in = rp.concat_pruned(prog.ins, vjp_in.ins)
        # second order: reverse of the dual program seeded on the output tangents
        self.hins = [rp.Val(x.w, x.nc, name=f"h{x.name}") for x in self.ins]
        self.dual, tan = rp.dual(prog, dict(zip(self.ins, self.hins)))
        self.touts = [tan.get(o.base.id) for o in self.outs]
        seeds = {t: g for t, g in zip(self.touts, self.gouts) if t is not None}
        vvjp, self.vvjp_res, self.vvjp_wg = rp.reverse(self.dual, seeds, self.ins)
        wg_reads = [r[3] for r in self.vvjp_wg if r[0] == "w"] + [r[4] for r in self.vvjp_wg if r[0] == "w"] + \
            [r[2] for r in self.vvjp_wg if r[0] == "b"]
        self.vvjp = rp.concat_pruned(self.dual.ins, vvjp.ins, keep_out=[t for t in self.touts if t is not None] +
                                     wg_reads)


def _run(cp, prog, env_in, mask, N, wg=None):
    env = {v.base.id: t.reshape(N, -1) for v, t in env_in.items()}
    rp.run_torch(prog, env, cp.weights_t, mask, N)
    grads = None
    if wg is not None:
        grads = rp.wgrads_torch(wg, env, N, cp.weights_t, [None] * len(cp.weights_t))
    return env, grads


def _device(t):
    from .. import _native

    return t.is_cuda and t.dtype == torch.float32 and _native.available()


class _DevMode:
    """One program lowered for the interpreter: tables on the device + external roots."""

    def __init__(self, prog, ext_roots, inputs, n_weights, wg, dev):
        keep = []
        for rec in (wg or []):
            keep += [rec[3].base, rec[4].base] if rec[0] == "w" else [rec[2].base]
        ins, bufs, width, lds_w, where = rp.compile_device(prog, ext_roots, n_weights, inputs=inputs,
                                                           keep_global=keep)
        self.ins = torch.from_numpy(ins).to(dev)
        self.bufs = torch.from_numpy(bufs).to(dev)
        self.width = width
        self.lds_w = lds_w
        self.where = where
        self.bufs_np = bufs
        self.ext = list(ext_roots)
        self.rounds = rp.wgrad_rounds(wg) if wg else []


def _dev_mode(cp, mode, dev):
    key = (mode, str(dev))
    dm = cp.dev.get(key)
    if dm is None:
        nW = len(cp.weights)
        if mode == "fwd":
            prog, ext, wg = cp.prog, cp.ins + [o.base for o in cp.outs], None
            inputs = cp.ins
        elif mode == "vjp_in":
            prog, wg = cp.vjp_in, None
            ext = cp.ins + cp.gouts + [a.base for a in cp.vjp_in_res.values() if a is not None]
            inputs = cp.ins + cp.gouts
        elif mode == "vjp":
            prog, wg = cp.vjp, cp.vjp_wg
            ext = cp.ins + cp.gouts + [a.base for a in cp.vjp_res.values() if a is not None]
            inputs = cp.ins + cp.gouts
        else:
            prog, wg = cp.vvjp, cp.vvjp_wg
            ext = cp.ins + cp.hins + cp.gouts + [t for t in cp.touts if t is not None] + \
                [a.base for a in cp.vvjp_res.values() if a is not None]
            inputs = cp.ins + cp.hins + cp.gouts
        seen, uniq = set(), []
        for v in ext:
            if v.id not in seen:
                seen.add(v.id)
                uniq.append(v)
        dm = _DevMode(prog, uniq, inputs, nW, wg, dev)
        cp.dev[key] = dm
    return dm


def _dev_exec(cp, mode, N, mask, feeds, ws):
    """Run program ``mode`` on the device.  feeds: {root Val: tensor}; returns a getter
    Val -> [N, nc * w] view (external tensor or workspace slot) and the workspace."""
    from .. import _native

    x0 = next(iter(feeds.values()))
    dm = _dev_mode(cp, mode, x0.device)
    tens = {}
    ptrs = [w if w.is_contiguous() else w.contiguous() for w in ws]
    for v in dm.ext:
        t = feeds.get(v)
        if t is None:
            t = torch.empty(N, v.nc * v.w, device=x0.device, dtype=torch.float32)
        t = t.reshape(N, v.nc * v.w)
        if not t.is_contiguous():
            t = t.contiguous()
        tens[v.id] = t
        ptrs.append(t)
    wsb = torch.empty(max(N * dm.width, 1), device=x0.device, dtype=torch.float32)
    _native.ops().rowprog_run(dm.ins, wsb, mask, ptrs, N, dm.lds_w, None, len(ws))

    def get(v):
        b = v.base
        if b.id in tens:
            t = tens[b.id]
        else:
            k = dm.where[b.id]
            assert int(dm.bufs_np[k][0]) in (rp.B_WS, rp.B_LDS_WS), f"{b} has no global home"
            off = int(dm.bufs_np[k][1]) * N
            t = wsb[off:off + N * b.nc * b.w].view(N, b.nc * b.w)
        if v.full:
            return t
        return t.view(N, b.nc, b.w)[:, :, v.c0:v.c0 + v.w].reshape(N, -1) if b.nc == 1 else \
            t.view(N, b.nc, b.w)[:, :, v.c0:v.c0 + v.w]

    return get, dm


def _defer_ok(ws):
    from .linear import _defer

    return _defer["on"] and not torch.is_grad_enabled() and all(isinstance(w, torch.nn.Parameter) for w in ws)


def _dev_wgrads_defer(dm, get, N, ws):
    """Record a device run's weight-gradient products with the backward's deferred grouped
    weight-gradient launch (ops/linear.py deferred_wgrad): every row program of the
    backward, first- and second-order, shares one launch pair per round, accumulating in
    place into ``.grad`` (no per-program launches, no autograd accumulation adds)."""
    from .linear import _record

    for rnd in dm.rounds:
        for (pid, k0, G, X, bias, acc) in rnd:
            g, x = get(G), get(X)
            if G.nc == 3:
                g = g.reshape(N * 3, G.w)
                x = x.reshape(N * 3, X.w)
            _record((g, x, ws[pid], ws[bias] if bias is not None else None, k0))


def _dev_wgrads(dm, get, N, ws):
    """Weight gradients of a device run: one grouped MFMA launch pair per round."""
    from .. import _native

    grads = [None] * len(ws)
    covered = {}
    for (pid, k0, G, X, bias, acc) in (dm.rounds[0] if dm.rounds else []):
        covered.setdefault(pid, 0)
        covered[pid] += X.w
    for pid, K in covered.items():
        grads[pid] = torch.empty_like(ws[pid]) if K == ws[pid].shape[1] else torch.zeros_like(ws[pid])
    for rnd in dm.rounds:
        dys, xs, dws, dbs, accs = [], [], [], [], []
        for (pid, k0, G, X, bias, acc) in rnd:
            g, x = get(G), get(X)
            if G.nc == 3:
                g = g.reshape(N, 3, G.w).reshape(N * 3, G.w) if g.is_contiguous() else \
                    g.reshape(N * 3, G.w)
                x = x.reshape(N * 3, X.w) if x.is_contiguous() else x.reshape(N * 3, X.w)
            if grads[pid] is None:
                grads[pid] = torch.zeros_like(ws[pid])
            if bias is not None and grads[bias] is None:
                grads[bias] = torch.empty_like(ws[bias])
            dys.append(g)
            xs.append(x)
            dws.append(grads[pid][:, k0:k0 + X.w])
            dbs.append(grads[bias] if bias is not None else torch.empty(0, device=g.device))
            accs.append(1 if acc else 0)
        _native.ops().linear_wgrad_grouped(dys, xs, dws, dbs, accs)
    return grads


class _Chain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cp, mask, n_in, *args):
        xs, ws = args[:n_in], args[n_in:]
        N = xs[0].shape[0]
        if _device(xs[0]):
            get, _ = _dev_exec(cp, "fwd", N, mask, dict(zip(cp.ins, xs)), ws)
            outs = [get(o).reshape(N, o.nc, o.w) if o.nc == 3 else get(o) for o in cp.outs]
        else:
            cp.weights_t = ws
            env, _ = _run(cp, cp.prog, dict(zip(cp.ins, xs)), mask, N)
            outs = [_slot(env, o, N).reshape(N, o.nc, o.w) if o.nc == 3 else _slot(env, o, N) for o in cp.outs]
        ctx.cp, ctx.mask, ctx.n_in = cp, mask, n_in
        ctx.save_for_backward(*xs, *ws)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        cp, n_in = ctx.cp, ctx.n_in
        saved = ctx.saved_tensors
        xs, ws = saved[:n_in], saved[n_in:]
        gouts = [g.contiguous() if g is not None else
                 torch.zeros(xs[0].shape[0], o.nc * o.w, dtype=xs[0].dtype, device=xs[0].device)
                 for g, o in zip(gouts, cp.outs)]
        need_w = not _state["inputs_only"] and any(ctx.needs_input_grad[3 + n_in:])
        res = _ChainBwd.apply(cp, ctx.mask, n_in, len(gouts), need_w, *gouts, *xs, *ws)
        gx, gw = res[:n_in], res[n_in:]
        if need_w and gw and gw[0].numel() == 0 and ws[0].numel() != 0:  # deferred to the grouped flush
            need_w = False
        return (None, None, None, *gx, *(gw if need_w else [None] * len(ws)))


class _ChainBwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cp, mask, n_in, n_out, need_w, *args):
        gouts, xs, ws = args[:n_out], args[n_out:n_out + n_in], args[n_out + n_in:]
        N = xs[0].shape[0]
        res = cp.vjp_res if need_w else cp.vjp_in_res
        feeds = {**dict(zip(cp.ins, xs)), **dict(zip(cp.gouts, gouts))}
        deferred = False
        if _device(xs[0]):
            get, dm = _dev_exec(cp, "vjp" if need_w else "vjp_in", N, mask, feeds, ws)
            if need_w and _defer_ok(ws):
                _dev_wgrads_defer(dm, get, N, ws)
                grads, deferred = [None] * len(ws), True
            else:
                grads = _dev_wgrads(dm, get, N, ws) if need_w else None
        else:
            cp.weights_t = ws
            env, grads = _run(cp, cp.vjp if need_w else cp.vjp_in, feeds, mask, N, cp.vjp_wg if need_w else None)
            get = lambda v: _slot(env, v, N)  # noqa: E731
        gx = [get(res[x]).reshape(t.shape) if res[x] is not None else torch.zeros_like(t) for x, t in zip(cp.ins, xs)]
        gw = [g if g is not None else torch.zeros_like(w) for g, w in zip(grads, ws)] if (need_w and not deferred) \
            else [torch.zeros(0, dtype=xs[0].dtype, device=xs[0].device) for _ in ws]
        ctx.mark_non_differentiable(*gw)
        ctx.deferred = deferred
        ctx.params = list(ws)  # the Parameter objects themselves (deferred weight gradients)
        ctx.cp, ctx.mask, ctx.n_in, ctx.n_out = cp, mask, n_in, n_out
        ctx.save_for_backward(*gouts, *xs, *ws)
        return (*gx, *gw)

    @staticmethod
    def backward(ctx, *hs):
        cp, n_in, n_out = ctx.cp, ctx.n_in, ctx.n_out
        saved = ctx.saved_tensors
        gouts, xs, ws = saved[:n_out], saved[n_out:n_out + n_in], saved[n_out + n_in:]
        N = xs[0].shape[0]
        hx = [h.contiguous() if h is not None else torch.zeros_like(x) for h, x in zip(hs[:n_in], xs)]
        feeds = {**dict(zip(cp.ins, xs)), **dict(zip(cp.hins, hx)), **dict(zip(cp.gouts, gouts))}
        if _device(xs[0]):
            get, dm = _dev_exec(cp, "vvjp", N, ctx.mask, feeds, ws)
            if _defer_ok(ctx.params):
                _dev_wgrads_defer(dm, get, N, ctx.params)
                grads = [None] * len(ws)
            else:
                grads = _dev_wgrads(dm, get, N, ws)
        else:
            cp.weights_t = ws
            env, grads = _run(cp, cp.vvjp, feeds, ctx.mask, N, cp.vvjp_wg)
            get = lambda v: _slot(env, v, N)  # noqa: E731
        g_gouts = [get(t).reshape(g.shape) if t is not None else torch.zeros_like(g) for t, g in zip(cp.touts, gouts)]
        g_xs = [get(cp.vvjp_res[x]).reshape(t.shape) if cp.vvjp_res[x] is not None else torch.zeros_like(t)
                for x, t in zip(cp.ins, xs)]
        g_ws = [g if g is not None else (None if _defer_ok(ctx.params) else torch.zeros_like(w))
                for g, w in zip(grads, ws)]
        return (None, None, None, None, None, *g_gouts, *g_xs, *g_ws)


def _slot(env, v, N):
    t = env[v.base.id]
    if v.full:
        return t
    return t.view(N, v.base.nc, v.base.w)[:, :, v.c0:v.c0 + v.w].reshape(N, -1)


def run_chain(cp, mask, xs, ws):
    """Outputs of the chain ``cp`` for inputs ``xs`` (vectors as [N, 3, w]) and weights ``ws``
    (aligned with the chain's weight list)."""
    return _Chain.apply(cp, mask, len(xs), *xs, *ws)


# ============================================================================ PAINN model
def _act_name(m):
    for name, cls in (("relu", torch.nn.ReLU), ("silu", torch.nn.SiLU), ("tanh", torch.nn.Tanh),
                      ("sigmoid", torch.nn.Sigmoid), ("identity", torch.nn.Identity)):
        if isinstance(m, cls):
            return name
    return None


def model_ok(model, ctx):
    """The native path covers PAINNStack without global attention, edge-feature filters or
    activation checkpointing, with a supported activation (``HYDRA_UNFUSED=painn`` turns it
    off; it is NOT affected by ``composite_mode``: it is itself twice differentiable)."""
    from .pna import _state as _mode_state

    if "painn" in _mode_state["off"] or model.use_global_attn or model.conv_checkpointing:
        return False
    if _act_name(model.activation_function) is None:
        return False
    data = ctx.data
    if data.pos is None or ctx.dst_si is None or ctx.src_si is None:
        return False
    for conv in model.graph_convs:
        msg = conv.message
        if msg.edge_dim is not None and ctx.get("edge_attr") is not None:
            return False
    return True


class _ChainBuilder:
    """Row-program builder that maps program weights to module parameters."""

    def __init__(self):
        self.P = rp.Prog()
        self.params = []

    def W(self, lin):
        pid = len(self.params)
        self.params.append(lin.weight)
        bid = None
        if lin.bias is not None:
            bid = len(self.params)
            self.params.append(lin.bias)
        return rp.Weight(pid, lin.weight.shape[0], lin.weight.shape[1], bid)

    def linear(self, xs, lin, name=""):
        return self.P.lin(xs, self.W(lin), name=name)

    def mlp2(self, x, seq, act_mid, name):
        """Linear - act - Linear (scalar_message_mlp / node_embed_out)."""
        h = self.P.act(self.linear([(x, 0)], seq[0], name=f"{name}.0"), act_mid, name=f"{name}.a")
        return self.linear([(h, 0)], seq[2], name=name)


def _phi_prog(layer, F, mask):
    """Layer-0 prologue: phi = scalar_message_mlp(mask(x))."""
    cb = _ChainBuilder()
    s = cb.P.input(F, 1, "s0")
    x = cb.P.mask(s, name="s0m") if mask else s
    phi = cb.mlp2(x, layer.message.scalar_message_mlp, "silu", "phi0")
    cb.P.outputs = [phi]
    return ChainProg(cb.P, [s], [phi], [None] * len(cb.params)), cb.params


def _head_seq(model):
    """The node-level MLP head (``MLPNode`` 'mlp': Linear/activation chain) when the model
    has exactly one node head and one branch, else None."""
    if model.num_heads != 1 or model.head_type[0] != "node" or getattr(model, "num_branches", 1) != 1 or \
            model.var_output:
        return None
    head = model.heads_NN[0]["branch-0"]
    if getattr(head, "node_type", None) != "mlp":
        return None
    seq = list(head.mlp[0])
    for m in seq:
        if not isinstance(m, torch.nn.Linear) and _act_name(m) is None:
            return None
    return seq


def _layer_prog(layer, next_layer, act, mask, head=None):
    """update -> node_embed_out -> activation (+ mask) [-> vec_embed_out, next phi | node head]."""
    upd = layer.update
    F = upd.update_V.weight.shape[1]
    cb = _ChainBuilder()
    P = cb.P
    s = P.input(F, 1, "s")
    v = P.input(F, 3, "v")
    Uv = cb.linear([(v, 0)], getattr(upd, upd._u), name="Uv")
    Vv = cb.linear([(v, 0)], upd.update_V, name="Vv")
    n = P.norm3(Vv, name="nVv")
    a1 = P.act(cb.linear([(n, 0), (s, F)], upd.update_mlp[0], name="a1p"), "silu", name="a1")
    a = cb.linear([(a1, 0)], upd.update_mlp[2], name="a")
    inner = P.dot3(Uv, Vv, name="inner")
    if upd.last_layer:
        s2 = P.add(s, P.mul(a.slice(0, F), inner), a.slice(F, F), name="s2")
        v2 = None
    else:
        s2 = P.add(s, P.mul(a.slice(F, F), inner), a.slice(2 * F, F), name="s2")
        v2 = P.add(v, P.mul(a.slice(0, F), Uv), name="v2")
    s3 = cb.mlp2(s2, layer.node_embed_out, "tanh", "s3")
    so = P.act(s3, act, name="so_a")
    if mask:
        so = P.mask(so, name="so")
    outs = [so]
    if v2 is not None:
        outs.append(cb.linear([(v2, 0)], layer.vec_embed_out, name="v3"))
    if next_layer is not None:
        outs.append(cb.mlp2(so, next_layer.message.scalar_message_mlp, "silu", "phi"))
    elif head is not None:
        h = so
        for k, m in enumerate(head):
            h = cb.linear([(h, 0)], m, name=f"head{k}") if isinstance(m, torch.nn.Linear) else \
                P.act(h, _act_name(m), name=f"head{k}a")
        outs.append(h)
    P.outputs = outs
    return ChainProg(P, [s, v], outs, [None] * len(cb.params)), cb.params


def _programs(model, mask):
    key = ("painn_progs", bool(mask), _act_name(model.activation_function))
    cache = model.__dict__.setdefault("_native_force_progs", {})
    if key not in cache:
        layers = list(model.graph_convs)
        act = _act_name(model.activation_function)
        F0 = layers[0].update.update_V.weight.shape[1]
        progs = [_phi_prog(layers[0], F0, mask)]
        head = _head_seq(model)
        for i, layer in enumerate(layers):
            nxt = layers[i + 1] if i + 1 < len(layers) else None
            progs.append(_layer_prog(layer, nxt, act, mask, head if nxt is None else None))
        cache[key] = progs
    return cache[key]


def painn_encode(model, inv, ctx):
    """Native PAINN encoder: (node features, vector features, ctx), the same values as the
    layer-by-layer composite (``Base.encode`` over ``_EqLayer``)."""
    data = ctx.data
    keep = data.get("node_mask")
    mask = keep.to(inv.dtype) if keep is not None else None
    layers = list(model.graph_convs)
    msg0 = layers[0].message
    B, U = edge_geometry(data.pos, ctx.dst_si, ctx.src_si, msg0.num_radial, msg0.cutoff,
                         shifts=data.get("edge_shifts"))
    progs = _programs(model, mask is not None)
    cp, params = progs[0]
    s = inv
    (phi,) = run_chain(cp, mask, [s], params)
    v = torch.zeros(s.shape[0], 3, s.shape[1], device=s.device, dtype=s.dtype)
    for i, layer in enumerate(layers):
        flt = layer.message.filter_layer
        s1, v1 = painn_message(s, v, phi, B, U, flt.weight, flt.bias, ctx.dst_si, ctx.src_si)
        cp, params = progs[i + 1]
        outs = run_chain(cp, mask, [s1, v1], params)
        s = outs[0]
        if len(outs) > 1 and cp.outs[1].nc == 3:
            v = outs[1]
            phi = outs[2] if len(outs) > 2 else None
        else:
            v = v1
            phi = outs[1] if len(outs) > 1 else None
    if phi is not None and i == len(layers) - 1:
        ctx.native_node_head = phi  # the fused node head's output (PAINNStack.decode)
    return s, v, ctx
