"""Native twice-differentiable PAINN ops (``ops/painn_force.py``, ``ops/rowprog.py``):
fp64 gradcheck + gradgradcheck of every op family's CPU twin (the same formulas the HIP
kernels run), and the whole native force step against the torch composite."""
import copy

import numpy as np
import pytest
import torch

from hydragnn_amd.ops import painn_force as pf
from hydragnn_amd.ops import rowprog as rp
from hydragnn_amd.ops.segment import SegIndex

DT = torch.float64


def _graph(N=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    pos = torch.randn(N, 3, generator=g, dtype=DT) * 1.3
    src, dst = [], []
    for i in range(N):
        for j in range(N):
            if i != j and (i + 2 * j) % 3 != 0:
                src.append(i)
                dst.append(j)
    src, dst = torch.tensor(src), torch.tensor(dst)
    o = torch.argsort(dst, stable=True)
    src, dst = src[o], dst[o]
    dst_si = SegIndex.from_index(dst, N, sorted_=True)
    src_si = SegIndex.from_index(src, N)
    return pos, dst_si, src_si


def test_edge_geometry_grad_gradgrad():
    pos, dsi, ssi = _graph()
    pos.requires_grad_(True)

    def f(p):
        B, U = pf.edge_geometry(p, dsi, ssi, 4, 5.0)
        return B, U

    assert torch.autograd.gradcheck(f, (pos,))
    assert torch.autograd.gradgradcheck(f, (pos,))
    # matches the composite (PainnMessage._edge_terms: sinc * cut, cut, d̂/d)
    from hydragnn_amd.ops.geometry import edge_vectors_and_lengths
    from hydragnn_amd.models.painn import sinc_expansion, cosine_cutoff
    vec, d = edge_vectors_and_lengths(pos, dsi, ssi, None, normalize=True)
    rbf, cut = sinc_expansion(d, 4, 5.0), cosine_cutoff(d, 5.0)
    B, U = f(pos)
    torch.testing.assert_close(B[:, :4], rbf * cut)
    torch.testing.assert_close(B[:, 4:], cut)
    torch.testing.assert_close(U, vec / d)


def test_message_grad_gradgrad():
    pos, dsi, ssi = _graph(seed=1)
    N, F, R = pos.shape[0], 3, 4
    g = torch.Generator().manual_seed(2)
    E = dsi.index.numel()
    args = [torch.randn(N, F, generator=g, dtype=DT), torch.randn(N, 3, F, generator=g, dtype=DT),
            torch.randn(N, 3 * F, generator=g, dtype=DT), torch.randn(E, R + 1, generator=g, dtype=DT),
            torch.randn(E, 3, generator=g, dtype=DT), torch.randn(3 * F, R, generator=g, dtype=DT),
            torch.randn(3 * F, generator=g, dtype=DT)]
    args = [a.requires_grad_(True) for a in args]

    def f(*a):
        return pf.painn_message(*a, dsi, ssi)

    assert torch.autograd.gradcheck(f, args)
    assert torch.autograd.gradgradcheck(f, args)


def _chain_prog(F, Fo, last, act="relu"):
    P = rp.Prog()
    s = P.input(F, 1, "s")
    v = P.input(F, 3, "v")
    ws = []

    def W(O, K, bias=True):
        pid = len(ws)
        ws.append((O, K))
        bid = None
        if bias:
            bid = len(ws)
            ws.append((O,))
        return rp.Weight(pid, O, K, bid)

    WU, WV = W(F, F, False), W(F, F, False)
    Wu1, Wu2 = W(F, 2 * F), W(2 * F if last else 3 * F, F)
    Wa1, Wa2 = W(Fo, F), W(Fo, Fo)
    Uv = P.lin([(v, 0)], WU, name="Uv")
    Vv = P.lin([(v, 0)], WV, name="Vv")
    n = P.norm3(Vv, name="n")
    a1 = P.act(P.lin([(n, 0), (s, F)], Wu1, name="a1p"), "silu", name="a1")
    a = P.lin([(a1, 0)], Wu2, name="a")
    inner = P.dot3(Uv, Vv, name="inner")
    if last:
        s2 = P.add(s, P.mul(a.slice(0, F), inner), a.slice(F, F), name="s2")
    else:
        s2 = P.add(s, P.mul(a.slice(F, F), inner), a.slice(2 * F, F), name="s2")
        v2 = P.add(v, P.mul(a.slice(0, F), Uv), name="v2")
    t = P.act(P.lin([(s2, 0)], Wa1, name="tp"), "tanh", name="t")
    so = P.mask(P.act(P.lin([(t, 0)], Wa2, name="s3"), act), name="so")
    outs = [so]
    if not last:
        Wv = W(Fo, F, False)
        outs.append(P.lin([(v2, 0)], Wv, name="v3"))
        W1, W2 = W(Fo, Fo), W(3 * Fo, Fo)
        p1 = P.act(P.lin([(so, 0)], W1, name="p1p"), "silu", name="p1")
        outs.append(P.lin([(p1, 0)], W2, name="phi"))
    P.outputs = outs
    return pf.ChainProg(P, [s, v], outs, ws), ws


@pytest.mark.parametrize("last", [False, True])
def test_node_chain_grad_gradgrad(last):
    F, Fo, N = 3, 4, 5
    cp, shapes = _chain_prog(F, Fo, last, act="silu")
    g = torch.Generator().manual_seed(3)
    ws = [(torch.randn(*sh, generator=g, dtype=DT) * 0.5).requires_grad_(True) for sh in shapes]
    s = torch.randn(N, F, generator=g, dtype=DT, requires_grad=True)
    v = torch.randn(N, 3, F, generator=g, dtype=DT, requires_grad=True)
    mask = torch.tensor([1, 1, 0, 1, 1], dtype=DT)

    def f(s, v, *w):
        return pf.run_chain(cp, mask, [s, v], list(w))

    assert torch.autograd.gradcheck(f, [s, v, *ws])
    assert torch.autograd.gradgradcheck(f, [s, v, *ws])


def _md_model_batch(dtype=DT, seed=0):
    from hydragnn_amd.data.graph import collate
    from hydragnn_amd.data.synthetic import md_trajectory
    from hydragnn_amd.data.transforms import radius_graph
    from hydragnn_amd.models.create import create_model

    s = md_trajectory(6, seed=2, num_atoms=7)
    for d in s:
        d.edge_index = radius_graph(d.pos, 5.0, max_num_neighbors=6)
        d.sort_edges_by_dst()
    heads = {"node": [{"type": "branch-0", "architecture": {"num_headlayers": 2, "dim_headlayers": [8, 8],
                                                            "type": "mlp"}}]}
    torch.manual_seed(seed)
    m = create_model("PAINN", 1, 8, [1], 0, "", "", 0, ["node"], heads, "relu", "mse", [1.0], 3, num_radial=5,
                     radius=5.0, max_neighbours=6, edge_dim=None, equivariance=True, use_gpu=False, dropout=0.0)
    m = m.to(dtype)
    b = collate(s)
    for k in ("x", "pos", "energy", "forces"):
        b[k] = b[k].to(dtype)
    return m, b


def _force_step(m, b):
    from hydragnn_amd.ops.pna import composite_mode

    m.zero_grad(set_to_none=True)
    b.pos = b.pos.detach().requires_grad_(True)
    with composite_mode(True):
        pred = m(b)
        loss, _ = m.energy_force_loss(pred, b)
    loss.backward()
    return loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}


def test_native_painn_force_step_equals_composite():
    """Energy + force loss and every parameter gradient of the native PAINN force path equal
    the layer-by-layer torch composite (fp64; ``HYDRA_UNFUSED=painn`` is the composite)."""
    from hydragnn_amd.ops.pna import _state

    m, b = _md_model_batch()
    ref = copy.deepcopy(m)
    calls = {"n": 0}
    orig = pf.painn_encode

    def spy(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    pf.painn_encode = spy
    try:
        ln, gn = _force_step(m, b)
    finally:
        pf.painn_encode = orig
    assert calls["n"] == 1
    _state["off"].add("painn")
    try:
        lr, gr = _force_step(ref, b)
    finally:
        _state["off"].discard("painn")
    torch.testing.assert_close(ln, lr, rtol=1e-10, atol=1e-12)
    assert gn.keys() == gr.keys()
    for k in gr:
        torch.testing.assert_close(gn[k], gr[k], rtol=1e-8, atol=1e-10, msg=k)


def _emulate(ins, bufs, width, ptrs, N, mask, lds_w=0):
    """numpy model of csrc/rowprog.hip over the lowered instructions (embedded operand
    descriptors; the LDS of all row blocks modelled as one [N, lds_w] array, values with a
    global home written to both)."""
    ws = np.zeros(max(N * width, 1))
    lds = np.full((N, max(lds_w, 1)), np.nan)  # unwritten LDS reads poison the results
    O = rp.OPD_INTS

    def opd(I, q):
        d = I[8 + O * q: 8 + O * (q + 1)]
        if not d[0]:
            return None
        _, gk, gi, gld, lo, lld, cs, c0, w, nc = d[:10]
        ncr = gld // cs
        g = None
        if gk == 1:
            g = ws[gi * N: gi * N + N * gld].reshape(N, ncr, cs)
        elif gk == 2:
            g = ptrs[gi].reshape(N, ncr, cs)
        loc = lds[:, lo:lo + gld].reshape(N, ncr, cs) if lo >= 0 else None
        return (loc if loc is not None else g, c0, w, nc, g if loc is not None else None)

    def view(d):
        arr, c0, w, nc, _ = d
        return arr[:, :, c0:c0 + w]

    def mirror(d):
        if d[4] is not None:
            d[4][:, :, d[1]:d[1] + d[2]] = d[0][:, :, d[1]:d[1] + d[2]]

    act = rp._act
    for I in ins:
        y = opd(I, 0)
        Y = view(y)
        if I[0] == 1:
            xs = [opd(I, 1), opd(I, 2)]
            W = ptrs[I[56]].reshape(-1, I[57])
            r = 0
            for x, k0 in zip(xs, (I[58], I[59])):
                if x is None:
                    continue
                X = view(x)
                if I[61]:
                    r = r + np.einsum("nck,ok->nco", X, W[:, k0:k0 + X.shape[2]])
                else:
                    r = r + np.einsum("nco,ok->nck", X, W[:, k0:k0 + Y.shape[2]])
            if I[60] >= 0:
                r = r + ptrs[I[60]].reshape(1, 1, -1)
            Y[...] = Y + r if I[4] else r
            mirror(y)
            continue
        op, arg, acc = I[1], I[2], I[4]
        coef = np.array([I[3]], dtype=np.int32).view(np.float32)[0]
        A, B, C = (view(d) if d is not None else None for d in (opd(I, 1), opd(I, 2), opd(I, 3)))
        if op == rp.E_ZERO:
            Y[...] = 0
            mirror(y)
            continue
        if op == rp.E_COPY:
            r = A
        elif op == rp.E_MUL:
            r = A * B
        elif op == rp.E_MUL3:
            r = A * B * C
        elif op == rp.E_ACT:
            r = act(torch.from_numpy(np.ascontiguousarray(A)), arg >> 2, arg & 3).numpy()
            if B is not None:
                r = r * B
            if C is not None:
                r = r * C
        elif op == rp.E_DOT3:
            r = (A * B).sum(1, keepdims=True)
            if C is not None:
                r = r * C
        elif op == rp.E_NORM3:
            r = np.sqrt((A * A).sum(1, keepdims=True))
        elif op == rp.E_SINV:
            r = np.where(A > 0, 1.0 / np.where(A > 0, A, 1.0), 0.0)
        elif op == rp.E_MASK:
            r = A * (mask.reshape(N, 1, 1) if mask is not None else 1.0)
        r = np.broadcast_to(r * coef, Y.shape)
        Y[...] = Y + r if acc else r
        mirror(y)
    return ws


@pytest.mark.parametrize("budget", [2400, 40, 0])
@pytest.mark.parametrize("mode", ["fwd", "vjp_in", "vjp", "vvjp"])
def test_rowprog_lowering_matches_twin(mode, budget):
    """The tables the interpreter kernel runs (rowprog.compile_device), executed by a numpy
    model of the kernel, reproduce the torch twin of every program mode."""
    F, Fo, N = 3, 4, 5
    cp, shapes = _chain_prog(F, Fo, False, act="silu")
    g = torch.Generator().manual_seed(5)
    ws = [torch.randn(*sh, generator=g, dtype=DT) * 0.5 for sh in shapes]
    xs = [torch.randn(N, F, generator=g, dtype=DT), torch.randn(N, 3, F, generator=g, dtype=DT)]
    gouts = [torch.randn(N, o.nc * o.w, generator=g, dtype=DT) for o in cp.outs]
    hins = [torch.randn_like(x) for x in xs]
    mask = torch.tensor([1, 0, 1, 1, 1], dtype=DT)
    feeds = dict(zip(cp.ins, xs))
    if mode == "fwd":
        prog, wanted = cp.prog, [o.base for o in cp.outs]
    elif mode in ("vjp_in", "vjp"):
        feeds.update(zip(cp.gouts, gouts))
        res = cp.vjp_in_res if mode == "vjp_in" else cp.vjp_res
        prog, wanted = (cp.vjp_in if mode == "vjp_in" else cp.vjp), [a.base for a in res.values() if a is not None]
    else:
        feeds.update(zip(cp.gouts, gouts))
        feeds.update(zip(cp.hins, hins))
        prog = cp.vvjp
        wanted = [t for t in cp.touts if t is not None] + [a.base for a in cp.vvjp_res.values() if a is not None]
    ext = list(feeds.keys()) + [v for v in wanted if v not in feeds]
    ins, bufs, width, lds_w, where = rp.compile_device(prog, ext, len(ws), inputs=list(feeds.keys()),
                                                       lds_budget=budget)
    ptrs = [w.numpy().copy() for w in ws]
    for v in ext:
        t = feeds.get(v)
        ptrs.append(t.reshape(N, -1).numpy().copy() if t is not None else np.zeros((N, v.nc * v.w)))
    _emulate(ins, bufs, width, ptrs, N, mask.numpy(), lds_w)
    cp.weights_t = ws
    env, _ = pf._run(cp, prog, feeds, mask, N)
    for k, v in enumerate(ext):
        if v in feeds:
            continue
        np.testing.assert_allclose(ptrs[len(ws) + k], env[v.id].numpy(), rtol=1e-12, atol=1e-12)
