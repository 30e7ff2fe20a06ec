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
