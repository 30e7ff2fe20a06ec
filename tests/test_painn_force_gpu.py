"""HIP kernels of the native PAINN force path (csrc/painn_force.hip, csrc/rowprog.hip)
against their CPU twins (ops/painn_force.py, fp64-gradgradchecked in test_painn_force.py),
and the whole native force step against the torch composite on the GPU."""
import copy
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_painn_force import _chain_prog, _graph, _md_model_batch  # noqa: E402

from hydragnn_amd.ops import painn_force as pf  # noqa: E402
from hydragnn_amd.ops.segment import SegIndex  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _si_to(si, dev):
    return SegIndex(si.index.to(dev), si.rowptr.to(dev), None if si.perm is None else si.perm.to(dev),
                    si.num_segments)


def _grads2(f, args, seed=0):
    """outputs, first-order input grads (create_graph) and the second-order grads of a
    random contraction of them: exercises forward, VJP and VVJP of every op."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    outs = f(*args)
    outs = outs if isinstance(outs, tuple) else (outs,)
    ws = [torch.randn(o.shape, generator=g, dtype=o.dtype).to(o.device) for o in outs]
    first = torch.autograd.grad(sum((o * w).sum() for o, w in zip(outs, ws)), args, create_graph=True,
                                allow_unused=True)
    hs = [torch.randn(a.shape, generator=g, dtype=a.dtype).to(a.device) for a in args]
    tot = sum((t * h).sum() for t, h in zip(first, hs) if t is not None)
    second = torch.autograd.grad(tot, args, allow_unused=True)
    return [o.detach() for o in outs], [t.detach() if t is not None else None for t in first], \
        [t if t is not None else None for t in second]


def _cmp(a, b, rtol=2e-4, atol=2e-5):
    for x, y in zip(a, b):
        if x is None or y is None:
            assert (x is None or x.abs().max() == 0) and (y is None or y.abs().max() == 0)
            continue
        scale = y.abs().max().item() + 1e-6
        assert (x.cpu() - y.cpu()).abs().max().item() <= rtol * scale + atol, ((x.cpu() - y.cpu()).abs().max(), scale)


def test_geometry_kernels_match_twin():
    pos, dsi, ssi = _graph(N=9, seed=3)
    pos = pos.float()
    d2, s2 = _si_to(dsi, DEV), _si_to(ssi, DEV)
    pc = pos.clone().requires_grad_(True)
    pg = pos.to(DEV).requires_grad_(True)
    rc = _grads2(lambda p: pf.edge_geometry(p, dsi, ssi, 6, 5.0), [pc])
    rg = _grads2(lambda p: pf.edge_geometry(p, d2, s2, 6, 5.0), [pg])
    for a, b in zip(rg, rc):
        _cmp(a, b)


def test_message_kernels_match_twin():
    pos, dsi, ssi = _graph(N=8, seed=4)
    N, F, R = pos.shape[0], 64, 6
    E = dsi.index.numel()
    g = torch.Generator().manual_seed(5)
    args = [torch.randn(N, F, generator=g), torch.randn(N, 3, F, generator=g), torch.randn(N, 3 * F, generator=g),
            torch.randn(E, R + 1, generator=g), torch.randn(E, 3, generator=g), torch.randn(3 * F, R, generator=g),
            torch.randn(3 * F, generator=g)]
    ac = [a.clone().requires_grad_(True) for a in args]
    ag = [a.to(DEV).requires_grad_(True) for a in args]
    d2, s2 = _si_to(dsi, DEV), _si_to(ssi, DEV)
    rc = _grads2(lambda *a: pf.painn_message(*a, dsi, ssi), ac)
    rg = _grads2(lambda *a: pf.painn_message(*a, d2, s2), ag)
    for a, b in zip(rg, rc):
        _cmp(a, b)


@pytest.mark.parametrize("last", [False, True])
def test_rowprog_interpreter_matches_twin(last):
    F, Fo, N = 64, 64, 37
    cp, shapes = _chain_prog(F, Fo, last, act="relu")
    g = torch.Generator().manual_seed(7)
    ws = [torch.randn(*sh, generator=g) * 0.2 for sh in shapes]
    xs = [torch.randn(N, F, generator=g), torch.randn(N, 3, F, generator=g)]
    mask = (torch.rand(N, generator=g) > 0.2).float()
    wc = [w.clone().requires_grad_(True) for w in ws]
    wg = [w.to(DEV).requires_grad_(True) for w in ws]
    xc = [x.clone().requires_grad_(True) for x in xs]
    xg = [x.to(DEV).requires_grad_(True) for x in xs]
    rc = _grads2(lambda *a: pf.run_chain(cp, mask, list(a[:2]), list(a[2:])), xc + wc)
    rg = _grads2(lambda *a: pf.run_chain(cp, mask.to(DEV), list(a[:2]), list(a[2:])), xg + wg)
    for a, b in zip(rg, rc):
        _cmp(a, b, rtol=5e-4, atol=5e-5)


def test_native_force_step_matches_composite_gpu():
    from hydragnn_amd.ops.pna import _state, composite_mode

    m, b = _md_model_batch(dtype=torch.float32)
    m = m.to(DEV)
    b = b.to(DEV)
    ref = copy.deepcopy(m)

    def step(model):
        model.zero_grad(set_to_none=True)
        b.pos = b.pos.detach().requires_grad_(True)
        with composite_mode(True):
            pred = model(b)
            loss, _ = model.energy_force_loss(pred, b)
        loss.backward()
        return loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}

    calls = {"n": 0}
    orig = pf.painn_encode

    def spy(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    pf.painn_encode = spy
    try:
        ln, gn = step(m)
    finally:
        pf.painn_encode = orig
    assert calls["n"] == 1
    _state["off"].add("painn")
    try:
        lr, gr = step(ref)
    finally:
        _state["off"].discard("painn")
    torch.testing.assert_close(ln, lr, rtol=1e-4, atol=1e-5)
    bad = []
    for k in gr:
        scale = gr[k].abs().max().item() + 1e-6
        err = (gn[k] - gr[k]).abs().max().item()
        if err > 2e-3 * scale + 1e-5:
            bad.append(f"{k}: {err:.3e} (scale {scale:.3e})")
    assert not bad, "\n".join(bad)
