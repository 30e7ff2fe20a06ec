"""Fused GPS(PNAPlus) encoder (``ops/gps_encoder.py`` over ``csrc/gps_fused.hip``) ==
the layer-by-layer module path on the GPU: identical weights, padded batch and dropout
masks; compares the loss, every parameter gradient and the BatchNorm running statistics
after one training forward + backward (fp32 tolerances: the two paths sum in different
orders).  The module path is itself checked against plain-torch CPU composites in
``test_model_parity_gpu.py``."""
import copy

import pytest
import torch

from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import degree_histogram, oc20_like
from hydragnn_amd.models.create import create_model
from hydragnn_amd.ops import gps_encoder
from hydragnn_amd.ops import pna as _mode
from hydragnn_amd.ops import rng as _rng
from hydragnn_amd.train.step import batch_loss

pytestmark = pytest.mark.gpu


def _setup(hidden, dropout, layers=3, heads=8, n=24):
    dev = torch.device("cuda")
    samples = oc20_like(n, seed=3, radius=8.0, max_neighbours=10, pe_dim=8, min_atoms=12, max_atoms=40)
    deg = degree_histogram(samples, 10)
    hd = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 16,
                                                           "num_headlayers": 2, "dim_headlayers": [16, 8]}}]}
    torch.manual_seed(0)
    model = create_model("PNAPlus", 4, hidden, [1], 8, "GPS", "multihead", heads, ["graph"], hd, "relu", "mae",
                         [1.0], layers, pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=8.0,
                         max_neighbours=10, dropout=dropout).to(dev)
    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    idx = list(range(16))
    N, E = store.sizes_of(idx)
    Np, Ep = ((N + 2 + 255) // 256) * 256, ((E + 2047) // 2048) * 2048
    lay = store.layout(idx, Np=Np, Ep=Ep, Gp=len(idx) + 1)
    batch = store.assemble(store.upload(idx, lay), lay)
    return model, batch


def _step(model, batch, fused, c0):
    calls = {"n": 0}
    orig = gps_encoder.encode

    def spy(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    gps_encoder.encode = spy
    off = _mode._state["off"]
    if not fused:
        off.add("gpsfused")
    try:
        _rng.counter(batch.x.device).fill_(c0)
        model.train()
        model.zero_grad(set_to_none=True)
        pred = model(batch)
        loss, _ = batch_loss(model, pred, batch)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        off.discard("gpsfused")
        gps_encoder.encode = orig
    assert calls["n"] == (1 if fused else 0), "fused encoder path did not run as expected"
    return loss.detach()


@pytest.mark.parametrize("hidden,dropout", [(64, 0.0), (64, 0.25), (32, 0.25)])
def test_fused_encoder_matches_module_path(hidden, dropout):
    model, batch = _setup(hidden, dropout)
    ref = copy.deepcopy(model)
    lf = _step(model, batch, True, 1234)
    lr = _step(ref, batch, False, 1234)
    torch.testing.assert_close(lf, lr, rtol=1e-4, atol=1e-5)
    bad = []
    for (n, a), (_, b) in zip(model.named_parameters(), ref.named_parameters()):
        if b.grad is None:
            assert a.grad is None or a.grad.abs().max() == 0, n
            continue
        assert a.grad is not None, f"no gradient for {n}"
        scale = b.grad.abs().max().item() + 1e-6
        err = (a.grad - b.grad).abs().max().item()
        if err > 2e-3 * scale + 1e-5:
            bad.append(f"{n}: max err {err:.3e} (scale {scale:.3e})")
    assert not bad, "gradient mismatch:\n" + "\n".join(bad)
    for (n, a), (_, b) in zip(model.named_buffers(), ref.named_buffers()):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=n)
        else:
            assert torch.equal(a, b), n


def test_fused_encoder_captured_step():
    """The fused encoder inside the hipGraph-captured TrainStep: replays train (finite,
    decreasing loss over a few steps on a fixed batch) and bucket capture works."""
    from hydragnn_amd.train.step import TrainStep

    dev = torch.device("cuda")
    samples = oc20_like(32, seed=5, radius=8.0, max_neighbours=10, pe_dim=8, min_atoms=12, max_atoms=40)
    deg = degree_histogram(samples, 10)
    hd = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 16,
                                                           "num_headlayers": 2, "dim_headlayers": [16, 8]}}]}
    torch.manual_seed(0)
    model = create_model("PNAPlus", 4, 64, [1], 8, "GPS", "multihead", 8, ["graph"], hd, "relu", "mae",
                         [1.0], 3, pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=8.0,
                         max_neighbours=10, dropout=0.0).to(dev)
    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    step = TrainStep(model, lr=1e-3, mode="graph")
    step.prepare(store, 8)
    idx = list(range(8))
    losses = [float(step(store, idx)[0]) for _ in range(8)]
    assert all(l == l and abs(l) < 1e6 for l in losses)
    assert losses[-1] < losses[0]


def test_fused_encoder_bitwise_reproducible():
    """BatchNorm statistics are accumulated with integer fixed-point atomics (order-
    independent): two identical training steps give bitwise-identical losses, gradients and
    running statistics (fp64 float atomics did not guarantee this)."""
    model, batch = _setup(64, 0.25)
    twin = copy.deepcopy(model)
    la = _step(model, batch, True, 777)
    lb = _step(twin, batch, True, 777)
    assert torch.equal(la, lb)
    for (n, a), (_, b) in zip(model.named_parameters(), twin.named_parameters()):
        if a.grad is not None:
            assert torch.equal(a.grad, b.grad), n
    for (n, a), (_, b) in zip(model.named_buffers(), twin.named_buffers()):
        assert torch.equal(a, b), n


@pytest.mark.parametrize("F,E", [(64, 26624), (64, 1000), (32, 77)])
def test_edge_fwd_multi_and_wprep_multi_match_torch(F, E):
    """One-launch edge terms / weight preps of every layer (csrc/gps_fused.hip
    edge_fwd_multi_kernel, csrc/pna.hip pna_wprep_fwd_multi) == fp32 torch and == the
    per-layer launches."""
    from hydragnn_amd import _native

    ops = _native.ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(F + E)
    L, d = 3, F
    rs = [torch.randn(E, F, generator=g).to(dev) for _ in range(L)]
    e = torch.randn(E, d, generator=g).to(dev)
    Ws = [(torch.randn(F, 3 * F, generator=g) * 0.1).to(dev) for _ in range(L)]
    bs = [torch.randn(F, generator=g).to(dev) for _ in range(L)]
    encW = [(torch.randn(F, d + F, generator=g) * 0.1).to(dev) for _ in range(L)]
    encb = [torch.randn(F, generator=g).to(dev) for _ in range(L)]
    pw = ops.pna_wprep_fwd_multi(Ws, bs, encW, encb)
    Cs = ops.gf_edge_fwd_multi(rs, e, pw[1::4], pw[2::4], pw[3::4])
    for l in range(L):
        one = ops.pna_wprep_fwd(Ws[l], bs[l], encW[l], encb[l])
        for a, b in zip(pw[4 * l:4 * l + 4], one):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
        Wr, Wd, bc = one[1], one[2], one[3]
        ref = rs[l].double() @ Wr.double().t() + e.double() @ Wd.double().t() + bc.double()
        torch.testing.assert_close(Cs[l].double(), ref, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(Cs[l], ops.gf_edge_fwd(rs[l], e, Wr, Wd, bc), rtol=1e-5, atol=1e-5)
