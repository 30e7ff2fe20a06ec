"""Force training (energy + forces = -dE/dpos, reference ``Base.energy_force_loss``,
``Base.py:582-636``) through the training engine: the statically padded step (the CPU
twin of the captured hipGraph step) equals the eager step, i.e. the dummy graph and
padding atoms are masked out of both the energy and the force loss."""
import copy

import numpy as np
import pytest
import torch

from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import md_trajectory
from hydragnn_amd.data.transforms import radius_graph
from hydragnn_amd.models.create import create_model
from hydragnn_amd.train.step import TrainStep

HEADS = {"node": [{"type": "branch-0", "architecture": {"num_headlayers": 2, "dim_headlayers": [16, 16],
                                                        "type": "mlp"}}]}


def _samples(n=16):
    s = md_trajectory(n, seed=2, num_atoms=9)
    for d in s:
        d.edge_index = radius_graph(d.pos, 5.0, max_num_neighbors=8)
        d.edge_attr = (d.pos[d.edge_index[1]] - d.pos[d.edge_index[0]]).norm(dim=-1, keepdim=True) / 5.0
        d.sort_edges_by_dst()
    return s


def _model(mpnn):
    return create_model(mpnn, 1, 16, [1], 0, "", "", 0, ["node"], HEADS, "relu", "mae", [1.0], 2, num_nodes=9,
                        edge_dim=1, radius=5.0, num_radial=6, envelope_exponent=5, equivariance=True, use_gpu=False,
                        dropout=0.0, max_neighbours=8, pna_deg=[0, 2, 4, 6, 8, 10, 6, 4, 2])


@pytest.mark.parametrize("mpnn", ["PAINN", "EGNN", "PNAEq"])
def test_padded_force_step_equals_eager(mpnn):
    samples = _samples()
    m1 = _model(mpnn)
    m2 = copy.deepcopy(m1)
    store = DeviceGraphStore(samples, "cpu")
    eager = TrainStep(m1, lr=1e-3, mode="eager", compute_grad_energy=True)
    padded = TrainStep(m2, lr=1e-3, mode="graph", compute_grad_energy=True, node_bucket=64, edge_bucket=512)
    rng = np.random.default_rng(0)
    for _ in range(3):
        idx = list(rng.choice(len(store), 4, replace=False))
        le = float(eager(store, idx)[0])
        lp = float(padded(store, idx)[0])
        assert abs(le - lp) <= 1e-4 * max(1.0, abs(le)), (le, lp)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn,n,B", [("PAINN", 16, 4), ("EGNN", 400, 150), ("PNAEq", 400, 150)])
def test_captured_force_step_matches_eager_gpu(mpnn, n, B, monkeypatch):
    """Captured force step == eager.  EGNN / PNAEq run big enough batches for the composite
    split-K linears (deferred into the grouped launch in the captured step); their eager twin
    runs plain F.linear (library GEMMs), so this also checks the split-K path end to end."""
    from hydragnn_amd.ops import linear as lin

    samples = _samples(n)
    m1 = _model(mpnn).cuda()
    m2 = copy.deepcopy(m1)
    store = DeviceGraphStore(samples, "cuda")
    eager = TrainStep(m1, lr=1e-3, mode="eager", compute_grad_energy=True)
    graph = TrainStep(m2, lr=1e-3, mode="graph", compute_grad_energy=True, node_bucket=512, edge_bucket=4096)
    rng = np.random.default_rng(0)
    for step in range(4):
        idx = list(rng.choice(len(store), B, replace=False))
        monkeypatch.setattr(lin, "_COMPOSITE_SK", False)
        le = float(eager(store, idx)[0])
        monkeypatch.setattr(lin, "_COMPOSITE_SK", True)
        lg = float(graph(store, idx)[0])
        assert abs(le - lg) <= 1e-3 * max(1.0, abs(le)), (le, lg)
        if step == 0:
            # parameters after the first update (later AdamW steps amplify the fp32 rounding
            # noise of near-zero gradients into +-lr moves, whatever the GEMM's summation order)
            for p1, p2 in zip(m1.parameters(), m2.parameters()):
                torch.testing.assert_close(p1, p2, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn", ["EGNN", "PNAEq"])
def test_composite_linear_splitk_matches_library_gemms_gpu(mpnn, monkeypatch):
    """Force training's composite linears (ops/linear.py _LinearC: both backward passes' weight
    gradients on the split-K kernel, twice differentiable) == plain F.linear: one force
    step's energy / force loss and every parameter gradient."""
    from hydragnn_amd.ops import linear as lin
    from hydragnn_amd.ops.pna import composite_mode

    samples = _samples(160)  # >= MIN_ROWS node and edge rows: the split-K path runs
    store = DeviceGraphStore(samples, "cuda")
    batch = store.batch(list(range(150)))
    grads = []
    for on in (True, False):
        monkeypatch.setattr(lin, "_COMPOSITE_SK", on)
        torch.manual_seed(0)
        m = _model(mpnn).cuda()
        b = store.batch(list(range(150)))
        b.pos.requires_grad_(True)
        with composite_mode(True):
            pred = m(b)
            loss, _ = m.energy_force_loss(pred, b)
            ps = [p for p in m.parameters() if p.requires_grad]
            gs = torch.autograd.grad(loss, ps, allow_unused=True)
        grads.append((float(loss), gs))
    assert batch.num_nodes >= lin.MIN_ROWS
    (l1, g1), (l2, g2) = grads
    assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l2)), (l1, l2)
    for a, c in zip(g1, g2):
        if a is None or c is None:
            assert a is None and c is None
            continue
        torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-5)


def test_force_test_returns_samples_and_dump(tmp_path, monkeypatch):
    """``test()`` on a force run returns per-graph energy samples (head 0) and, with
    HYDRAGNN_DUMP_TESTDATA=1, per-sample energy/force records (ref ``train_validate_test.py:642-705``)."""
    from hydragnn_amd.data.graph import collate
    from hydragnn_amd.train.train_validate_test import test as run_test

    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("HYDRAGNN_DUMP_TESTDATA", "1")
    samples = _samples(8)
    loader = [collate(samples[:4]), collate(samples[4:])]
    m = _model("PAINN")
    err, _, true, pred = run_test(loader, m, 0, compute_grad_energy=True)
    assert true[0].shape == (8, 1) and pred[0].shape == (8, 1)
    assert torch.allclose(true[0].view(-1), torch.stack([s.energy.reshape(()) for s in samples]).float())
    recs = torch.load(tmp_path / "testdata_rank0.pt", weights_only=True)
    assert len(recs) == 8
    assert recs[0]["forces_pred"].numel() == samples[0].num_nodes * 3
    assert abs(recs[3]["energy_pred"] - float(pred[0][3])) < 1e-5


@pytest.mark.parametrize("equivariance", [False, True])
def test_schnet_static_inforward_graph_padded_equals_eager(equivariance):
    """SchNet's in-forward radius graph (SCFStack.py:175-190) in the padded (capturable)
    step is rebuilt with a fixed edge capacity on the device (ops.radius
    .interaction_graph_static); the step equals the eager step (dynamic builder)."""
    samples = _samples()
    heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 8,
                                                             "num_headlayers": 1, "dim_headlayers": [8]}}]}
    for s in samples:
        s.y = s.energy.view(-1, 1) if "energy" in s else s.y.view(-1, 1)
        s.y_loc = torch.tensor([[0, 1]])
    m1 = create_model("SchNet", 1, 16, [1], 0, "", "", 0, ["graph"], heads, "relu", "mae", [1.0], 3,
                      num_gaussians=10, num_filters=16, radius=3.0, max_neighbours=4, dropout=0.0,
                      equivariance=equivariance, use_gpu=False)
    m2 = copy.deepcopy(m1)
    assert m1.capturable
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1])
    eager = TrainStep(m1, lr=1e-3, mode="eager")
    padded = TrainStep(m2, lr=1e-3, mode="graph", node_bucket=64, edge_bucket=512)
    rng = np.random.default_rng(1)
    for _ in range(3):
        idx = list(rng.choice(len(store), 4, replace=False))
        le = float(eager(store, idx)[0])
        lp = float(padded(store, idx)[0])
        assert abs(le - lp) <= 1e-4 * max(1.0, abs(le)), (le, lp)


def _dimenet(samples):
    heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 8,
                                                             "num_headlayers": 1, "dim_headlayers": [8]}}]}
    for s in samples:
        s.y = s.energy.view(-1, 1) if "energy" in s else s.y.view(-1, 1)
        s.y_loc = torch.tensor([[0, 1]])
    torch.manual_seed(0)
    return create_model("DimeNet", 1, 16, [1], 0, "", "", 0, ["graph"], heads, "relu", "mae", [1.0], 2,
                        radius=5.0, max_neighbours=8, num_radial=5, envelope_exponent=5, basis_emb_size=4,
                        int_emb_size=8, out_emb_size=8, num_after_skip=1, num_before_skip=1, num_spherical=3,
                        dropout=0.0, use_gpu=False)


def test_store_triplet_cap_bounds_every_batch():
    """DeviceGraphStore.triplet_cap(G) >= the real triplet count of any G-graph batch."""
    from hydragnn_amd.models.dimenet import triplets_csr
    from hydragnn_amd.ops.segment import SegIndex

    samples = _samples()
    store = DeviceGraphStore(samples, "cpu")
    per = []
    for s in samples:
        n = s.num_nodes
        dst_si = SegIndex.from_index(s.edge_index[1], n, sorted_=True)
        src_si = SegIndex.from_index(s.edge_index[0], n)
        per.append(triplets_csr(dst_si, src_si, n)[0].numel())
    ne = [s.num_edges for s in samples]
    ratio = max(t / e for t, e in zip(per, ne))
    srt = sorted(per, reverse=True)
    for G in (1, 3, 4, 16):
        cap = store.triplet_cap(G)
        assert cap >= sum(srt[:G]) and cap % 256 == 0 and cap < sum(srt[:G]) + 256
    rng = np.random.default_rng(0)
    for _ in range(20):  # the edge-ratio bound holds for every batch within the edge budget
        idx = rng.choice(len(samples), 4, replace=False)
        E = sum(ne[i] for i in idx)
        cap = store.triplet_cap(4, E)
        assert sum(per[i] for i in idx) <= cap <= max(256, ratio * E + 257)


def test_dimenet_static_triplets_padded_equals_eager():
    """DimeNet's triplets in the padded (capturable) step come from the fixed-capacity
    builder (models/dimenet.triplets_static: valid receivers only, dummy tail with zero
    basis rows); the step equals the eager step (data-dependent builder)."""
    samples = _samples()
    m1 = _dimenet(samples)
    m2 = copy.deepcopy(m1)
    assert m1.capturable
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1])
    eager = TrainStep(m1, lr=1e-3, mode="eager")
    padded = TrainStep(m2, lr=1e-3, mode="graph", node_bucket=64, edge_bucket=512)
    rng = np.random.default_rng(1)
    for _ in range(3):
        idx = list(rng.choice(len(store), 4, replace=False))
        le = float(eager(store, idx)[0])
        lp = float(padded(store, idx)[0])
        assert abs(le - lp) <= 1e-4 * max(1.0, abs(le)), (le, lp)


@pytest.mark.gpu
def test_dimenet_captured_step_matches_eager_gpu():
    """The captured DimeNet step (device triplet builder with static capacity, sbf kernels
    honouring the device limit) follows the eager trajectory."""
    samples = _samples()
    m1 = _dimenet(samples).cuda()
    m2 = copy.deepcopy(m1)
    store = DeviceGraphStore(samples, "cuda", head_types=["graph"], head_dims=[1])
    eager = TrainStep(m1, lr=1e-3, mode="eager")
    graph = TrainStep(m2, lr=1e-3, mode="graph", node_bucket=64, edge_bucket=512)
    rng = np.random.default_rng(1)
    for _ in range(4):
        idx = list(rng.choice(len(store), 4, replace=False))
        le = float(eager(store, idx)[0])
        lg = float(graph(store, idx)[0])
        assert abs(le - lg) <= 1e-3 * max(1.0, abs(le)), (le, lg)
    assert graph.graphs, "the DimeNet step was not captured"


@pytest.mark.gpu
def test_dimenet_static_triplets_device_matches_cpu():
    """csrc/graph.hip triplets_static_* == the CPU twin (indices, CSR views, limit)."""
    from hydragnn_amd.models.dimenet import triplets_static

    samples = _samples()
    store = DeviceGraphStore(samples, "cpu")
    idx = [0, 3, 5, 7]
    N, E = store.sizes_of(idx)
    lay = store.layout(idx, Np=N + 9, Ep=E + 40, Gp=len(idx) + 1)
    b = store.assemble(store.upload(idx, lay), lay)
    cap = b.get("triplet_cap")()
    a_kj, a_ji = triplets_static(b.dst_si, b.src_si, b.get("node_mask"), cap)
    d = lambda si: si.to("cuda")  # noqa: E731
    b_kj, b_ji = triplets_static(d(b.dst_si), d(b.src_si), b.get("node_mask").cuda(), cap)
    for x, y in ((a_kj, b_kj), (a_ji, b_ji)):
        assert torch.equal(x.index, y.index.cpu()) and torch.equal(x.rowptr, y.rowptr.cpu())
        assert torch.equal(x.limit, y.limit.cpu())
    assert torch.equal(a_kj.perm, b_kj.perm.cpu())
    assert 0 < int(a_kj.limit) <= cap


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mse", "mae"])
def test_fused_energy_force_loss_matches_masked_torch(kind):
    """models/base.py _EFLoss (csrc/conv_misc.hip ef_loss, one launch each way) == the torch
    masked energy + force loss of a padded batch: total, energy loss and both gradients."""
    from hydragnn_amd.models.base import _EF_KIND, _EFLoss
    from hydragnn_amd.train.step import masked_loss

    g = torch.Generator().manual_seed(len(kind))
    G, N, w = 9, 70, 0.7
    ep, et = torch.randn(G, generator=g), torch.randn(G, generator=g)
    fp, ft = torch.randn(N, 3, generator=g), torch.randn(N, 3, generator=g)
    gm = torch.rand(G, generator=g) > 0.2
    nm = torch.rand(N, generator=g) > 0.2
    ep[~gm] = float("nan")  # padding rows never reach the loss
    dev = torch.device("cuda")
    a = [t.to(dev).requires_grad_() for t in (ep, fp)]
    tot, el = _EFLoss.apply(a[0], et.to(dev), gm.to(dev), a[1], ft.to(dev), nm.to(dev), _EF_KIND[kind], w)
    (tot * 1.3 + el * 0.4).backward()
    b = [t.clone().double().requires_grad_() for t in (ep, fp)]
    e_loss = masked_loss(kind, b[0].view(-1, 1), et.double().view(-1, 1), gm)
    f_loss = masked_loss(kind, b[1], ft.double(), nm)
    ge = et.double().abs()[gm].sum() / gm.sum().clamp(min=1)
    fa = ft.double().abs()[nm].sum() / (nm.sum().clamp(min=1) * 3)
    ref = e_loss * w + f_loss * (w * ge / (fa + 1e-8))
    (ref * 1.3 + e_loss * 0.4).backward()
    torch.testing.assert_close(tot.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(el.double().cpu(), e_loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a[0].grad.double().cpu(), torch.nan_to_num(b[0].grad), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a[1].grad.double().cpu(), b[1].grad, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_composite_linear_relu_keeps_splitk():
    """A tall Linear+ReLU in force training stays on the twice-differentiable split-K linear
    (a regression once sent it to F.linear, whose weight gradients are 2-workgroup GEMMs)."""
    from hydragnn_amd.ops.linear import ACT_RELU, MIN_ROWS, linear
    from hydragnn_amd.ops.pna import composite_mode as _cm

    x = torch.randn(max(MIN_ROWS, 4096), 64, device="cuda", requires_grad=True)
    W = torch.nn.Parameter(torch.randn(32, 64, device="cuda"))
    b = torch.nn.Parameter(torch.zeros(32, device="cuda"))
    with _cm(True):
        y = linear(x, W, b, act=ACT_RELU)
    assert "LinearC" in y.grad_fn.next_functions[0][0].name()
    with _cm(True):
        ref = torch.relu(torch.nn.functional.linear(x, W, b))
    torch.testing.assert_close(y, ref)
