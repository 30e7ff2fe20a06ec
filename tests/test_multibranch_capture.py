"""Multi-branch models on the captured (statically padded) training step.

The reference decodes a multi-dataset batch by masking graphs per branch
(``Base.py:482-560``); the host-side branch ranges used by the eager store path change
from batch to batch, so the captured step decodes densely instead: every branch head on
every row, selected per row by the dataset id on the device (``Base._decode_dense``).
A batch of ONE branch (every batch of an SC25 rank, which loads one dataset) is captured
under a branch-keyed bucket and decodes only that branch's heads.
Checks: padded step (the CPU twin of the captured step) == eager step, on CPU for
EGNN / SchNet / MACE, and captured == eager on the GPU, mixed and single-branch batches."""
import copy

import numpy as np
import pytest
import torch

from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import oc20_like
from hydragnn_amd.models.create import create_model
from hydragnn_amd.train.step import TrainStep

NB = 3


def _data(n=18):
    s = oc20_like(n, seed=20, radius=5.0, max_neighbours=8, pe_dim=2, min_atoms=5, max_atoms=10)
    from hydragnn_amd.data.transforms import radius_graph

    for i, g in enumerate(s):
        # the models' own radius / cap (index policy): SchNet's captured step uses these edges
        g.edge_index = radius_graph(g.pos, 5.0, max_num_neighbors=8)
        g.edge_attr = None
        g.sort_edges_by_dst()
        g.dataset_name = torch.tensor([[i % NB]])
        g.x = torch.randint(1, 9, (g.x.shape[0], 1)).float()
        g.y = torch.cat([g.y.view(-1)[:1], torch.sin(g.pos[:, 0])])
        g.y_loc = torch.tensor([[0, 1, 1 + g.num_nodes]])
    return s


def _model(mt):
    heads = {"graph": [{"type": f"branch-{b}", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 8,
                                                                  "num_headlayers": 1, "dim_headlayers": [8]}}
                       for b in range(NB)],
             "node": [{"type": f"branch-{b}", "architecture": {"num_headlayers": 1, "dim_headlayers": [8],
                                                                 "type": "mlp"}} for b in range(NB)]}
    torch.manual_seed(0)
    return create_model(mt, 1, 12, [1, 1], 2, "", "multihead", 1, ["graph", "node"], heads, "relu", "mse",
                        [1.0, 1.0], 2, use_gpu=False, edge_dim=None, dropout=0.0, radius=5.0, num_radial=5,
                        num_gaussians=8, num_filters=12, max_neighbours=8, envelope_exponent=5, max_ell=1,
                        node_max_ell=1, avg_num_neighbors=5.0, correlation=2)


def _compare(mt, dev, tol, plan=(None,) * 4):
    """``plan``: per step, the branch id every graph of the batch comes from (an SC25 rank's
    batches; the branch-keyed captured step), or None for a mixed batch."""
    samples = _data()
    m1 = _model(mt).to(dev)
    m2 = copy.deepcopy(m1)
    store = DeviceGraphStore(samples, dev, head_types=["graph", "node"], head_dims=[1, 1])
    eager = TrainStep(m1, lr=1e-3, mode="eager")
    cap = TrainStep(m2, lr=1e-3, mode="graph", node_bucket=64, edge_bucket=256)
    assert cap.mode == "graph"
    rng = np.random.default_rng(0)
    for b in plan:
        pool = np.arange(len(samples)) if b is None else np.arange(b, len(samples), NB)
        idx = list(rng.choice(pool, min(6, len(pool)), replace=False))
        le, lc = float(eager(store, idx)[0]), float(cap(store, idx)[0])
        assert abs(le - lc) <= tol * max(1.0, abs(le)), (le, lc)
    # heads of branches absent from a step kept torch's skip-if-no-grad semantics
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p1, p2, rtol=100 * tol, atol=100 * tol)
    return cap


@pytest.mark.parametrize("mt", ["EGNN", "SchNet", "MACE"])
def test_multibranch_padded_step_equals_eager(mt):
    _compare(mt, "cpu", 1e-4)


SC25_PLAN = (0, 1, 0, 2, None, 1)  # single-branch batches, one mixed


@pytest.mark.parametrize("mt", ["EGNN", "MACE"])
@pytest.mark.parametrize("dense", ["1", "0"])
def test_multibranch_branch_keyed_padded_step_equals_eager(mt, dense, monkeypatch):
    """Single-branch batches decode only their branch's heads under a branch-keyed bucket;
    a mixed batch takes the dense decode (dense=1) or an eager step (dense=0)."""
    monkeypatch.setenv("HYDRA_MULTIBRANCH_CAPTURE", dense)
    cap = _compare(mt, "cpu", 1e-4, SC25_PLAN)
    assert cap.branch_keyed and cap.dense_ok == (dense == "1")


def test_multibranch_capture_policy(monkeypatch):
    m = _model("EGNN")
    ts = TrainStep(m, mode="graph")
    assert ts.mode == "graph" and ts.dense_ok and ts.branch_keyed  # small model: dense capture
    monkeypatch.setenv("HYDRA_MULTIBRANCH_CAPTURE", "0")
    ts = TrainStep(m, mode="graph")
    assert ts.mode == "graph" and not ts.dense_ok  # single-branch batches still capture
    monkeypatch.setenv("HYDRA_BRANCH_KEYED", "0")
    assert TrainStep(m, mode="graph").mode == "eager"


@pytest.mark.gpu
@pytest.mark.parametrize("mt", ["EGNN", "MACE"])
def test_multibranch_captured_step_equals_eager_gpu(mt):
    _compare(mt, "cuda", 2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("mt", ["EGNN", "MACE"])
@pytest.mark.parametrize("dense", ["1", "0"])
def test_multibranch_branch_keyed_captured_equals_eager_gpu(mt, dense, monkeypatch):
    monkeypatch.setenv("HYDRA_MULTIBRANCH_CAPTURE", dense)
    cap = _compare(mt, "cuda", 2e-3, SC25_PLAN)
    keys = set(cap.graphs)
    assert {k[2] for k in keys} >= {0, 1, 2}  # one capture per branch (same bucket)
    assert (None in {k[2] for k in keys}) == (dense == "1")


@pytest.mark.gpu
def test_multibranch_bf16_grouped_heads_captured_vs_eager_gpu():
    """bf16: the captured step decodes branch-grouped (ops.bgemm.branch_mlp for graph and
    node heads, rows sorted by branch) on the wide-EGNN encoder; the eager step decodes
    per-branch ranges with BF16Linear.  Same losses within bf16 tolerance."""
    from hydragnn_amd.ops.linear import precision

    heads = {"graph": [{"type": f"branch-{b}", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 32,
                                                                  "num_headlayers": 2, "dim_headlayers": [160, 160]}}
                       for b in range(NB)],
             "node": [{"type": f"branch-{b}", "architecture": {"num_headlayers": 2, "dim_headlayers": [160, 160],
                                                                 "type": "mlp"}} for b in range(NB)]}
    with precision("bf16"):
        torch.manual_seed(0)
        m1 = create_model("EGNN", 1, 128, [1, 1], 2, "", "multihead", 1, ["graph", "node"], heads, "relu", "mse",
                          [1.0, 1.0], 2, edge_dim=None, dropout=0.0, radius=5.0, max_neighbours=8,
                          equivariance=True).cuda()
        m2 = copy.deepcopy(m1)
        samples = _data()
        store = DeviceGraphStore(samples, "cuda", head_types=["graph", "node"], head_dims=[1, 1])
        eager = TrainStep(m1, lr=1e-3, mode="eager")
        cap = TrainStep(m2, lr=1e-3, mode="graph", node_bucket=64, edge_bucket=256)
        assert cap.mode == "graph"
        rng = np.random.default_rng(0)
        for _ in range(4):
            idx = list(rng.choice(len(samples), 6, replace=False))
            le, lc = float(eager(store, idx)[0]), float(cap(store, idx)[0])
            assert abs(le - lc) <= 3e-2 * max(1.0, abs(le)), (le, lc)


def test_mace_stacked_dense_decode_matches_branch_loop(monkeypatch):
    """MACE's dense multi-branch read-out runs the branches stacked (one GEMM per layer for
    all branches + a per-row gather); gradients equal the per-branch torch.where loop."""
    from hydragnn_amd.models.mace import MultiheadDecoderBlock

    samples = _data()
    m = _model("MACE")
    store = DeviceGraphStore(samples, "cpu", head_types=["graph", "node"], head_dims=[1, 1])
    ts = TrainStep(m, lr=1e-3, mode="eager")
    idx = store.branch_order(list(range(7)))[0]
    Np, Ep = ts.bucket_of(*store.sizes_of(idx))
    lay = store.layout(idx, Np=Np, Ep=Ep, Gp=len(idx) + 1)
    buf = store.upload(idx, lay)
    calls = []
    orig = MultiheadDecoderBlock._stacked_dense

    def spy(self, *a, **kw):
        out = orig(self, *a, **kw)
        calls.append(out is not None)
        return out

    def run():
        m.zero_grad(set_to_none=True)
        loss, _ = ts._loss(store.assemble(buf, lay, branch_sorted=True))
        loss.backward()
        return float(loss), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    monkeypatch.setattr(MultiheadDecoderBlock, "_stacked_dense", spy)
    l1, g1 = run()
    assert calls and all(calls)
    monkeypatch.setattr(MultiheadDecoderBlock, "_stacked_dense", lambda self, *a, **kw: None)
    l2, g2 = run()
    assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l2))
    assert g1.keys() == g2.keys()
    for k in g1:
        torch.testing.assert_close(g1[k], g2[k], rtol=1e-4, atol=1e-6, msg=k)


def test_absent_branch_heads_skip_update_like_eager():
    """Heads of a branch absent from a batch: the eager step leaves them alone (grad is
    None -> AdamW skips them, no weight / moment decay); the captured step (here its CPU
    twin, the padded step) gets the same through the per-branch usage flags packed with the
    gradients -> every parameter and its AdamW state match after steps that miss branches."""
    samples = _data()
    m1 = _model("EGNN")
    m2 = copy.deepcopy(m1)
    store = DeviceGraphStore(samples, "cpu", head_types=["graph", "node"], head_dims=[1, 1])
    eager = TrainStep(m1, lr=1e-2, mode="eager", weight_decay=0.1)
    cap = TrainStep(m2, lr=1e-2, mode="graph", node_bucket=64, edge_bucket=256, weight_decay=0.1)
    assert cap.mode == "graph" and cap.sync.nflags == NB
    by_branch = {b: [i for i in range(len(samples)) if i % NB == b] for b in range(NB)}
    batches = [by_branch[0][:3] + by_branch[1][:2], by_branch[1][2:5], by_branch[0][3:5] + by_branch[2][:3]]
    absent2 = [p.detach().clone() for p in m2.branch_param_groups()[2]]
    for k, idx in enumerate(batches):
        le, lc = float(eager(store, idx)[0]), float(cap(store, idx)[0])
        assert abs(le - lc) <= 1e-4 * max(1.0, abs(le)), (k, le, lc)
        if k < 2:  # branch 2 not seen yet: its parameters are exactly the initial values
            for a, b in zip(absent2, m2.branch_param_groups()[2]):
                assert torch.equal(a, b)
    # branch heads: compared tightly (the point of this test); encoder weights see ~1e-6
    # gradient differences between the padded and eager batches, which Adam's normalisation
    # can turn into lr-sized update differences on near-zero gradient entries
    for g1, g2 in zip(m1.branch_param_groups(), m2.branch_param_groups()):
        for a, b in zip(g1, g2):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-2, atol=2e-2, msg=n)
