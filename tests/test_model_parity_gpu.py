"""GPU == CPU parity of every model family (HIP kernels vs the plain-torch reference
paths of the same modules): one forward + backward on identical weights and batch,
graph + node heads (``mlp`` and ``conv`` node heads), with and without GPS.

The batches are large enough (48 graphs, ~5k edges) to route the tall linears
through the split-K weight-gradient kernel and the segment ops through their
vectorised variants."""
import copy

import pytest
import torch

from hydragnn_amd.data.graph import collate
from hydragnn_amd.data.synthetic import degree_histogram, oc20_like
from hydragnn_amd.models.create import create_model

pytestmark = pytest.mark.gpu

ALL = ["GIN", "SAGE", "MFC", "PNA", "PNAPlus", "GAT", "CGCNN", "SchNet", "DimeNet", "EGNN", "PAINN", "PNAEq", "MACE"]


def _heads(node_type):
    return {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 8,
                                                             "num_headlayers": 2, "dim_headlayers": [8, 8]}}],
            "node": [{"type": "branch-0", "architecture": {"num_headlayers": 2, "dim_headlayers": [8, 8],
                                                            "type": node_type}}]}


def _samples(n, atomic=False):
    s = oc20_like(n, seed=7, radius=5.0, max_neighbours=10, pe_dim=4, min_atoms=8, max_atoms=20)
    for g in s:
        g.edge_attr = torch.ones(g.edge_index.shape[1], 1)
        if atomic:
            g.x = torch.randint(1, 9, (g.x.shape[0], 1)).float()
    return s


def _model(mt, samples, gps, node_type):
    deg = degree_histogram(samples, max_degree=10)
    in_dim = samples[0].x.shape[1]
    hidden = in_dim if (mt == "CGCNN" and not gps) else 16
    torch.manual_seed(0)
    return create_model(mt, in_dim, hidden, [1, 1], 4, "GPS" if gps else "", "multihead", 2, ["graph", "node"],
                        _heads(node_type), "relu", "mse", [1.0, 1.0], 2, pna_deg=deg, edge_dim=1 if gps else None,
                        envelope_exponent=5, num_radial=5, radius=5.0, max_neighbours=10, num_gaussians=8,
                        num_filters=16, basis_emb_size=4, int_emb_size=8, out_emb_size=8, num_after_skip=1,
                        num_before_skip=1, num_spherical=3, use_gpu=False, max_ell=2, node_max_ell=1,
                        avg_num_neighbors=5.0, correlation=2, dropout=0.0)


def _run(m, b):
    m.train()
    pred = m(b)
    loss = sum(p.pow(2).mean() for p in pred)
    loss.backward()
    return loss.detach()


@pytest.mark.parametrize("mt", ALL)
@pytest.mark.parametrize("node_type", ["mlp", "conv"])
@pytest.mark.parametrize("gps", [False, True])
def test_gpu_matches_cpu(mt, node_type, gps):
    if node_type == "conv" and mt in ("CGCNN", "MACE"):
        pytest.skip("conv node heads are not supported by this stack (reference raises)")
    samples = _samples(48, atomic=(mt == "MACE"))
    m_cpu = _model(mt, samples, gps, node_type)
    m_gpu = copy.deepcopy(m_cpu).cuda()
    b = collate(samples)
    lc = _run(m_cpu, b)
    lg = _run(m_gpu, b.to("cuda"))
    assert torch.isfinite(lg).item()
    torch.testing.assert_close(lg.cpu(), lc, rtol=2e-4, atol=2e-5)
    for (n, a), (_, c) in zip(m_gpu.named_parameters(), m_cpu.named_parameters()):
        if c.grad is None:
            assert a.grad is None or float(a.grad.abs().max()) == 0.0, n
            continue
        assert a.grad is not None, n
        scale = max(1.0, float(c.grad.abs().max()))
        torch.testing.assert_close(a.grad.cpu() / scale, c.grad / scale, rtol=5e-3, atol=5e-4, msg=n)
