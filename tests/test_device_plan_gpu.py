"""Device-side batch plan (csrc/assemble.hip store_plan_expand, data/device_store.py
plan_device): from the sample ids alone it must produce exactly the host builder's packed plan
(store_plan: node / edge rows, src / dst, source permutation, both CSR row pointers, batch,
graph pointers, attention segments, sample ids, scalars), padded or not, batch or graph
attention scope."""
import numpy as np
import pytest
import torch

from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import oc20_like

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scope", ["batch", "graph"])
@pytest.mark.parametrize("padded", [True, False])
def test_device_plan_matches_host(scope, padded):
    dev = torch.device("cuda")
    samples = oc20_like(40, seed=11, radius=6.0, max_neighbours=8, pe_dim=4, min_atoms=5, max_atoms=30)
    store = DeviceGraphStore(samples, dev, attn_scope=scope)
    rng = np.random.default_rng(3)
    for trial in range(6):
        G = int(rng.integers(1, 24))
        idx = rng.choice(len(samples), size=G, replace=trial % 2 == 0).tolist()
        N, E = store.sizes_of(idx)
        if padded:
            lay = store.layout(idx, Np=N + 2 + int(rng.integers(0, 300)), Ep=E + int(rng.integers(0, 3000)),
                               Gp=G + 1 + int(rng.integers(0, 4)))
        else:
            lay = store.layout(idx)
        host = store.plan(idx, lay)
        seed = np.zeros(lay.Gp + 1, dtype=np.int32)
        store.seed(idx, lay, seed)
        out = torch.full((lay.total,), -7, dtype=torch.int32, device=dev)
        store.plan_device(torch.from_numpy(seed).to(dev), lay, out)
        got = out.cpu().numpy()
        assert np.array_equal(got, host), (trial, np.flatnonzero(got != host)[:10])


def test_device_plan_padded_edges_without_slack():
    """pe = 0 (no padded edges) and the smallest padded node tail."""
    dev = torch.device("cuda")
    samples = oc20_like(10, seed=2, radius=6.0, max_neighbours=8, pe_dim=4, min_atoms=5, max_atoms=20)
    store = DeviceGraphStore(samples, dev)
    idx = [0, 3, 5]
    N, E = store.sizes_of(idx)
    lay = store.layout(idx, Np=N + 2, Ep=E, Gp=4)
    seed = np.zeros(lay.Gp + 1, dtype=np.int32)
    store.seed(idx, lay, seed)
    out = torch.empty(lay.total, dtype=torch.int32, device=dev)
    store.plan_device(torch.from_numpy(seed).to(dev), lay, out)
    assert np.array_equal(out.cpu().numpy(), store.plan(idx, lay))
