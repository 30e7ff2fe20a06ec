"""Native packed batch plan (``csrc/collate.cpp`` store_plan, the per-step host work of the
captured training step) against the numpy reference ``DeviceGraphStore.plan_numpy``:
bit-identical int32 plans for random draws, padded and unpadded layouts, batch and graph
attention scopes.  CPU only (host code)."""
import numpy as np
import pytest
import torch

from hydragnn_amd import _native
from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import oc20_like

pytestmark = pytest.mark.skipif(not _native.available(), reason="native library not built")


@pytest.mark.parametrize("scope", ["batch", "graph"])
@pytest.mark.parametrize("padded", [True, False])
def test_native_plan_matches_numpy(scope, padded):
    samples = oc20_like(40, seed=3, radius=6.0, max_neighbours=8, pe_dim=4)
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1], attn_scope=scope)
    rng = np.random.default_rng(0)
    for trial in range(12):
        G = int(rng.integers(1, 12))
        idx = list(rng.choice(len(store), G, replace=False))
        N, E = store.sizes_of(idx)
        if padded:
            lay = store.layout(idx, Np=(N + 2 + 31) // 32 * 32 + 32 * (trial % 2), Ep=E + 7 * trial,
                               Gp=G + 1 + trial % 3)
        else:
            lay = store.layout(idx)
        a = store.plan(idx, lay, np.full(lay.total, -7, dtype=np.int32))
        b = store.plan_numpy(idx, lay, np.full(lay.total, -7, dtype=np.int32))
        np.testing.assert_array_equal(a, b)


def test_native_plan_rejects_overflow():
    samples = oc20_like(8, seed=1, radius=6.0, max_neighbours=8, pe_dim=4)
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1])
    idx = [0, 1, 2]
    N, E = store.sizes_of(idx)
    lay = store.layout(idx)
    small = torch.zeros(lay.total - 1, dtype=torch.int32)
    with pytest.raises(RuntimeError):
        _native.ops().store_plan(torch.tensor(idx), *store._native_plan_args(), small, lay.Np, lay.Ep, lay.Gp,
                                 False, True)
