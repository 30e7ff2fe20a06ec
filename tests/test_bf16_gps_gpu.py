"""bf16 mode of the OC20 PNAPlus + GPS configuration (BASELINE config 4 shape, smaller
dataset): the GPS attention products run on bf16 MFMA (csrc/attention8.hip, BF kernels) in the
captured training step, and the training trajectory stays with fp32's: final-loss ratio <= 1.05
after 200 steps on the same batches from the same initial weights (measured on MI355X: 0.9996).
"""
import numpy as np
import pytest
import torch

from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import degree_histogram, oc20_like
from hydragnn_amd.models.create import create_model
from hydragnn_amd.ops.linear import get_precision, set_precision
from hydragnn_amd.train.step import TrainStep

pytestmark = pytest.mark.gpu


def _train(precision, steps=200, B=16):
    dev = torch.device("cuda")
    prev = get_precision()
    set_precision(precision)
    try:
        samples = oc20_like(96, seed=1000, radius=10.0, max_neighbours=10, pe_dim=16)
        deg = degree_histogram(samples, max_degree=10).to(torch.float64)
        heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 50,
                                                                 "num_headlayers": 2, "dim_headlayers": [50, 25]}}]}
        torch.manual_seed(0)
        model = create_model("PNAPlus", 4, 64, [1], 16, "GPS", "multihead", 8, ["graph"], heads, "relu", "mae", [1.0],
                             3, pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=10.0,
                             max_neighbours=10).to(dev)
        store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
        step = TrainStep(model, lr=1e-3, mode="graph")
        step.prepare(store, B)
        rng = np.random.default_rng(5)
        losses = []
        for _ in range(steps):
            idx = rng.choice(len(store), size=B, replace=False).tolist()
            losses.append(step(store, idx)[0].detach().clone())  # (the graph's output buffer is reused)
        return torch.stack([l.float().reshape(()) for l in losses]).cpu().numpy()
    finally:
        set_precision(prev)


def test_bf16_gps_attention_trajectory_matches_fp32():
    l32 = _train("fp32")
    l16 = _train("bf16")
    assert np.all(np.isfinite(l16))
    f32, f16 = float(l32[-20:].mean()), float(l16[-20:].mean())
    ratio = f16 / f32
    print(f"loss first/last 20 steps: fp32 {l32[:20].mean():.4f} -> {f32:.4f}  bf16 {l16[:20].mean():.4f} -> "
          f"{f16:.4f}  ratio {ratio:.4f}")
    assert ratio <= 1.05, ratio
    # the whole trajectory too, in 20-step windows (single steps of a random-batch MAE are noisy)
    w32, w16 = l32.reshape(-1, 20).mean(1), l16.reshape(-1, 20).mean(1)
    assert np.all(np.abs(w16 / w32 - 1.0) < 0.05), w16 / w32
