"""Step-by-step check of the hipGraph train step: loss per step, bucket, timing."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from hydragnn_amd.data.synthetic import oc20_like, degree_histogram
from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.models.create import create_model
from hydragnn_amd.train.step import TrainStep
dropout = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25
samples = oc20_like(256, seed=1000)
deg = degree_histogram(samples, 10).double()
heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 50, "num_headlayers": 2, "dim_headlayers": [50, 25]}}]}
model = create_model("PNAPlus", 4, 64, [1], 16, "GPS", "multihead", 8, ["graph"], heads, "relu", "mae", [1.0], 3,
                     pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=10.0, max_neighbours=10, dropout=dropout).cuda()
store = DeviceGraphStore(samples, "cuda", head_types=["graph"], head_dims=[1])
step = TrainStep(model, lr=1e-3, mode="graph")
step.prepare(store, 32)
print("expected buckets", step.expected)
rng = np.random.default_rng(0)
for it in range(40):
    idx = rng.choice(len(store), 32, replace=False)
    N, E = store.sizes_of(idx)
    torch.cuda.synchronize(); t = time.perf_counter()
    l, _ = step(store, idx)
    torch.cuda.synchronize(); dt = time.perf_counter() - t
    bad = [n for n, p in model.named_parameters() if not torch.isfinite(p).all()]
    print(it, N, E, step._pick(N, E), "loss", float(l), "ms", round(dt * 1e3, 2), "nonfinite params", bad[:3], flush=True)
    if bad: break
