"""Op-level attribution of the bench step's kernels (torch.profiler, eager mode).

Usage: python tools/op_profile.py [steps]   -> per-aten-op device time / kernel counts per step
(eager dispatch: the same kernels as the captured hipGraph step, attributed to their ops)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.data.synthetic import degree_histogram, oc20_like  # noqa: E402
from hydragnn_amd.models.create import create_model  # noqa: E402
from hydragnn_amd.train.step import TrainStep  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
padded = "--padded" in sys.argv  # the captured step's computation (static padded buckets), run eagerly
stacks = "--stacks" in sys.argv  # python call sites of the small elementwise kernels
dev = torch.device("cuda:0")
samples = oc20_like(256, seed=1000, radius=10.0, max_neighbours=10, pe_dim=16)
deg = degree_histogram(samples, max_degree=10).to(torch.float64)
heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 50,
                                                         "num_headlayers": 2, "dim_headlayers": [50, 25]}}]}
model = create_model("PNAPlus", 4, 64, [1], 16, "GPS", "multihead", 8, ["graph"], heads, "relu", "mae", [1.0], 3,
                     pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=10.0,
                     max_neighbours=10).to(dev)
store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
step = TrainStep(model, lr=1e-3, mode="eager")
rng = np.random.default_rng(0)
run = step.padded_step if padded else step
for _ in range(3):
    run(store, list(rng.choice(len(store), 32, replace=False)))
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=stacks) as prof:
    for _ in range(steps):
        run(store, list(rng.choice(len(store), 32, replace=False)))
    torch.cuda.synchronize()
ka = prof.key_averages()
rows = []
for e in ka:
    dt = getattr(e, "self_device_time_total", None)
    if dt is None:
        dt = getattr(e, "self_cuda_time_total", 0)
    if dt and dt > 0:
        rows.append((dt / steps, e.count / steps, e.key))
rows.sort(key=lambda r: -r[0])
tot = sum(r[0] for r in rows)
print(f"self device time per step: {tot / 1e3:.3f} ms")
for dt, n, k in rows[:70]:
    print(f"{dt:9.1f} us {n:7.1f}/step  {k[:120]}")
if stacks:  # shapes of the small elementwise ops (autograd accumulation has no python stack)
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in ("aten::add_", "aten::fill_", "aten::add", "aten::copy_", "aten::mul", "aten::where",
                     "aten::cat", "aten::mm", "aten::clamp_min", "aten::sum", "aten::addmv_") and \
                getattr(e, "self_device_time_total", 0) > 0:
            print(f"--- {e.key:16s} {e.count / steps:5.1f}/step {e.self_device_time_total / steps:7.1f} us  "
                  f"{str(e.input_shapes)[:120]}")
