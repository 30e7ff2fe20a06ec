"""Bisect GPU-vs-CPU training-trajectory differences op family by op family.

Trains the CI-sized PNA+lengths model (hidden 8, lr 0.02) for 25 steps on
the CPU reference path (fp32 and fp64) and on the GPU with every fused HIP op family
switched off one at a time (ops.pna.fused / HYDRA_UNFUSED), then prints the max
per-step loss deviation from the CPU fp32 trajectory.
Usage: python tools/trajectory_bisect.py [model]"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.data.synthetic import degree_histogram, oc20_like  # noqa: E402
from hydragnn_amd.models.create import create_model  # noqa: E402
from hydragnn_amd.ops import pna as mode  # noqa: E402
from hydragnn_amd.optim.adamw import FusedAdamW  # noqa: E402
from hydragnn_amd.train.step import TrainStep  # noqa: E402

MODEL = sys.argv[1] if len(sys.argv) > 1 else "PNA"
samples = oc20_like(96, seed=8, min_atoms=4, max_atoms=12, radius=4.0, max_neighbours=6, pe_dim=1)
e = torch.stack([s["energy"].reshape(()) for s in samples])
for s in samples:
    s["x"] = s["x"][:, :1]
    s["y"] = ((s["energy"].reshape(1) - e.min()) / (e.max() - e.min())).float()
    s["y_loc"] = torch.tensor([[0, 1]])
deg = degree_histogram(samples, 6)
heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 4,
                                                         "num_headlayers": 2, "dim_headlayers": [10, 10]}}]}
base = create_model(MODEL, 1, 8, [1], 1, None, None, 0, ["graph"], heads, "relu", "mse", [1.0], 2, pna_deg=deg,
                    edge_dim=1, use_gpu=False, init_seed=3, num_radial=6, envelope_exponent=5, radius=4.0)


def run(dev, dtype=torch.float32, mode_="graph", off=()):
    if "adamw" in off:
        mode_ = "eager"  # the torch AdamW reads its step counter on the host: not capturable
    mode._state["off"] = set(off)
    m = copy.deepcopy(base).to(dev, dtype)
    st = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1], dtype=dtype)
    t = TrainStep(m, mode=mode_, optimizer=FusedAdamW(m.parameters(), lr=0.02), node_bucket=128, edge_bucket=1024)
    g = torch.Generator().manual_seed(0)
    out = [float(t(st, torch.randperm(96, generator=g)[:32].tolist())[0]) for _ in range(25)]
    mode._state["off"] = set()
    return out


ref = run("cpu")
ref64 = run("cpu", torch.float64)


def dev_(tr):
    return max(abs(a - b) for a, b in zip(ref, tr)), abs(ref[3] - tr[3])


print(f"{'config':40s} {'max|d|':>10s} {'|d| step3':>10s}")
print(f"{'cpu fp64':40s} {dev_(ref64)[0]:10.3e} {dev_(ref64)[1]:10.3e}")
if torch.cuda.is_available():
    fams = ["pna", "wprep", "linear", "mlp", "norm", "radial", "attn", "adamw"]
    for name, kw in [("gpu graph all fused", {}), ("gpu eager all fused", {"mode_": "eager"}),
                     ("gpu graph all unfused", {"off": fams})] + [(f"gpu graph -{f}", {"off": [f]}) for f in fams] + \
            [(f"gpu graph only {f}", {"off": [x for x in fams if x != f]}) for f in fams]:
        d = dev_(run("cuda", **kw))
        print(f"{name:40s} {d[0]:10.3e} {d[1]:10.3e}", flush=True)
