"""The grouped weight-gradient launch of the headline step (OC20 PNAPlus + GPS), replayed
in isolation: records the (dY, X) problem list of one real training step's
``linear_wgrad_grouped`` call and times it whole, its wide (I > 16) and narrow (I <= 16)
parts, and one launch per problem.  Usage: python tools/bench_wgrad_step.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402
from tools.bench_ops import graph_time  # noqa: E402


class _Rec:
    def __init__(self, ops):
        self._ops = ops
        self.calls = []

    def __getattr__(self, k):
        f = getattr(self._ops, k)
        if k != "linear_wgrad_grouped":
            return f

        def rec(dys, xs, dws, dbs, acc):
            self.calls.append([(dy.clone(), x.clone(), dw.shape, db.numel()) for dy, x, dw, db in zip(dys, xs, dws, dbs)])
            return f(dys, xs, dws, dbs, acc)
        return rec


def main():
    from hydragnn_amd.data.synthetic import oc20_like, degree_histogram
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.models.create import create_model
    from hydragnn_amd.ops import gps_encoder
    from hydragnn_amd.train.step import TrainStep

    dev = torch.device("cuda")
    samples = oc20_like(128, seed=1000, radius=10.0, max_neighbours=10, pe_dim=16)
    deg = degree_histogram(samples, max_degree=10).to(torch.float64)
    heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 50,
                                                             "num_headlayers": 2, "dim_headlayers": [50, 25]}}]}
    model = create_model("PNAPlus", 4, 64, [1], 16, "GPS", "multihead", 8, ["graph"], heads, "relu", "mae", [1.0], 3,
                         pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=10.0,
                         max_neighbours=10).to(dev)
    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    step = TrainStep(model, lr=1e-3, mode="eager")
    rec = _Rec(_native.ops())
    orig = gps_encoder._native.ops
    gps_encoder._native.ops = lambda: rec
    try:
        step(store, list(np.arange(32)))
    finally:
        gps_encoder._native.ops = orig
    torch.cuda.synchronize()
    probs = rec.calls[-1]
    ops = _native.ops()
    print(f"{len(probs)} problems")
    for dy, x, shp, nb in probs:
        print(f"  M {dy.shape[0]:6d}  O {dy.shape[1]:4d}  I {x.shape[1]:4d}  bias {nb > 0}")

    def run(sel):
        dys = [probs[k][0] for k in sel]
        xs = [probs[k][1] for k in sel]
        dws = [torch.empty(probs[k][2], device=dev) for k in sel]
        dbs = [torch.empty(probs[k][3], device=dev) for k in sel]
        return graph_time(lambda: ops.linear_wgrad_grouped(dys, xs, dws, dbs, [0] * len(sel)))

    allk = list(range(len(probs)))
    wide = [k for k in allk if probs[k][1].shape[1] > 16]
    narrow = [k for k in allk if probs[k][1].shape[1] <= 16]
    print(f"all {run(allk):7.1f} us   wide {run(wide):7.1f} us   narrow {run(narrow):7.1f} us", flush=True)
    for k in allk:
        dy, x = probs[k][0], probs[k][1]
        print(f"  single M {dy.shape[0]:6d} O {dy.shape[1]:4d} I {x.shape[1]:4d}: {run([k]):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
