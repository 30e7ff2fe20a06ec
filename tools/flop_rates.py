"""FLOP rate of every GEMM-shaped op of a ``bench_configs`` configuration's training step.

Runs eager steps (the same kernels the captured step replays, attributed to their ops) under
the torch profiler with input shapes, and prints per (op, shapes): calls per step, device
time per call, GFLOP per call and the achieved TFLOP/s against the fp32 matrix peak of an
MI355X (157 TF/s: 256 CUs x 4 SIMDs x 64 FLOP/clk of v_mfma_f32_16x16x4 x 2.4 GHz).  The
grouped weight-gradient op (``hydra::linear_wgrad_grouped``, one launch pair for every
deferred dW = dY^T X of the step) is counted from its operand lists.

Usage: python tools/flop_rates.py multibranch_egnn [--steps 3] [--single-branch]
"""
import argparse
import collections
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_configs as bc  # noqa: E402
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.train.step import TrainStep  # noqa: E402

PEAK_TF = 157.0


def _flops(name, shapes):
    """2*M*N*K for the GEMM-shaped aten ops (None for anything else)."""
    try:
        if name in ("aten::mm",):
            (m, k), (_, n) = shapes[0], shapes[1]
            return 2.0 * m * n * k
        if name in ("aten::addmm", "aten::_addmm_activation"):
            (m, k), (_, n) = shapes[1], shapes[2]
            return 2.0 * m * n * k
        if name in ("aten::bmm",):
            (b, m, k), (_, _, n) = shapes[0], shapes[1]
            return 2.0 * b * m * n * k
    except (ValueError, IndexError, TypeError):
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--single-branch", action="store_true")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    model, samples, B, ht, hd, forces = bc.CONFIGS[a.name](dev)
    model = model.to(dev)
    if not forces:
        samples = bc._targets_for_store(samples, ht)
    store = DeviceGraphStore(samples, dev, head_types=None if forces else ht, head_dims=None if forces else hd)
    ts = TrainStep(model, lr=1e-3, mode="eager", compute_grad_energy=forces)
    rng = np.random.default_rng(0)
    pools = None
    if a.single_branch and store.dataset_name is not None:
        dn = store.dataset_name.reshape(-1)
        pools = [np.flatnonzero(dn == b) for b in np.unique(dn)]
    turn = [0]

    def draw():
        if pools is None:
            return list(rng.choice(len(store), size=B, replace=False))
        p = pools[turn[0] % len(pools)]
        turn[0] += 1
        return list(rng.choice(p, size=min(B, len(p)), replace=False))

    # grouped weight gradients: FLOPs from the operand lists, recorded at the call
    from hydragnn_amd import _native

    ops = _native.ops()
    grouped = []
    orig = ops.linear_wgrad_grouped

    def spy(dys, xs, dws, dbs, modes, *rest):
        grouped.append(sum(2.0 * dy.shape[0] * dy.shape[1] * x.shape[1] for dy, x in zip(dys, xs)))
        return orig(dys, xs, dws, dbs, modes, *rest)

    for _ in range(3):
        ts(store, draw())
    torch.cuda.synchronize()
    grouped.clear()
    ops.linear_wgrad_grouped = spy
    try:
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            for _ in range(a.steps):
                ts(store, draw())
            torch.cuda.synchronize()
    finally:
        ops.linear_wgrad_grouped = orig
    S = a.steps
    rows = collections.defaultdict(lambda: [0, 0.0, 0.0])
    total_dev = 0.0
    for e in prof.key_averages(group_by_input_shape=True):
        dt = getattr(e, "self_device_time_total", None)
        if dt is None:
            dt = e.self_cuda_time_total
        total_dev += dt
        if e.key.startswith("hydra::linear_wgrad_grouped"):
            rows[("hydra::linear_wgrad_grouped", "(grouped dW = dY^T X)")] = [e.count, dt, sum(grouped)]
            continue
        f = _flops(e.key, e.input_shapes)
        if f is None:
            continue
        r = rows[(e.key, str(e.input_shapes[:3]))]
        r[0] += e.count
        r[1] += dt
        r[2] += f * e.count
    print(f"{a.name}: {S} eager steps, device time {total_dev / 1e3 / S:.3f} ms/step (all ops); "
          f"fp32 matrix peak {PEAK_TF:.0f} TF/s")
    print(f"{'calls/st':>8} {'us/call':>9} {'ms/step':>8} {'GFLOP/st':>9} {'TF/s':>7} {'%peak':>6}  op  shapes")
    gem_t = gem_f = 0.0
    for (k, shp), (n, dt, fl) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        tf = fl / max(dt, 1e-9) / 1e6  # FLOP / us -> TF/s
        gem_t += dt
        gem_f += fl
        print(f"{n / S:8.1f} {dt / max(n, 1):9.1f} {dt / 1e3 / S:8.3f} {fl / 1e9 / S:9.2f} {tf:7.1f} "
              f"{100 * tf / PEAK_TF:6.1f}  {k}  {shp[:90]}")
    print(f"GEMM-shaped total: {gem_t / 1e3 / S:.3f} ms/step, {gem_f / 1e9 / S:.1f} GFLOP/step, "
          f"{gem_f / max(gem_t, 1e-9) / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
