"""Where do the bucket all-reduces sit in the training step's backward?  (1-rank RCCL.)

The captured step records each gradient bucket's all-reduce on the comm stream when the
bucket's last gradient arrives (parallel/ddp.py BucketedGradSync); every backward kernel
enqueued after that point can run while RCCL moves the bucket.  This tool runs the captured
step's exact computation eagerly (``TrainStep.padded_step``) on a 1-rank ``nccl`` group with
HYDRA_GRADSYNC_FORCE=1 under the torch profiler and counts, in host launch order (the order
the captured graph preserves), the backward kernel launches that follow the FIRST bucket's
all-reduce.  A 1-rank all-reduce moves no data, so only the position is measured.

    python tools/overlap_check.py [--config multibranch_egnn] [--precision bf16]

Prints one JSON line: per bucket its bytes and the backward launches after its all-reduce,
and the headline ``bytes_overlapped_fraction``: the share of gradient bytes whose all-reduce
is enqueued before the last 20 % of the backward launches.  Run as its own process."""
import argparse
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="multibranch_egnn")
    ap.add_argument("--precision", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--bucket-mb", type=float, default=None)
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      HYDRA_GRADSYNC_FORCE="1")
    import numpy as np
    import torch
    import torch.distributed as dist
    from torch.profiler import ProfilerActivity, profile, record_function

    from hydragnn_amd.parallel.distributed import rccl_env

    rccl_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)

    import bench_configs as bc
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.ops.linear import set_precision
    from hydragnn_amd.train.step import TrainStep

    set_precision(a.precision)
    model, samples, B, ht, hd, forces = bc.CONFIGS[a.config](dev)
    model = model.to(dev)
    if not forces:
        samples = bc._targets_for_store(samples, ht)
    store = DeviceGraphStore(samples, dev, head_types=None if forces else ht, head_dims=None if forces else hd)
    nbk = 512
    cap = a.bucket_mb
    if cap is None:
        # the bucket size a multi-rank run picks (ddp.default_bucket_cap); a lone rank would
        # otherwise keep one bucket
        from hydragnn_amd.parallel.ddp import default_bucket_cap

        nbytes = 4 * sum(p.numel() for p in model.parameters() if p.requires_grad)
        cap = default_bucket_cap(nbytes) / (1024 * 1024)
    ts = TrainStep(model, lr=1e-3, mode="graph", world=1, node_bucket=nbk, edge_bucket=8 * nbk,
                   bucket_cap_mb=cap, compute_grad_energy=forces)
    syncs = getattr(ts.sync, "syncs", [ts.sync])
    for k, s in enumerate(syncs):
        def launch(bi, o=s._launch, k=k):
            with record_function(f"gradsync_bucket_{k}_{bi}"):
                return o(bi)
        s._launch = launch
    orig_bwd = ts._backward

    def bwd(loss, sync=True):
        with record_function("hydra_backward"):
            return orig_bwd(loss, sync=sync)
    ts._backward = bwd
    rng = np.random.default_rng(0)
    draw = lambda: list(rng.choice(len(store), size=B, replace=False))  # noqa: E731
    for _ in range(2):
        ts.padded_step(store, draw())
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        ts.padded_step(store, draw())
        torch.cuda.synchronize()
    ev = prof.events()
    win = [e for e in ev if e.name == "hydra_backward"]
    assert win, "no backward marker"
    b0, b1 = win[0].time_range.start, win[0].time_range.end
    launches = sorted(e.time_range.start for e in ev
                      if "LaunchKernel" in e.name and b0 <= e.time_range.start <= b1)
    first = {}
    for e in ev:  # one marker per bucket launch (the profiler may report a range twice)
        if e.name.startswith("gradsync_bucket_"):
            first[e.name] = min(first.get(e.name, e.time_range.start), e.time_range.start)
    ars = sorted((t, n) for n, t in first.items())
    after = [sum(1 for t in launches if t > s0) for s0, _ in ars]
    nb = max(len(launches), 1)

    def nbytes(name):
        k, bi = (int(v) for v in name[len("gradsync_bucket_"):].split("_"))
        s0, e0, _ = syncs[k].buckets[bi]
        return 4 * (e0 - s0)

    per = [{"bucket": n[len("gradsync_bucket_"):], "bytes": nbytes(n), "launches_after": c,
            "fraction_after": round(c / nb, 4)} for (_, n), c in zip(ars, after)]
    total = sum(b["bytes"] for b in per) or 1
    # headline: the share of gradient BYTES whose all-reduce is enqueued before the last 20 %
    # of the backward kernel launches (those reduces have >= 20 % of backward left to hide in)
    over = sum(b["bytes"] for b in per if b["fraction_after"] >= 0.2)
    res = {"config": a.config, "precision": a.precision, "buckets": sum(len(s.buckets) for s in syncs),
           "allreduces": len(ars), "backward_kernel_launches": len(launches),
           "bytes_overlapped_fraction": round(over / total, 4), "gradient_bytes": total,
           "per_bucket": per, "launches_after_each_allreduce": after,
           "fraction_after_first": round(after[0] / nb, 4) if after else 0.0}
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
