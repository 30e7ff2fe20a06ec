"""1-rank RCCL check of the captured gradient all-reduce path (parallel.ddp.BucketedGradSync).

On one GPU the production multi-GPU step structure is exercised end to end: a 1-rank
``nccl`` (RCCL) process group, HYDRA_GRADSYNC_FORCE=1 so backward's bucket hooks launch
their all-reduces on the comm stream INSIDE the captured step graph (several buckets), and
graph replays.  A 1-rank all-reduce is the identity and the 1/world pre-scale is x1.0, so
the synced step must reproduce the unsynced step bit for bit.  Prints one JSON line and
exits non-zero on a mismatch.  Run as its own process (the test spawns it)."""
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch
    import torch.distributed as dist

    from hydragnn_amd.parallel.distributed import rccl_env

    rccl_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.data.synthetic import degree_histogram, oc20_like
    from hydragnn_amd.models.create import create_model
    from hydragnn_amd.train.step import TrainStep

    samples = oc20_like(24, seed=3, radius=8.0, max_neighbours=10, pe_dim=8, min_atoms=12, max_atoms=40)
    deg = degree_histogram(samples, 10)
    hd = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 16,
                                                           "num_headlayers": 2, "dim_headlayers": [16, 8]}}]}

    def build():
        torch.manual_seed(0)
        return create_model("PNAPlus", 4, 64, [1], 8, "GPS", "multihead", 8, ["graph"], hd, "relu", "mae", [1.0], 3,
                            pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=8.0, max_neighbours=10,
                            dropout=0.0).to(dev)

    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    batches = [list(range(0, 8)), list(range(8, 16)), list(range(16, 24)), list(range(0, 8))]
    out = {}
    for tag, force in (("synced", "1"), ("plain", "0")):
        os.environ["HYDRA_GRADSYNC_FORCE"] = force
        model = build()
        step = TrainStep(model, lr=1e-3, mode="graph", world=1, bucket_cap_mb=0.05)
        launched = []
        orig = step.sync._launch
        step.sync._launch = lambda bi, o=orig: (launched.append(bi), o(bi))[1]
        step.prepare(store, 8)
        losses = [float(step(store, b)[0]) for b in batches]
        torch.cuda.synchronize()
        out[tag] = dict(losses=losses, buckets=len(step.sync.buckets), launched_at_capture=len(launched),
                        params=torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu())
    same = torch.equal(out["synced"]["params"], out["plain"]["params"])
    res = {"rccl_world": dist.get_world_size(), "backend": dist.get_backend(), "buckets": out["synced"]["buckets"],
           "allreduces_recorded": out["synced"]["launched_at_capture"], "plain_recorded": out["plain"]["launched_at_capture"],
           "losses_synced": out["synced"]["losses"], "losses_plain": out["plain"]["losses"], "params_bitwise_equal": same}
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    ok = same and out["synced"]["launched_at_capture"] >= 2 and out["plain"]["launched_at_capture"] == 0
    print("GRADSYNC_OK" if ok else "GRADSYNC_FAIL", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
