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

    if "--taskpar" in sys.argv:
        sys.exit(taskpar(dev, samples, deg))
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


def taskpar(dev, samples, deg):
    """``--taskpar``: TrainStep drives MultiTaskModelMP (branch 0 of 2) in graph mode — two
    bucketed syncs (encoder over WORLD, decoder over a 1-rank branch group created with
    ``new_group``), their all-reduces recorded into the captured step on one comm stream —
    and must equal the same pruned model stepped without any sync, bit for bit."""
    import copy

    import torch
    import torch.distributed as dist

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.models.create import create_model
    from hydragnn_amd.models.multitask import MultiTaskModelMP, prune_branches
    from hydragnn_amd.train.step import TrainStep

    for g in samples:
        g.dataset_name = torch.tensor([[0]])
    hd = {"graph": [{"type": f"branch-{b}", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 16,
                                                              "num_headlayers": 1, "dim_headlayers": [16]}}
                    for b in range(2)]}
    torch.manual_seed(0)
    base = create_model("PNAPlus", 4, 64, [1], 8, "GPS", "multihead", 8, ["graph"], hd, "relu", "mae", [1.0], 3,
                        pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=8.0, max_neighbours=10,
                        dropout=0.0).to(dev)
    plain = copy.deepcopy(base)
    prune_branches(plain, 0)
    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    batches = [list(range(0, 8)), list(range(8, 16)), list(range(16, 24)), list(range(0, 8))]
    group = dist.new_group([0])
    out = {}
    for tag, model, force in (("taskpar", MultiTaskModelMP(base, 0, group), "1"), ("plain", plain, "0")):
        os.environ["HYDRA_GRADSYNC_FORCE"] = force
        step = TrainStep(model, lr=1e-3, mode="graph", world=1, bucket_cap_mb=0.05)
        assert step.mode == "graph"
        syncs = getattr(step.sync, "syncs", [step.sync])
        launched = []
        for k, s in enumerate(syncs):
            s._launch = lambda bi, o=s._launch, k=k: (launched.append((k, bi)), o(bi))[1]
        step.prepare(store, 8)
        losses = [float(step(store, b)[0]) for b in batches]
        torch.cuda.synchronize()
        out[tag] = dict(losses=losses, recorded=launched, captured=len(step.graphs),
                        params=torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu())
    same = torch.equal(out["taskpar"]["params"], out["plain"]["params"])
    groups_recorded = sorted({k for k, _ in out["taskpar"]["recorded"]})
    res = {"mode": "taskpar", "losses_taskpar": out["taskpar"]["losses"], "losses_plain": out["plain"]["losses"],
           "allreduces_recorded": len(out["taskpar"]["recorded"]), "communicators": groups_recorded,
           "graphs": out["taskpar"]["captured"], "params_bitwise_equal": same}
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    ok = same and groups_recorded == [0, 1] and out["taskpar"]["captured"] >= 1 and not out["plain"]["recorded"]
    print("GRADSYNC_OK" if ok else "GRADSYNC_FAIL", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    main()
