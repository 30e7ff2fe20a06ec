"""RCCL probe: plain all-reduce, and an all-reduce captured into a hipGraph on a side
(comm) stream forked from / joined to the capture stream — the structure the
training step uses (``parallel.ddp.BucketedGradSync``).  Run under torchrun:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/rccl_probe.py

With N ranks on ONE device this also tells whether RCCL accepts several ranks per GPU.
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.parallel.distributed import rccl_env  # noqa: E402


def main():
    rccl_env()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    dist.init_process_group("nccl", device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    x = torch.full((1 << 18,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    print(f"[{rank}] eager all_reduce ok={bool((x == want).all())} val={float(x[0])}", flush=True)

    comm = torch.cuda.Stream(priority=-1)
    buf = torch.zeros(1 << 18, device=dev)
    src = torch.full_like(buf, float(rank + 1))
    other = torch.zeros(1 << 20, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        buf.copy_(src)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        buf.copy_(src)
        buf.mul_(1.0 / world)
        comm.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(comm):
            dist.all_reduce(buf)
        other.add_(1.0)  # independent work on the capture stream (overlaps the collective)
        torch.cuda.current_stream().wait_stream(comm)
        buf.add_(0.0)
    for it in range(5):
        g.replay()
    torch.cuda.synchronize()
    want = sum(r + 1 for r in range(world)) / world
    ok = bool(torch.allclose(buf, torch.full_like(buf, want))) and float(other[0]) == 5.0
    print(f"[{rank}] captured all_reduce ok={ok} val={float(buf[0])} want={want}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
