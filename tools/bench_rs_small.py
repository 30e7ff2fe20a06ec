"""Time the one-workgroup static radius-graph builder (csrc/graph.hip rs_small_kernel)
against the multi-launch builder on QM9-shaped padded batches of growing size."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.ops.radius import interaction_graph_static  # noqa: E402


class D(dict):
    def get(self, k, d=None):
        return dict.get(self, k, d)


def batch(G, seed=0):
    g = torch.Generator().manual_seed(seed)
    sizes = [int(x) for x in torch.randint(9, 29, (G,), generator=g)]
    pos = torch.cat([torch.rand(n, 3, generator=g) * 4 for n in sizes] + [torch.zeros(8, 3)])
    b = torch.cat([torch.full((n,), i) for i, n in enumerate(sizes)] + [torch.full((8,), G)])
    ptr = torch.tensor([0] + torch.tensor(sizes + [8]).cumsum(0).tolist())
    mask = torch.cat([torch.ones(sum(sizes), dtype=torch.bool), torch.zeros(8, dtype=torch.bool)])
    d = D(node_mask=mask.cuda())
    d.batch, d.ptr = b.cuda(), ptr.cuda()
    return pos.cuda(), d


for G in (4, 16, 64, 128, 256):
    pos, d = batch(G)
    for small in ("1", "0"):
        os.environ["HYDRA_RS_SMALL"] = small
        for _ in range(3):
            interaction_graph_static(pos, d, 5.0, 5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            interaction_graph_static(pos, d, 5.0, 5)
        torch.cuda.synchronize()
        print(f"G {G:4d} N {pos.shape[0]:5d} small={small}: {1e6 * (time.perf_counter() - t0) / 20:8.1f} us/call",
              flush=True)

# per-phase shader-clock stamps of one call (thread 0 of the workgroup, s_memtime)
from hydragnn_amd import _native  # noqa: E402

for G, probe in ((4, 0), (64, 0), (64, 1)):
    pos, d = batch(G)
    dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
    dbg[15] = probe
    N = pos.shape[0]
    for _ in range(2):
        _native.ops().radius_static_small(pos, d.batch.long(), d.ptr.long(), d["node_mask"], 5.0, 5, N * 5, N - 1, dbg)
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        _native.ops().radius_static_small(pos, d.batch.long(), d.ptr.long(), d["node_mask"], 5.0, 5, N * 5, N - 1, dbg)
    torch.cuda.synchronize()
    print(f"  {1e6 * (time.perf_counter() - t0) / 50:.1f} us per raw call")
    st = dbg.cpu().tolist()[:14]
    names = ["stage", "count", "scan", "fill", "srccnt", "dummy", "scan2", "cap", "place"]
    ph = [f"{n} +{st[i + 1] - st[i]}" for i, n in enumerate(names)] + [f"out +{st[11] - st[9]}"]
    print(f"G {G} probe {probe}: " + ", ".join(ph), flush=True)
