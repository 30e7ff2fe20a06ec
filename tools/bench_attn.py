"""Time the GPS attention kernels at the OC20 bench shape for several split counts.
Usage: python tools/bench_attn.py [N] [H] [D]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402
from hydragnn_amd.ops.attention import make_segments  # noqa: E402
from tools.bench_ops import graph_time  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
H = int(sys.argv[2]) if len(sys.argv) > 2 else 8
D = int(sys.argv[3]) if len(sys.argv) > 3 else 8
ops = _native.ops()
qkv = torch.randn(N, 3 * H * D, device="cuda")
sid, sptr = make_segments(N, "batch", num_valid=N - 200, device="cuda")
dO = torch.randn(N, H * D, device="cuda")
sc = 1.0 / D ** 0.5
for S in [0, 1, 2, 4, 5, 6, 8, 12, 16]:
    O, L = ops.attn_fwd(qkv, sid, sptr, H, sc, N, S)
    tf = graph_time(lambda: ops.attn_fwd(qkv, sid, sptr, H, sc, N, S))
    tb = graph_time(lambda: ops.attn_bwd(dO, qkv, O, L, sid, sptr, H, sc, N, S))
    fl = 4.0 * N * N * H * D
    print(f"splits {S:2d}: fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF/s)  bwd {tb:7.1f} us", flush=True)
