"""Short driver for counter passes over the 8-wide-head attention kernels at the OC20
headline shape: a few launches of the v2 (W=8) and v3 (persistent) forward and backward.
Usage: python tools/attn8_prof.py [N] [NV] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402
from hydragnn_amd.ops.attention import make_segments  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
NV = int(sys.argv[2]) if len(sys.argv) > 2 else 2311
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
H = 8
ops = _native.ops()
torch.manual_seed(0)
qkv = torch.randn(N, 24 * H, device="cuda") * 1.5
sid, sptr = make_segments(N, "batch", num_valid=NV, device="cuda")
dO = torch.randn(N, 8 * H, device="cuda")
sc = 8 ** -0.5
pk = ops.attn8_pack(qkv, H)
for S in (0, -8):  # v3 (auto), v2 with 8 waves
    for _ in range(reps):
        O8, L8 = ops.attn8_fwd(pk[0], pk[2], pk[5], sid, sptr, N, sc, S)
        ops.attn8_bwd(dO, O8, L8, pk[0], pk[1], pk[2], pk[3], pk[4], sid, sptr, sc, S)
torch.cuda.synchronize()
print("done")
