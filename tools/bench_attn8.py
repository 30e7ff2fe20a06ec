"""Time the 8-wide-head MFMA attention (csrc/attention8.hip) against the VALU kernels
(csrc/attention.hip) at the OC20 headline shape.  Usage: python tools/bench_attn8.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402
from hydragnn_amd.ops.attention import make_segments  # noqa: E402
from tools.bench_ops import graph_time  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
H, D = 8, 8
ops = _native.ops()
qkv = torch.randn(N, 3 * H * D, device="cuda")
sid, sptr = make_segments(N, "batch", num_valid=N - 249, device="cuda")
dO = torch.randn(N, H * D, device="cuda")
sc = 1.0 / D ** 0.5
O, L = ops.attn_fwd(qkv, sid, sptr, H, sc, N, 0)
tf = graph_time(lambda: ops.attn_fwd(qkv, sid, sptr, H, sc, N, 0))
tb = graph_time(lambda: ops.attn_bwd(dO, qkv, O, L, sid, sptr, H, sc, N, 0))
print(f"valu  : fwd {tf:7.1f} us  bwd {tb:7.1f} us", flush=True)
pk = ops.attn8_pack(qkv, H)
for S in [0, 1, 2, 4, 8]:
    O8, L8 = ops.attn8_fwd(pk[0], pk[2], pk[5], sid, sptr, N, sc, S)
    tf = graph_time(lambda: ops.attn8_fwd(pk[0], pk[2], pk[5], sid, sptr, N, sc, S))
    tb = graph_time(lambda: ops.attn8_bwd(dO, O8, L8, pk[0], pk[1], pk[2], pk[3], pk[4], sid, sptr, sc, S))
    err = (O8 - O).abs().max().item()
    print(f"mfma S={S}: fwd {tf:7.1f} us  bwd {tb:7.1f} us  (max |O - O_valu| {err:.2e})", flush=True)
