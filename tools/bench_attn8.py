"""Time the 8-wide-head MFMA attention (csrc/attention8.hip) at the OC20 headline shape:
the v2 single-launch kernels (variants 0..4: splits = 0, -1 .. -4) against the grid-split
kernels (splits = S > 0) and the VALU kernels (csrc/attention.hip).
Usage: python tools/bench_attn8.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402
from hydragnn_amd.ops.attention import make_segments  # noqa: E402
from tools.bench_ops import graph_time  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
NV = int(sys.argv[2]) if len(sys.argv) > 2 else 2311  # valid rows (the rest: padding segment)
H, D = 8, 8
ops = _native.ops()
torch.manual_seed(0)
qkv = torch.randn(N, 3 * H * D, device="cuda") * 1.5
sid, sptr = make_segments(N, "batch", num_valid=NV, device="cuda")
dO = torch.randn(N, H * D, device="cuda")
sc = 1.0 / D ** 0.5
O, L = ops.attn_fwd(qkv, sid, sptr, H, sc, N, 0)
dref = ops.attn_bwd(dO, qkv, O, L, sid, sptr, H, sc, N, 0)
tf = graph_time(lambda: ops.attn_fwd(qkv, sid, sptr, H, sc, N, 0))
tb = graph_time(lambda: ops.attn_bwd(dO, qkv, O, L, sid, sptr, H, sc, N, 0))
print(f"valu      : fwd {tf:7.1f} us  bwd {tb:7.1f} us", flush=True)
pk = ops.attn8_pack(qkv, H)
print("v2 auto shape (W fwd, W bwd):", list(ops.attn8_v2_shape(N, H)), flush=True)
names = {0: "v3 auto" if os.environ.get("HYDRA_ATTN8_V3", "1") != "0" else "v2 auto"}
for S in [8, 0, -2, -3, -4, -5, -6, -8]:
    O8, L8 = ops.attn8_fwd(pk[0], pk[2], pk[5], sid, sptr, N, sc, S)
    d8 = ops.attn8_bwd(dO, O8, L8, pk[0], pk[1], pk[2], pk[3], pk[4], sid, sptr, sc, S)
    tf = graph_time(lambda: ops.attn8_fwd(pk[0], pk[2], pk[5], sid, sptr, N, sc, S))
    tb = graph_time(lambda: ops.attn8_bwd(dO, O8, L8, pk[0], pk[1], pk[2], pk[3], pk[4], sid, sptr, sc, S))
    eo = (O8 - O).abs().max().item()
    ed = (d8 - dref).abs().max().item()
    nm = names.get(S, f"grid S={S}" if S > 0 else f"v2 W={-S}")
    print(f"{nm:10s}: fwd {tf:7.1f} us  bwd {tb:7.1f} us  (max |dO| {eo:.2e}, max |d dqkv| {ed:.2e})", flush=True)
