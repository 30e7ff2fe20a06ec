import math, sys, os, torch
sys.path.insert(0, os.getcwd())
from hydragnn_amd import _native
from hydragnn_amd.ops.attention import make_segments
ops = _native.ops()
dev = torch.device("cuda")
N, H = 2311, 8
qkv = torch.randn(N, 24 * H, device=dev).contiguous()
sid, sptr = make_segments(N, "batch", num_valid=N, device=dev)
sc = 1 / math.sqrt(8)
Qp, Qq, Kp, Kq, Vp, Vq = ops.attn8_pack(qkv, H)
Nq = Qp.shape[1]
dO = torch.randn(N, 8 * H, device=dev)
dOp, dOq = ops.attn8_pack(torch.cat([dO, dO, dO], 1).contiguous(), H)[:2]
nd = torch.zeros(H, Nq, device=dev)
def t(fn, it=50):
    for _ in range(5): fn()
    torch.cuda.synchronize(); a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): fn()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b) / it * 1000
for bf in (False, True):
    O, L = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0, bf)
    tf = t(lambda: ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0, bf))
    tb = t(lambda: ops.attn8_bwd_packed(nd, dOp, dOq, L, Qp, Qq, Kp, Kq, Vp, sid, sptr, N, sc, bf))
    print(f"bf16={bf}: fwd {tf:6.1f} us  bwd {tb:6.1f} us", flush=True)
