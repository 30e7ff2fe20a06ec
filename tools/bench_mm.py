"""Microbenchmark of the MFMA GEMM engine vs torch (hipBLASLt) on the headline's GEMM shapes.
Usage: python tools/bench_mm.py   (HYDRA_MM_SPLIT=k forces the split-K factor)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402

ops = _native.ops()


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


shapes = [("AB node", 2311, 64, 128), ("post_nn", 2311, 1088, 64), ("C edge", 23105, 7, 64), ("qkv", 2311, 64, 192),
          ("mlp1", 2311, 64, 128), ("head", 33, 64, 50)]
for name, M, K, N in shapes:
    x = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    dy = torch.randn(M, N, device="cuda")
    for prec in (0, 1):
        tf = timeit(lambda: ops.mm_fwd([x], [W], b, None, 0, prec))
        tb = timeit(lambda: ops.mm_bwd(dy, None, [x], [W], [1], True, True, prec))
        tw = timeit(lambda: ops.mm_bwd(dy, None, [x], [W], [0], True, True, prec))
        tdx = timeit(lambda: ops.mm_bwd(dy, None, [x], [W], [1], False, False, prec))
        print(f"{name:8s} M={M:6d} K={K:5d} N={N:4d} prec={prec}: fwd {tf:7.2f} us  bwd(dx+dw+db) {tb:7.2f}  "
              f"dw+db {tw:7.2f}  dx {tdx:7.2f}", flush=True)
    tt = timeit(lambda: torch.nn.functional.linear(x, W, b))
    tdx = timeit(lambda: dy @ W)
    tdw = timeit(lambda: ops.linear_wgrad(dy, x, True))
    print(f"{name:8s} torch: fwd {tt:7.2f}  dgrad {tdx:7.2f}  wgrad(split-K+sum) {tdw:7.2f}", flush=True)
