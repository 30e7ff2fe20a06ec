"""bf16 MFMA engine (csrc/bgemm.hip) vs torch/hipBLASLt on the SC25 EGNN-866 shapes.

Edge GEMMs: [E=35k, 896] x [896, 896]^T (forward / data gradient) and the weight
gradient G^T X over E rows; node GEMMs: [N=2.2k, 896|1792]; decoder heads [2.2k, 896].
Interleaved rounds in one process (median of 5 x 20 calls), random operands."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.ops import bgemm as bg  # noqa: E402

dev = torch.device("cuda")


def timeit(fn, n=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1000.0


def rb(*shape):
    return (torch.randn(*shape, device=dev) * 0.5).to(torch.bfloat16)


def main():
    cases = []
    for M, K, Np in [(35000, 896, 896), (2200, 1792, 896), (2200, 896, 1792), (2200, 896, 896)]:
        A, B = rb(M, K), rb(Np, K)
        outb = torch.empty(M, Np, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * K * Np
        for bm in (64, 128, 256, 1064, 1128, 1256):
            cases.append((f"NT{bm} M={M} K={K} N={Np}", fl,
                          lambda A=A, B=B, K=K, Np=Np, outb=outb, bm=bm: bg.nt(A, B, K, Np, act=1, outb=outb, bm=bm)))
        cases.append((f"torch   M={M} K={K} N={Np}", fl, lambda A=A, B=B: torch.relu(A @ B.T)))
    for M, Np, Kp in [(35000, 896, 896), (2200, 896, 1792), (2200, 1792, 896)]:
        G, X = rb(M, Np), rb(M, Kp)
        out = torch.empty(Np, Kp, device=dev)
        fl = 2.0 * M * Np * Kp
        cases.append((f"TN  M={M} N={Np} K={Kp}", fl, lambda G=G, X=X, Np=Np, Kp=Kp, out=out:
                      bg.wgrad(G, X, Np, Kp, [(out, 0, None, -1)])))
        cases.append((f"torch TN M={M} N={Np} K={Kp}", fl, lambda G=G, X=X: G.T @ X))
    res = {c[0]: [] for c in cases}
    for _ in range(5):
        for name, fl, fn in cases:
            res[name].append(timeit(fn))
    for name, fl, fn in cases:
        us = statistics.median(res[name])
        print(f"{name:36s} {us:9.1f} us  {fl / us / 1e6:8.1f} TF/s  (min {min(res[name]):.1f})", flush=True)


if __name__ == "__main__":
    main()
