"""Micro-benchmark of the row-program interpreter (csrc/rowprog.hip): per-instruction cost
of element-wise (LDS) and LIN (MFMA) instructions at the PAINN node-chain shapes.
Usage: python tools/bench_rowprog.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(name, build, N=1024, F=64, reps=20):
    from hydragnn_amd.ops import rowprog as rp
    from hydragnn_amd import _native

    P = rp.Prog()
    x = P.input(F, 1, "x")
    ws, out = build(P, x, F)
    P.outputs = [out]
    ins, bufs, width, lds_w, where = rp.compile_device(P, [x, out.base], len(ws), inputs=[x])
    dev = torch.device("cuda")
    tins = torch.from_numpy(ins).to(dev)
    wts = [w.to(dev) for w in ws]
    xt = torch.randn(N, F, device=dev)
    ot = torch.empty(N, out.base.nc * out.base.w, device=dev)
    wsb = torch.empty(max(N * width, 1), device=dev)
    ptrs = wts + [xt, ot]
    for _ in range(3):
        _native.ops().rowprog_run(tins, wsb, None, ptrs, N, lds_w, None, len(wts))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        _native.ops().rowprog_run(tins, wsb, None, ptrs, N, lds_w, None, len(wts))
    e1.record()
    torch.cuda.synchronize()
    us = 1000 * e0.elapsed_time(e1) / reps
    dbg = torch.zeros(4 * len(ins), dtype=torch.int64, device=dev)
    _native.ops().rowprog_run(tins, wsb, None, ptrs, N, lds_w, dbg, len(wts))
    torch.cuda.synchronize()
    d = dbg.view(-1, 4).cpu().double()
    dec, run, bar = (d[:, 1] - d[:, 0]).mean(), (d[:, 2] - d[:, 1]).mean(), (d[:, 3] - d[:, 2]).mean()
    gap = (d[1:, 0] - d[:-1, 3]).mean() if len(d) > 1 else 0.0
    print(f"{name:34s} {len(ins):4d} instr  {us:8.1f} us  {us / max(len(ins), 1):6.2f} us/instr  lds_w {lds_w}"
          f"  cycles/instr: decode {dec:.0f} run {run:.0f} barrier {bar:.0f} next {gap:.0f}", flush=True)


def main():
    from hydragnn_amd.ops import rowprog as rp

    def ew_chain(n, op="mul"):
        def b(P, x, F):
            h = x
            for _ in range(n):
                h = P.mul(h, x) if op == "mul" else P.act(h, "silu")
            return [], h
        return b

    def lin_chain(n, O):
        def b(P, x, F):
            ws = [torch.randn(F, F) * 0.1, torch.randn(F) * 0.1]
            W = rp.Weight(0, F, F, 1)
            h = x
            for _ in range(n):
                h = P.lin([(h, 0)], W)
            return ws, h
        return b

    def lin_wide(n):
        def b(P, x, F):
            ws = [torch.randn(3 * F, F) * 0.1, torch.randn(3 * F) * 0.1, torch.randn(F, 3 * F) * 0.1]
            W1, W2 = rp.Weight(0, 3 * F, F, 1), rp.Weight(2, F, 3 * F)
            h = x
            for _ in range(n):
                h = P.lin([(P.lin([(h, 0)], W1), 0)], W2, bias=False)
            return ws, h
        return b

    def vec_lin(n):
        def b(P, x, F):
            ws = [torch.randn(F, F) * 0.1]
            W = rp.Weight(0, F, F)
            v = P.mul(P.add(x, x), x)
            h = P.ew(rp.E_COPY, v, nc=3)
            for _ in range(n):
                h = P.lin([(h, 0)], W)
            return ws, P.dot3(h, h)
        return b

    run("empty-ish (1 copy)", ew_chain(1))
    run("ew mul x100", ew_chain(100))
    run("ew silu x100", ew_chain(100, "act"))
    run("lin 64->64 x30", lin_chain(30, 64))
    run("lin 64->192->64 x15", lin_wide(15))
    run("vector lin 3x64->64 x30", vec_lin(30))


if __name__ == "__main__":
    main()
