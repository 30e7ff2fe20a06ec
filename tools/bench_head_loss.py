"""Micro-benchmark of the one-workgroup head+loss kernels (csrc/mlp.hip) against the
multi-launch path (fused MLP + masked loss): per-call time for several row counts and
chain shapes.  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402
from hydragnn_amd.ops import mlp as _mlp  # noqa: E402,F401


def bench(fn, it=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = torch.device("cuda")
    ops = _native.ops()
    for G, dims in [(33, [64, 50, 50, 50, 25, 1]), (1, [64, 50, 50, 50, 25, 1]), (8, [64, 50, 50, 50, 25, 1]),
                    (33, [64, 1]), (33, [64, 50, 1]), (33, [8, 8, 1])]:
        Ws = [torch.randn(dims[i + 1], dims[i], device=dev) * 0.1 for i in range(len(dims) - 1)]
        bs = [torch.randn(dims[i + 1], device=dev) * 0.1 for i in range(len(dims) - 1)]
        if os.environ.get("HL_CONTIG") == "1":  # every weight and bias as a view of one buffer
            n = sum(w.numel() + b.numel() for w, b in zip(Ws, bs))
            buf = torch.empty(n, device=dev)
            off, W2, b2 = 0, [], []
            for w, b in zip(Ws, bs):
                W2.append(buf[off:off + w.numel()].view_as(w).copy_(w))
                off += w.numel()
                b2.append(buf[off:off + b.numel()].copy_(b))
                off += b.numel()
            Ws, bs = W2, b2
        relu = [1] * (len(dims) - 2) + [0]
        x = torch.randn(G, dims[0], device=dev)
        t = torch.randn(G, dims[-1], device=dev)
        m = torch.ones(G, dtype=torch.bool, device=dev)
        stats, pred, acts = ops.head_loss_fwd(x, Ws, bs, relu, t, m, 1)
        g = torch.ones(1, device=dev)
        tf = bench(lambda: ops.head_loss_fwd(x, Ws, bs, relu, t, m, 1))
        tb = bench(lambda: ops.head_loss_bwd(g, x, acts, Ws, bs, relu, t, m, stats, 1))
        tu = bench(lambda: ops.head_loss_fused(x, Ws, bs, relu, t, m, 1))
        to = bench(lambda: ops.mlp_fwd(x, Ws, bs, relu))
        dbg = torch.zeros(32, dtype=torch.int64, device=dev)
        ops.head_loss_fused(x, Ws, bs, relu, t, m, 1, dbg)
        torch.cuda.synchronize()
        st = dbg.cpu().tolist()
        # row-split kernel marks: 0 start, 1 table + zero fill, 2 staged, 3 forward chain,
        # 19 loss, 20 backward chain, 31 end (reduce by the last workgroup)
        names = {0: "start", 28: "table+mask", 29: "copies issued", 1: "zero", 2: "stage", 3: "fwd0", 19: "fwd+loss", 20: "bwd", 31: "end"}
        prev = st[0]
        txt = []
        for i, name in sorted(names.items(), key=lambda kv: [0, 28, 29, 1, 2, 3, 19, 20, 31].index(kv[0])):
            if st[i] == 0:
                continue
            txt.append(f"{name} +{st[i] - prev}")
            prev = st[i]
        print("   stamps (shader clocks, s_memtime): " + ", ".join(txt), flush=True)
        print(f"G {G:4d} dims {dims}: head_loss fwd {tf:7.1f} us  bwd {tb:7.1f} us  fused fwd+bwd {tu:7.1f} us"
              f"   (mlp_fwd {to:6.1f} us)", flush=True)


if __name__ == "__main__":
    main()
