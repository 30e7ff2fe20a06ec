"""Micro-benchmark of the hot ops on one GPU (median of timed repeats via HIP events).
Usage: python tools/bench_ops.py [wgrad|bn|all]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402


def timeit(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    return ts[len(ts) // 2]


def graph_time(fn, reps=20):
    """Per-call time of fn captured 20x in one hipGraph (launch overhead excluded)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    return timeit(g.replay, reps) / 20


def bench_wgrad():
    ops = _native.ops()
    x0 = torch.zeros(256, device="cuda")
    print(f"floor: fill(256) in graph {graph_time(lambda: x0.fill_(1.0)):.2f} us", flush=True)
    for M, O, I in [(2560, 64, 64), (2560, 128, 64), (2560, 64, 1088), (2560, 192, 64), (2560, 64, 128),
                    (22528, 64, 64), (22528, 64, 6), (22528, 64, 1), (22528, 64, 65)]:
        dy = torch.randn(M, O, device="cuda")
        x = torch.randn(M, I, device="cuda")
        t_k = graph_time(lambda: ops.linear_wgrad(dy, x, True))
        t_b = graph_time(lambda: (dy.t() @ x, dy.sum(0)))
        t_mm = graph_time(lambda: dy.t() @ x)
        print(f"wgrad M={M} O={O} I={I}: hip {t_k:.2f} us | torch mm+sum {t_b:.2f} us | mm {t_mm:.2f} us", flush=True)


def bench_bn():
    from hydragnn_amd.models.layers import BatchNorm
    from hydragnn_amd.ops.norm import norm_add
    from hydragnn_amd.ops import rng

    for N, C in [(2816, 64), (11264, 64), (2816, 128)]:
        a = torch.randn(N, C, device="cuda", requires_grad=True)
        b = torch.randn(N, C, device="cuda")
        bn = BatchNorm(C).cuda()
        nv = torch.tensor([N - 100], dtype=torch.int32, device="cuda")
        rng.advance("cuda")
        f1 = lambda: norm_add(a, bn, nv, residual=b, p=0.25, salt=3, training=True)  # noqa: E731
        f2 = lambda: norm_add(a, bn, nv, relu=True, zero_pad=True)  # noqa: E731
        with torch.no_grad():
            print(f"bn N={N} C={C}: fwd drop+res {graph_time(f1):.2f} us | fwd relu+pad {graph_time(f2):.2f} us",
                  flush=True)
        y = f1()
        g = torch.randn_like(y)
        fb = lambda: torch.autograd.grad(f1(), [a], g)  # noqa: E731
        print(f"bn N={N} C={C}: fwd+bwd eager {timeit(fb):.2f} us", flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("wgrad", "all"):
        bench_wgrad()
    if what in ("bn", "all"):
        bench_bn()
