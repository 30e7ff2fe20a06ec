"""Run the fused small kernels in isolation (for rocprofv3 counter passes).

Usage: python tools/micro_fused.py [reps]  -- mlp fwd/bwd (head chain of the bench),
radial fwd/bwd (E=24576, F=64, K=6, L=3), pna weight prep; prints graph-replay
microseconds per op."""
import os
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd import _native  # noqa: E402


def graph_us(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return 1000.0 * t0.elapsed_time(t1) / (reps * 10)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    ops = _native.ops()
    dev = "cuda"
    dims = [64, 50, 50, 50, 25, 1]
    G = 33
    Ws = [torch.randn(dims[i + 1], dims[i], device=dev) * 0.1 for i in range(5)]
    bs = [torch.randn(dims[i + 1], device=dev) * 0.1 for i in range(5)]
    relu = [1, 1, 1, 1, 0]
    x = torch.randn(G, 64, device=dev)
    out, acts = ops.mlp_fwd(x, Ws, bs, relu)
    dout = torch.randn_like(out.contiguous())
    print(f"mlp_fwd  {graph_us(lambda: ops.mlp_fwd(x, Ws, bs, relu), reps):8.2f} us", flush=True)
    x4 = x[:4].contiguous()
    print(f"mlp_fwd G=4 {graph_us(lambda: ops.mlp_fwd(x4, Ws, bs, relu), reps):8.2f} us", flush=True)
    print(f"mlp_fwd G=4 1 layer {graph_us(lambda: ops.mlp_fwd(x4, Ws[:1], bs[:1], relu[:1]), reps):8.2f} us",
          flush=True)
    W1 = [torch.randn(4, 64, device=dev)]
    b1 = [torch.randn(4, device=dev)]
    print(f"mlp_fwd G=4 64->4 {graph_us(lambda: ops.mlp_fwd(x4, W1, b1, [0]), reps):8.2f} us", flush=True)
    print(f"mlp_bwd  {graph_us(lambda: ops.mlp_bwd(dout, x, acts, Ws, bs, relu), reps):8.2f} us", flush=True)
    seq = nn.Sequential(*[m for i in range(5) for m in ([nn.Linear(dims[i], dims[i + 1])] +
                                                        ([nn.ReLU()] if relu[i] else []))]).to(dev)
    xr = x.clone().requires_grad_(True)

    def torch_chain():
        y = seq(xr)
        y.backward(dout)
    print(f"torch chain fwd+bwd {graph_us(torch_chain, reps):8.2f} us", flush=True)
    E, F, K, L = 24576, 64, 6, 3
    dist = 0.5 + torch.rand(E, device=dev) * 9.0
    freq = torch.arange(1, K + 1, device=dev, dtype=torch.float32) * 3.14159
    We = torch.randn(L, F, K, device=dev)
    be = torch.randn(L, F, device=dev)
    Wl = torch.randn(L, F, K, device=dev)
    R, Gt = ops.radial_fwd(dist, freq, We, be, Wl, 10.0, 5)
    dR, dG = torch.randn_like(R), torch.randn_like(Gt)
    print(f"radial_fwd {graph_us(lambda: ops.radial_fwd(dist, freq, We, be, Wl, 10.0, 5), reps):8.2f} us", flush=True)
    print(f"radial_bwd {graph_us(lambda: ops.radial_bwd(list(dR.unbind(0)), list(dG.unbind(0)), R, dist, freq, We, Wl, 10.0, 5), reps):8.2f} us",
          flush=True)
    Ee = 26624  # edges of the headline batch (1664 row blocks of 16)
    r = torch.randn(Ee, F, device=dev)
    e = torch.randn(Ee, F, device=dev)
    Wr, Wd = torch.randn(F, F, device=dev) * 0.1, torch.randn(F, F, device=dev) * 0.1
    bc = torch.randn(F, device=dev)
    print(f"gf_edge_fwd E={Ee} {graph_us(lambda: ops.gf_edge_fwd(r, e, Wr, Wd, bc), reps):8.2f} us", flush=True)
    dC, dGe = torch.randn(Ee, F, device=dev), torch.randn(Ee, F, device=dev)
    Wemb, Wrl = torch.randn(F, K, device=dev), torch.randn(F, K, device=dev)
    de = torch.zeros(Ee, F, device=dev)
    drbf = torch.zeros(Ee, K, device=dev)
    print(f"gf_edge_bwd E={Ee} {graph_us(lambda: ops.gf_edge_bwd(dC, Wr, Wd, r, de, dGe, Wemb, Wrl, drbf, K), reps):8.2f} us",
          flush=True)
    print(f"copy [E,F] {graph_us(lambda: r.clone(), reps):8.2f} us", flush=True)
    z = torch.zeros(256, device=dev)
    print(f"floor fill(256) {graph_us(lambda: z.fill_(1.0), reps):8.2f} us", flush=True)


if __name__ == "__main__":
    main()
