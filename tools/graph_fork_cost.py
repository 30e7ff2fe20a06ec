"""Cost of stream fork/join edges inside a captured hipGraph on MI355X.

Captures three graphs of tiny kernels (x.add_(1) on a 1K tensor) and times replays:
  seq   : 2K kernels on one stream
  fork  : K fork/join pairs (main and side stream each run one kernel, then join)
  chain : K kernels whose side-stream partner is joined back immediately (fork + join
          around ONE kernel)
Per-edge overhead = (fork - seq) / K.  GPU only."""
import torch


def timed(g, it=50):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = torch.device("cuda")
    a = torch.zeros(1024, device=dev)
    b = torch.zeros(1024, device=dev)
    side = torch.cuda.Stream()
    K = 32
    for _ in range(3):  # warm-up outside capture
        a.add_(1)
        b.add_(1)
    torch.cuda.synchronize()
    gs = {}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(2 * K):
            a.add_(1)
    gs["seq"] = g
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        main = torch.cuda.current_stream()
        for _ in range(K):
            side.wait_stream(main)
            with torch.cuda.stream(side):
                b.add_(1)
            a.add_(1)
            main.wait_stream(side)
    gs["fork"] = g
    for name, g in gs.items():
        us = timed(g)
        print(f"{name:5s}: {us:8.1f} us per replay ({2 * K} kernels) -> {us / (2 * K):6.2f} us per kernel", flush=True)
    d = (timed(gs["fork"]) - timed(gs["seq"])) / K
    print(f"fork/join pair overhead vs sequential: {d:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
