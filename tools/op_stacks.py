"""Where do a launch-bound step's small kernels come from?  Profiles eager training steps
of a ``bench_configs`` config on the GPU and prints, for the chosen aten ops, the call
counts per step by Python source line (forward) or by the autograd node that issued
them (backward).  Usage: python tools/op_stacks.py multibranch_mace [aten::copy_ ...]"""
import collections
import os
import sys

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_configs as bc  # noqa: E402
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.train.step import TrainStep  # noqa: E402


def main():
    name = sys.argv[1]
    ops = sys.argv[2:] or ["aten::copy_", "aten::fill_", "aten::mul", "aten::add_", "aten::add", "aten::cat",
                           "aten::mm", "aten::sum", "aten::div", "aten::clone", "aten::zeros", "aten::zero_",
                           "aten::index_add_", "aten::gather", "aten::where"]
    dev = torch.device("cuda:0")
    model, samples, B, ht, hd, forces = bc.CONFIGS[name](dev)
    model = model.to(dev)
    if not forces:
        samples = bc._targets_for_store(samples, ht)
    store = DeviceGraphStore(samples, dev, head_types=None if forces else ht, head_dims=None if forces else hd)
    padded = os.environ.get("OP_STACKS_PADDED", "1") == "1"  # the captured step's computation
    ts = TrainStep(model, lr=1e-3, mode="graph" if padded else "eager", compute_grad_energy=forces)
    run = ts.padded_step if padded else ts
    rng = np.random.default_rng(0)
    draw = lambda: list(rng.choice(len(store), size=B, replace=False))  # noqa: E731
    for _ in range(3):
        run(store, draw())
    torch.cuda.synchronize()
    steps = 2
    if os.environ.get("OP_STACKS_MODE") == "dispatch":
        # TorchDispatchMode: the Python call site of every aten op (forward) and the autograd
        # node of backward ops, without relying on the profiler's stack capture
        import traceback

        from torch.utils._python_dispatch import TorchDispatchMode

        c = collections.Counter()
        want = {o.split("::")[1] for o in ops}

        class Spy(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                base = func.overloadpacket.__name__
                if base in want:
                    st = [f"{f.filename.split('repo/')[-1]}:{f.lineno} {f.name}" for f in traceback.extract_stack()
                          if "hydragnn_amd" in f.filename]
                    key = " <- ".join(st[-2:][::-1]) if st else "(autograd / outside the package)"
                    if not st and os.environ.get("OP_STACKS_SHAPES") == "1":
                        key += " " + str([tuple(a.shape) for a in args if torch.is_tensor(a)][:3])
                    c[(base, key)] += 1
                return func(*args, **(kwargs or {}))

        with Spy():
            for _ in range(steps):
                run(store, draw())
            torch.cuda.synchronize()
        for (n, k), v in c.most_common(80):
            print(f"{v / steps:7.1f}  {n:14s} {k[:220]}")
        return
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(steps):
            run(store, draw())
        torch.cuda.synchronize()
    c = collections.Counter()
    for e in prof.events():
        if e.name not in ops:
            continue
        par = e.cpu_parent
        if par is not None and par.name.startswith("aten::"):
            continue  # nested inside another aten op
        st = [s for s in (e.stack or []) if "hydragnn_amd" in s or "tools/" in s]
        if st:
            key = st[0]
        else:
            p = e.cpu_parent
            while p is not None and not p.name.startswith("autograd::engine"):
                p = p.cpu_parent
            key = p.name if p is not None else "?"
        c[(e.name, key)] += 1
    for (n, k), v in c.most_common(60):
        print(f"{v / steps:7.1f}  {n:14s} {k[:150]}")


if __name__ == "__main__":
    main()
