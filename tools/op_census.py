"""Which Python lines issue the torch (aten) kernels of a captured step?  Runs the captured
step's exact computation eagerly (``TrainStep.padded_step``) of a ``bench_configs`` config
under a TorchDispatchMode and counts every aten op by the innermost ``hydragnn_amd`` frame
that issued it (forward; the backward runs on autograd's worker thread and is listed by
autograd node name through the profiler).  Usage:
    python tools/op_census.py multibranch_mace [--top 60]"""
import argparse
import collections
import os
import sys
import traceback

import numpy as np
import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_configs as bc  # noqa: E402
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.train.step import TrainStep  # noqa: E402

# aten ops that launch no kernel (metadata / views)
_FREE = ("view", "reshape", "_unsafe_view", "expand", "permute", "transpose", "t", "squeeze", "unsqueeze",
         "slice", "select", "split", "split_with_sizes", "narrow", "as_strided", "alias", "detach", "empty",
         "empty_like", "empty_strided", "_to_copy_noop", "lift_fresh", "unbind", "contiguous", "_reshape_alias",
         "new_empty", "new_empty_strided", "chunk", "is_same_size", "record_stream", "view_as", "resolve_conj",
         "resolve_neg")


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name not in _FREE and not name.startswith("hydra"):
            where = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "hydragnn_amd" in fr.filename and "_native" not in fr.filename:
                    where = f"{os.path.relpath(fr.filename)}:{fr.lineno} {fr.name}"
                    break
            self.c[(name, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    model, samples, B, ht, hd, forces = bc.CONFIGS[a.config](dev)
    model = model.to(dev)
    if not forces:
        samples = bc._targets_for_store(samples, ht)
    store = DeviceGraphStore(samples, dev, head_types=None if forces else ht, head_dims=None if forces else hd)
    ts = TrainStep(model, lr=1e-3, mode="graph", compute_grad_energy=forces)
    rng = np.random.default_rng(0)
    draw = lambda: list(rng.choice(len(store), size=B, replace=False))  # noqa: E731
    for _ in range(2):
        ts.padded_step(store, draw())
    torch.cuda.synchronize()
    cen = Census()
    with cen:
        ts.padded_step(store, draw())
    torch.cuda.synchronize()
    tot = sum(cen.c.values())
    print(f"forward-thread aten ops per step: {tot}")
    for (n, w), v in cen.c.most_common(a.top):
        print(f"{v:5d}  {n:28s} {w[:140]}")


if __name__ == "__main__":
    main()
