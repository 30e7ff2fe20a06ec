"""Branch-parallel HIP streams inside one training step.

A GPS layer's local MPNN and global attention (reference ``globalAtt/gps.py:103-152``)
are independent until they are summed; so are the decoder heads.  Running one branch
on a side stream lets the two branches' kernels execute concurrently: most kernels of
this workload are far below the chip's width (a ~5 us dispatch floor for a few hundred
workgroups), so two streams overlap almost perfectly.  Autograd runs every backward
node on the stream of its forward node and synchronises cross-stream edges, so the
backward branches overlap too, and the whole thing is captured into the step hipGraph
as parallel branches (fork = ``wait_stream`` on the capturing stream).

``HYDRA_BRANCH_STREAMS=0`` disables it (single stream, identical numerics: the two
branches touch disjoint outputs; only the join order is fixed)."""
import os

import torch

_side = {}


def enabled(t):
    return t.is_cuda and os.environ.get("HYDRA_BRANCH_STREAMS", "1") == "1"


def side_stream(device, slot=0):
    """Cached side stream ``slot`` of ``device`` (slot 0: branch forks; slot 1: the
    attention backward's dK/dV pass, which forks again from inside a side branch;
    slot 2: the fused GPS encoder's edge chain (forward) and per-layer weight gradients /
    edge backward (backward); slot 3: the first layer's edge backward; slot 4: the fused
    graph head's weight-gradient twin, ops/mlp.py)."""
    key = (torch.device(device).index, slot)
    s = _side.get(key)
    if s is None:
        # HYDRA_SIDE_PRIORITY: priority of the side-branch stream (torch convention: lower is
        # higher priority; 0 = default).  The captured step records branch priorities only
        # if the runtime keeps them per graph node (tools/gpu_r4_iter.sh A/B).
        # HYDRA_WGRAD_PRIORITY: the same for slot 2 (weight gradients / edge backward)
        env = "HYDRA_WGRAD_PRIORITY" if slot >= 2 else "HYDRA_SIDE_PRIORITY"
        s = torch.cuda.Stream(device=device, priority=int(os.environ.get(env, "0")))
        _side[key] = s
    return s


class Fork:
    """``with Fork(x) as f: <side-branch code>``; after the block ``f.join(*outs)`` makes
    the current stream wait for the side branch and keeps its outputs alive for it."""

    def __init__(self, *inputs, slot=0, enable=True):
        self.inputs = [t for t in inputs if torch.is_tensor(t)]
        self.on = enable and bool(self.inputs) and enabled(self.inputs[0])
        if self.on:
            self.main = torch.cuda.current_stream(self.inputs[0].device)
            self.side = side_stream(self.inputs[0].device, slot)

    def __enter__(self):
        if self.on:
            self.side.wait_stream(self.main)
            for t in self.inputs:
                t.record_stream(self.side)
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.on:
            self._ctx.__exit__(*exc)
        return False

    def join(self, *outs):
        if self.on:
            self.main.wait_stream(self.side)
            for t in outs:
                if torch.is_tensor(t):
                    t.record_stream(self.main)
        return outs[0] if len(outs) == 1 else outs
