"""Debug driver for the captured PNAEq conv-head divergence (VERDICT r4 missing #2): runs the
CI conv-head training of PNAEq (tests/test_graphs.py::test_train_gpu_conv_head) with
  MODE=padded  every training batch through TrainStep.padded_step (the captured step's exact
               padded computation, run eagerly: the fused PNA aggregation is used)
  MODE=graph   captured steps (set HYDRA_PNA_AGG_CAPTURE=1 for the fused op under capture),
               checking after every replay whether the loss and the gradient buffer are finite
and prints the first non-finite step plus the final test RMSE.
Usage: MODE=graph HYDRA_PNA_AGG_CAPTURE=1 python tools/pnaeq_capture_debug.py [workdir]"""
import os
import sys
import tempfile

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))

from hydragnn_amd.train import step as stepmod  # noqa: E402
from graph_train_util import run_ci  # noqa: E402

MODE = os.environ.get("MODE", "graph")
state = {"n": 0, "bad": 0, "first": None}

orig_graph_step = stepmod.TrainStep.graph_step


def checked_graph_step(self, store, indices):
    loss, tasks = orig_graph_step(self, store, indices)
    torch.cuda.synchronize()
    state["n"] += 1
    lf = bool(torch.isfinite(loss).all())
    gf = True
    if self.sync is not None and getattr(self.sync, "flat", None) is not None:
        gf = bool(torch.isfinite(self.sync.flat).all())
    else:
        for p in self.module.parameters():
            if p.grad is not None and not bool(torch.isfinite(p.grad).all()):
                gf = False
                break
    if not (lf and gf):
        state["bad"] += 1
        if state["first"] is None:
            state["first"] = state["n"]
            names = [n for n, p in self.module.named_parameters()
                     if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
            print(f"[debug] replay {state['n']}: loss finite {lf} ({float(loss):.4g}), grads finite {gf}; "
                  f"non-finite grads: {names[:8]}", flush=True)
    return loss, tasks


def padded_call(self, store, indices):
    state["n"] += 1
    return self.padded_step(store, indices)


def compare_call(self, store, indices):
    """MODE=compare: for the first 3 steps run the padded eager step and the captured step
    from the same parameters / optimizer state and compare loss and every gradient."""
    state["n"] += 1
    if state["n"] > int(os.environ.get("COMPARE_STEPS", "3")) or self.sync is None or state.get("diverged"):
        return orig_call(self, store, indices)
    N, E = store.sizes_of(indices)
    want, picked = self.bucket_of(N, E), self._pick(N, E)
    snap = self._snapshot()
    # on the capture stream: the AccumulateGrad nodes a default-stream backward creates would
    # break the later capture
    cs = self._capture_stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        lp, _ = self.padded_step(store, indices)
    torch.cuda.synchronize()
    gp = self.sync.flat.detach().clone()
    pp = [p.detach().clone() for p in self.module.parameters()]
    self._restore(snap)
    lg, _ = orig_call(self, store, indices)
    torch.cuda.synchronize()
    gg = self.sync.flat.detach().clone()
    gd = float((gp - gg).abs().max())
    if state["n"] <= 3 or gd > 0 or float(lp) != float(lg):
        print(f"[debug] step {state['n']}: loss padded {float(lp):.6g} graph {float(lg):.6g}; "
              f"flat grad max|diff| {gd:.3e} (scale {float(gp.abs().max()):.3e}); bucket wanted {want} "
              f"replayed {picked} (captured {len(self.graphs)})", flush=True)
    if gd > 0 or float(lp) != float(lg):
        state["diverged"] = state["n"]
    for name, prm in self.module.named_parameters():
        if not prm.requires_grad:
            continue
        off = self.sync.offset[prm] if prm in self.sync.offset else self.sync.offset[id(prm)]
        n = prm.numel()
        d = float((gp[off:off + n] - gg[off:off + n]).abs().max()) if n else 0.0
        sc = float(gp[off:off + n].abs().max()) if n else 0.0
        if d > 1e-4 * (1 + sc):
            print(f"[debug]   grad {name}: max|diff| {d:.3e} scale {sc:.3e} "
                  f"graph-zero {bool((gg[off:off + n] == 0).all())}", flush=True)
    return lg, _


orig_call = stepmod.TrainStep.__call__

from hydragnn_amd.train import train_validate_test as tvt  # noqa: E402

_orig_validate = tvt.validate


def logged_validate(*a, **k):
    v, t = _orig_validate(*a, **k)
    print(f"[debug] validate after {state['n']} steps: {float(v):.6g}", flush=True)
    return v, t


tvt.validate = logged_validate
if MODE == "graph":
    stepmod.TrainStep.graph_step = checked_graph_step
elif MODE == "compare":
    stepmod.TrainStep.__call__ = compare_call
else:
    stepmod.TrainStep.__call__ = padded_call

wd = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp()
torch.manual_seed(97)
error, error_task, true_values, pred_values = run_ci("PNAEq", "ci_conv_head", wd)
print(f"[debug] MODE={MODE} steps {state['n']} non-finite {state['bad']} first {state['first']} "
      f"RMSE {[round(float(e), 4) for e in error_task]}", flush=True)
