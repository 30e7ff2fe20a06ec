"""Find the first module / autograd node producing a non-finite value in a CI training run.

Usage: python tools/nan_hunt.py <mpnn_type> <ci_input> [lengths 0|1]
Runs the tests' unittest_train_model with a global forward hook (first module whose
output is non-finite) and autograd anomaly detection (first backward node)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("HYDRAGNN_CAPTURE", "0")

from graph_train_util import unittest_train_model  # noqa: E402

_seen = {"n": 0}


def _hook(mod, inp, out):
    outs = out if isinstance(out, (tuple, list)) else (out,)
    for o in outs:
        if torch.is_tensor(o) and o.is_floating_point() and not torch.isfinite(o).all():
            if _seen["n"] < 5:
                bad = [torch.is_tensor(i) and i.is_floating_point() and not torch.isfinite(i).all() for i in inp]
                amax = [float(i.abs().max()) if torch.is_tensor(i) and i.numel() and i.is_floating_point() else None
                         for i in inp]
                extra = ""
                bn = getattr(mod, "module", None)
                if isinstance(bn, torch.nn.BatchNorm1d):
                    extra = (f" training={mod.training} rm_finite={bool(torch.isfinite(bn.running_mean).all())} "
                             f"rv_min={float(bn.running_var.min())} w_finite={bool(torch.isfinite(bn.weight).all())} "
                             f"nonfinite_out_cols={int((~torch.isfinite(o)).any(0).sum())} "
                             f"nonfinite_out_rows={int((~torch.isfinite(o)).any(1).sum())}")
                    x = inp[0]
                    print("   col var:", x.var(0, unbiased=False).tolist()[:8], "col mean:", x.mean(0).tolist()[:8])
                print(f"NONFINITE output of {type(mod).__name__} (inputs nonfinite: {bad}, absmax {amax}) "
                      f"shape {tuple(o.shape)}{extra}", flush=True)
            _seen["n"] += 1


torch.nn.modules.module.register_module_forward_hook(_hook)
torch.autograd.set_detect_anomaly(True, check_nan=True)
m, ci = sys.argv[1], sys.argv[2]
ln = len(sys.argv) > 3 and sys.argv[3] == "1"
wd = os.path.join(ROOT, "gpurun_out", "nan_wd")
os.makedirs(wd, exist_ok=True)
try:
    print("result", unittest_train_model(m, "", "", ci, ln, wd))
except Exception as ex:  # noqa: BLE001
    print("EXC", type(ex).__name__, str(ex)[:2000])
