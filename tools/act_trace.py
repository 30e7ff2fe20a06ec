"""Trace the largest |input| seen by every BatchNorm per epoch-ish window during a CI run.

Usage: python tools/act_trace.py <mpnn_type> <ci_input> [every_n_calls]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("HYDRAGNN_CAPTURE", "0")
from graph_train_util import unittest_train_model  # noqa: E402

every = int(sys.argv[3]) if len(sys.argv) > 3 else 200
state = {"n": 0, "mx": {}}


def hook(mod, inp, out):
    if type(mod).__name__ != "BatchNorm":
        return
    x = inp[0]
    key = id(mod)
    state["mx"][key] = max(state["mx"].get(key, 0.0), float(x.detach().abs().max()))
    state["n"] += 1
    if state["n"] % every == 0:
        print(f"call {state['n']}: max|x| per BN:", " ".join(f"{v:.3g}" for v in state["mx"].values()), flush=True)
        state["mx"].clear()


torch.nn.modules.module.register_module_forward_hook(hook)
wd = os.path.join(os.environ.get("ACT_WD", os.path.join(ROOT, "gpurun_out")), "act_wd")
os.makedirs(wd, exist_ok=True)
try:
    print("result", unittest_train_model(sys.argv[1], "", "", sys.argv[2], False, wd))
except Exception as ex:  # noqa: BLE001
    print("EXC", type(ex).__name__, str(ex)[:500])
