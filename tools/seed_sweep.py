"""Run one CI accuracy case for several init seeds (reports error / per-head MAE).
Usage: python tools/seed_sweep.py <mpnn_type> <ci_input> <lengths 0|1> <seed> [<seed> ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from graph_train_util import unittest_train_model  # noqa: E402

mt, ci, ln = sys.argv[1], sys.argv[2], sys.argv[3] == "1"
wd = os.path.join(os.environ.get("SWEEP_WD", os.path.join(ROOT, "gpurun_out")), "sweep_wd")
os.makedirs(wd, exist_ok=True)
for s in sys.argv[4:]:
    try:
        e = unittest_train_model(mt, "", "", ci, ln, wd,
                                 overwrite_config={"NeuralNetwork": {"Architecture": {"init_seed": int(s)}}})
        print(f"seed {s}: PASS error {e:.5f}", flush=True)
    except AssertionError as ex:
        print(f"seed {s}: FAIL {ex}", flush=True)
