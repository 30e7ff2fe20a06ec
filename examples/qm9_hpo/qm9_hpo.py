"""Hyper-parameter search on the QM9 example (reference ``examples/qm9_hpo/
{qm9_deephyper.py, qm9_optuna.py, qm9_deephyper_multi.py}``: DeepHyper / Optuna drive
trials that each train ``qm9.py`` with sampled mpnn_type, hidden_dim, num_conv_layers,
learning rate, and report the validation / test error).

DeepHyper and Optuna are not installed here; the search is
``hydragnn_amd.utils.hpo.random_search`` over the same space, and every trial runs as a
``torchrun`` child on its own GPU slot of the node (``TrialScheduler``:
``HIP_VISIBLE_DEVICES`` per slot, one rendezvous port per trial).  Each trial prints its
result dict (``examples/common.run_example``); the best trial is reported and written
to ``<workdir>/hpo_result.json``.

Usage: python examples/qm9_hpo/qm9_hpo.py [--trials 8] [--gpus 8] [--gpus_per_trial 1] [--num_epoch 2]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from hydragnn_amd.utils.hpo import TrialScheduler, random_search  # noqa: E402

SPACE = {
    "--mpnn_type": ["EGNN", "PNA", "SchNet", "GIN", "SAGE", "PNAPlus", "PAINN"],
    "--hidden_dim": ["32", "64", "96"],
    "--num_conv_layers": ["2", "3", "4"],
    "--learning_rate": ["0.0003", "0.001", "0.003"],
}


def search(script, space, argv, description):
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--gpus", type=int, default=None, help="GPUs of the node (default: visible count, min 1)")
    ap.add_argument("--gpus_per_trial", type=int, default=1)
    ap.add_argument("--num_epoch", type=int, default=2)
    ap.add_argument("--num_samples", type=int, default=500)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=None, help="per-trial wall limit (s)")
    args, extra = ap.parse_known_args(argv)
    workdir = os.path.abspath(args.workdir or os.path.join(os.getcwd(), "hpo"))
    os.makedirs(workdir, exist_ok=True)
    gpus = args.gpus
    if gpus is None:
        import torch

        gpus = max(1, torch.cuda.device_count())
    sched = TrialScheduler(script, total_gpus=gpus, gpus_per_trial=args.gpus_per_trial, workdir=workdir,
                           timeout=args.timeout, env={"OMP_NUM_THREADS": "2"})
    fixed = ["--num_epoch", str(args.num_epoch), "--num_samples", str(args.num_samples)] + extra
    best, value, results = random_search(space, args.trials, sched, seed=args.seed, fixed_args=fixed)
    out = {"best_args": best, "best_test_error": value,
           "trials": [{"rc": r["returncode"], "result": r["result"]} for r in results]}
    with open(os.path.join(workdir, "hpo_result.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"best_args": best, "best_test_error": value, "n_ok": sum(r["returncode"] == 0 for r in results)}),
          flush=True)
    return out


if __name__ == "__main__":
    search(os.path.join(ROOT, "examples", "qm9", "qm9.py"), SPACE, sys.argv[1:], __doc__.splitlines()[0])
