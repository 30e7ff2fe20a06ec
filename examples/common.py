"""Shared driver for the examples (the reference's per-example ``train.py`` scripts all
end in the same ``update_config -> create_model -> train_validate_test`` sequence;
here that sequence is ``hydragnn_amd.run_training`` on serialized splits).

``run_example(config, train, val, test, workdir)`` writes the three splits as
serialized files (``<workdir>/serialized_dataset/<name>_{train,validate,test}.pkl``),
points ``Dataset.path`` at them, trains, predicts on the test split and returns a
result dict (also written to ``<workdir>/<log_name>_result.json``).

No dataset download is possible in this environment: every example generates
synthetic samples with the shapes / fields of the reference dataset it stands for.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import hydragnn_amd  # noqa: E402
from hydragnn_amd.data.serialized import write_serialized  # noqa: E402
from hydragnn_amd.parallel.distributed import get_comm_size_and_rank, setup_ddp  # noqa: E402
from hydragnn_amd.utils.config_utils import get_log_name_config  # noqa: E402


def base_parser(description, default_config):
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--inputfile", default=default_config, help="JSON config (next to this script)")
    ap.add_argument("--mpnn_type", default=None, help="override NeuralNetwork.Architecture.mpnn_type")
    ap.add_argument("--num_samples", type=int, default=None, help="number of synthetic samples")
    ap.add_argument("--num_epoch", type=int, default=None)
    ap.add_argument("--batch_size", type=int, default=None)
    ap.add_argument("--global_attn_engine", default=None)
    ap.add_argument("--global_attn_type", default=None)
    ap.add_argument("--pe_dim", type=int, default=None)
    ap.add_argument("--workdir", default=None, help="where logs/ and serialized_dataset/ go (default: cwd)")
    ap.add_argument("--seed", type=int, default=0)
    # hyper-parameter overrides (the HPO drivers' search space)
    ap.add_argument("--hidden_dim", type=int, default=None)
    ap.add_argument("--num_conv_layers", type=int, default=None)
    ap.add_argument("--learning_rate", type=float, default=None)
    return ap


def load_config(here, args):
    path = args.inputfile if os.path.isabs(args.inputfile) else os.path.join(here, args.inputfile)
    with open(path) as f:
        config = json.load(f)
    arch = config["NeuralNetwork"]["Architecture"]
    tr = config["NeuralNetwork"]["Training"]
    if args.mpnn_type:
        arch["mpnn_type"] = args.mpnn_type
    if args.num_epoch is not None:
        tr["num_epoch"] = args.num_epoch
    if args.batch_size is not None:
        tr["batch_size"] = args.batch_size
    if args.global_attn_engine is not None:
        arch["global_attn_engine"] = args.global_attn_engine or None
    if args.global_attn_type is not None:
        arch["global_attn_type"] = args.global_attn_type
    if args.pe_dim is not None:
        arch["pe_dim"] = args.pe_dim
    apply_hparams(config, args)
    return config


def apply_hparams(config, args):
    arch = config["NeuralNetwork"]["Architecture"]
    if getattr(args, "hidden_dim", None) is not None:
        arch["hidden_dim"] = args.hidden_dim
    if getattr(args, "num_conv_layers", None) is not None:
        arch["num_conv_layers"] = args.num_conv_layers
    if getattr(args, "learning_rate", None) is not None:
        config["NeuralNetwork"]["Training"]["Optimizer"]["learning_rate"] = args.learning_rate
    if getattr(args, "mpnn_type", None):
        arch["mpnn_type"] = args.mpnn_type
    return config


def split(samples, perc_train, seed=0):
    rng = np.random.default_rng(seed)
    idx = rng.permutation(len(samples))
    n_tr = int(len(samples) * perc_train)
    n_va = (len(samples) - n_tr) // 2
    pick = lambda ids: [samples[i] for i in ids]  # noqa: E731
    return pick(idx[:n_tr]), pick(idx[n_tr:n_tr + n_va]), pick(idx[n_tr + n_va:])


def run_example(config, train, val, test, workdir=None):
    workdir = os.path.abspath(workdir or os.getcwd())
    os.makedirs(workdir, exist_ok=True)
    setup_ddp()
    _, rank = get_comm_size_and_rank()
    name = config["Dataset"]["name"]
    sd = os.path.join(workdir, "serialized_dataset")
    paths = {k: os.path.join(sd, f"{name}_{k}.pkl") for k in ("train", "validate", "test")}
    if rank == 0:
        for k, s in zip(("train", "validate", "test"), (train, val, test)):
            write_serialized(paths[k], s)
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    config["Dataset"]["path"] = paths
    os.environ["SERIALIZED_DATA_PATH"] = workdir
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        hydragnn_amd.run_training(config)
        error, tasks, true_v, pred_v = hydragnn_amd.run_prediction(config)
    finally:
        os.chdir(cwd)
    res = {"log_name": get_log_name_config(config), "test_error": float(error),
           "task_errors": [float(t) for t in tasks],
           "task_mae": [float(torch.nn.functional.l1_loss(p, t)) for p, t in zip(pred_v, true_v)
                        if torch.is_tensor(p) and torch.is_tensor(t) and p.numel() == t.numel() and p.numel()]}
    if rank == 0:
        with open(os.path.join(workdir, res["log_name"] + "_result.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)
    return res
