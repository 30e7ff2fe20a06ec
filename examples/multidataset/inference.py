"""Inference of a trained GFM model on one or more dataset stores (reference
``run-scripts/SC25-inference.sh`` + ``examples/multidataset*/inference`` drivers: every
trained model (log directory) is evaluated on every dataset's test split and the
errors are logged).

Loads ``<workdir>/logs/<log>/config.json`` (the config ``train_model`` saved, with
the resolved output dims and PNA degrees) and ``<log>.pk``; reads each
``<workdir>/dataset/<name>.bp`` columnar store's ``testset``; runs ``test()`` (on a
GPU: the HBM-resident loader; sharded over ranks when launched with torchrun) and
prints one JSON line per dataset with the task errors and the inference throughput.

Usage: python examples/multidataset/inference.py --log GFM --datasets ANI1x,QM7-X [--workdir DIR]
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from hydragnn_amd.data.datasets import ColumnarDataset  # noqa: E402
from hydragnn_amd.data.load_data import create_dataloaders, to_device_loaders  # noqa: E402
from hydragnn_amd.models.create import create_model_config  # noqa: E402
from hydragnn_amd.parallel.distributed import (get_comm_size_and_rank, get_device, get_distributed_model,  # noqa: E402
                                               setup_ddp)
from hydragnn_amd.train.train_validate_test import test  # noqa: E402
from hydragnn_amd.utils.model import load_existing_model  # noqa: E402

COMMON_KEYS = ["x", "edge_index", "edge_attr", "energy", "forces", "pos", "y", "y_loc"]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--log", default="GFM")
    ap.add_argument("--datasets", default="ANI1x,QM7-X")
    ap.add_argument("--batch_size", type=int, default=None)
    ap.add_argument("--num_test_samples", type=int, default=None)
    ap.add_argument("--workdir", default=None)
    args = ap.parse_args(argv)
    wd = os.path.abspath(args.workdir or os.getcwd())
    os.chdir(wd)
    setup_ddp()
    _, rank = get_comm_size_and_rank()
    with open(os.path.join("logs", args.log, "config.json")) as f:
        config = json.load(f)
    nn_cfg = config["NeuralNetwork"]
    var = nn_cfg["Variables_of_interest"]
    model = create_model_config(config=nn_cfg, verbosity=0)
    model = get_distributed_model(model, 0)
    load_existing_model(model, args.log)
    module = model.module if hasattr(model, "module") else model
    bs = args.batch_size or nn_cfg["Training"]["batch_size"]
    out = []
    for name in args.datasets.split(","):
        ds = ColumnarDataset(os.path.join("dataset", f"{name}.bp"), "testset", keys=COMMON_KEYS, var_config=var)
        if args.num_test_samples:
            ds.setsubset(0, min(len(ds), args.num_test_samples))
        loader = create_dataloaders(ds, ds, ds, bs, test_sampler_shuffle=False)[2]
        if torch.cuda.is_available() and int(os.getenv("HYDRAGNN_DEVICE_DATA", "1")) == 1:
            loader = to_device_loaders((loader, loader, loader), get_device(), module.head_type, module.head_dims,
                                       attn_scope=getattr(module, "attn_scope", "batch"))[2]
        test(loader, model, 0, return_samples=False)  # warm-up (allocator, kernels)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        err, tasks, _, _ = test(loader, model, 0, return_samples=False)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res = {"model": args.log, "dataset": name, "test_error": float(err), "task_errors": [float(t) for t in tasks],
               "num_graphs": len(ds), "graphs_per_s": len(ds) / max(dt, 1e-9)}
        out.append(res)
        if rank == 0:
            print(json.dumps(res), flush=True)
    return out


if __name__ == "__main__":
    main()
