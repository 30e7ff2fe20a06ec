"""3-D Ising model: graph energy + per-site spin (reference
``examples/ising_model/{train_ising.py, ising_model.json}``).

Pipeline (the reference's low-level API sequence):
  1. every rank generates its share of the down-spin compositions
     (``create_configurations.generate``; the reference's ``create_dataset_mpi``);
  2. ``AbstractRawDataset.from_samples`` min-max normalises over all ranks and builds
     the radius graphs / targets like the raw-file pipeline;
  3. ``split_dataset`` -> train/val/test, stored with ``--format``:
       ``pickle``   SimplePickleWriter / SimplePickleDataset (one file per sample),
       ``columnar`` ColumnarWriter / ColumnarDataset (the ADIOS2 replacement, mmap'd),
       ``memory``   keep the lists in memory;
     ``--ddstore`` then serves each split from a ``DistDataset`` (shared-memory
     segments, any rank reads any sample: the reference's DDStore);
  4. ``create_dataloaders`` -> ``hydragnn_amd.train_model`` (update_config, model,
     DDP, optimizer, train_validate_test, save) -> test-set error.

Deviation: the reference reads these files with the LSMS text reader, which takes
positions from columns 2-4 ([y, z, spin]); positions here are the lattice sites.

Usage: python examples/ising_model/train_ising.py [--L 3] [--histogram_cutoff 100]
       [--format pickle|columnar|memory] [--ddstore] [--num_epoch 2]
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from common import base_parser, load_config  # noqa: E402
from create_configurations import compositions, generate  # noqa: E402

import hydragnn_amd  # noqa: E402
from hydragnn_amd.data.datasets import (AbstractRawDataset, ColumnarDataset, ColumnarWriter,  # noqa: E402
                                        DistDataset, SimplePickleDataset, SimplePickleWriter)
from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.load_data import create_dataloaders  # noqa: E402
from hydragnn_amd.data.splitting import split_dataset  # noqa: E402
from hydragnn_amd.parallel.distributed import get_comm_size_and_rank, nsplit, setup_ddp  # noqa: E402
from hydragnn_amd.train.train_validate_test import test  # noqa: E402


def raw_samples(L, cutoff, rank, world, seed, scale_spin=False):
    mine = list(nsplit(compositions(L), world))[rank]
    feats, energies = generate(L, cutoff, n_down_list=mine, scale_spin=scale_spin, seed=seed + rank)
    out = []
    for f, e in zip(feats, energies):
        f = torch.from_numpy(f).float()
        out.append(Graph(x=torch.stack([f[:, 0], f[:, 4]], 1), pos=f[:, 1:4].contiguous(),
                         y=torch.tensor([e], dtype=torch.float32)))
    return out


def store(fmt, splits, basedir, minmax, ddstore, ddstore_width):
    labels = ("trainset", "valset", "testset")
    if fmt == "pickle":
        for lab, s in zip(labels, splits):
            SimplePickleWriter(s, basedir, lab, minmax_node_feature=minmax[0], minmax_graph_feature=minmax[1])
        sets = [SimplePickleDataset(basedir, lab) for lab in labels]
    elif fmt == "columnar":
        w = ColumnarWriter(basedir)
        for lab, s in zip(labels, splits):
            w.add(lab, s)
        w.add_global("minmax_node_feature", np.asarray(minmax[0]))
        w.add_global("minmax_graph_feature", np.asarray(minmax[1]))
        w.save()
        sets = [ColumnarDataset(basedir, lab) for lab in labels]
    else:
        sets = [list(s) for s in splits]
    if ddstore:
        # each rank contributes its slice of the split; every rank can then read every sample
        rank, world = get_comm_size_and_rank()[1], get_comm_size_and_rank()[0]
        sets = [DistDataset([ds[i] for i in list(nsplit(range(len(ds)), world))[rank]], lab,
                            ddstore_width=ddstore_width) for ds, lab in zip(sets, labels)]
    return sets


def main(argv=None):
    ap = base_parser(__doc__.splitlines()[0], "ising_model.json")
    ap.add_argument("--L", type=int, default=3, help="lattice edge (L^3 sites)")
    ap.add_argument("--histogram_cutoff", type=int, default=100, help="configurations per composition")
    ap.add_argument("--scale_spin", action="store_true", help="scale spins by U(0,1) per site")
    ap.add_argument("--format", default="pickle", choices=["pickle", "columnar", "memory"])
    ap.add_argument("--ddstore", action="store_true", help="serve splits from DistDataset")
    ap.add_argument("--ddstore_width", type=int, default=None)
    args = ap.parse_args(argv)
    config = load_config(HERE, args)
    wd = os.path.abspath(args.workdir or os.getcwd())
    os.makedirs(wd, exist_ok=True)
    setup_ddp()
    world, rank = get_comm_size_and_rank()
    raw = raw_samples(args.L, args.histogram_cutoff, rank, world, args.seed, args.scale_spin)
    ds = AbstractRawDataset.from_samples(raw, config, dist=world > 1)
    tr, va, te = split_dataset(ds.dataset, config["NeuralNetwork"]["Training"]["perc_train"], False)
    basedir = os.path.join(wd, "dataset", f"{config['Dataset']['name']}.{args.format}")
    trainset, valset, testset = store(args.format, (tr, va, te), basedir,
                                      (ds.minmax_node_feature, ds.minmax_graph_feature), args.ddstore,
                                      args.ddstore_width)
    loaders = create_dataloaders(trainset, valset, testset, config["NeuralNetwork"]["Training"]["batch_size"])
    cwd = os.getcwd()
    os.chdir(wd)
    try:
        model = hydragnn_amd.train_model(config, *loaders)
        err, tasks, _, _ = test(loaders[2], model, 0, return_samples=False)
    finally:
        os.chdir(cwd)
    res = {"test_error": float(err), "task_errors": [float(t) for t in tasks], "num_samples_local": len(raw)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
