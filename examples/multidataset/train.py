"""Multi-dataset (GFM) training over several columnar stores (reference
``examples/multidataset/train.py`` + ``gfm_*.json``).

Formats (reference flags):
  ``--multi`` (default here): ``--multi_model_list A,B,C`` names one store per dataset
     (``dataset/<name>.bp``, ColumnarWriter layout).  Rank 0 reads every store's train
     size and PNA degree histogram; ranks are assigned to datasets in proportion to the
     sizes (``proportional_process_list``), the histograms are merged by spline
     resampling (``merge_pna_deg``, C21), both are broadcast; each rank then reads its
     slice of its own dataset (``setsubset``) inside a per-dataset process group;
  ``--adios``: one store (``--modelname``), every rank reads the whole split and the
     loaders shard it.
``--ddstore`` re-serves the splits from ``DistDataset`` (shared-memory segments;
every rank can read every sample, so the loaders shard the union of all datasets);
``--shmem`` keeps the stores memory-mapped (one page-cache copy per node shared by
all ranks) instead of loading a private copy per rank.  ``--num_samples`` /
``--num_test_samples`` cap the per-rank shard (weak-scaling runs).

The SC25 datasets (ANI1x, QM7-X, MPTrj, ...) are not downloadable here; a missing store is
generated (``--prepare_samples`` samples, rank 0): molecules of a per-dataset size
range with exact forces of a smooth pseudo-potential, node features
[Z, x, y, z, fx, fy, fz], graph feature [energy].

Usage: python examples/multidataset/train.py --multi_model_list ANI1x,QM7-X [--ddstore]
       torchrun --nproc-per-node 4 examples/multidataset/train.py --multi_model_list ANI1x,QM7-X,MPTrj
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import load_config  # noqa: E402

import hydragnn_amd  # noqa: E402
from hydragnn_amd.data.datasets import COMM_SELF, ColumnarDataset, ColumnarWriter, DistDataset  # noqa: E402
from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.load_data import create_dataloaders  # noqa: E402
from hydragnn_amd.data.serialized import SerializedDataLoader  # noqa: E402
from hydragnn_amd.data.splitting import split_dataset  # noqa: E402
from hydragnn_amd.data.synthetic import molecules_like  # noqa: E402
from hydragnn_amd.parallel.distributed import get_comm_size_and_rank, nsplit, setup_ddp  # noqa: E402
from hydragnn_amd.train.train_validate_test import test  # noqa: E402
from hydragnn_amd.utils.config_utils import gather_deg, merge_pna_deg, proportional_process_list  # noqa: E402

NODE_FEATURE_NAMES, NODE_FEATURE_DIMS = ["atomic_number", "cartesian_coordinates", "forces"], [1, 3, 3]
GRAPH_FEATURE_NAMES, GRAPH_FEATURE_DIMS = ["energy"], [1]
COMMON_KEYS = ["x", "edge_index", "edge_attr", "energy", "forces", "pos", "y", "y_loc"]


def make_store(path, name, k, num, config, seed=0):
    """Generate + preprocess dataset ``name`` (family index k) and write its columnar store."""
    lo, hi = 3 + 4 * k, 10 + 8 * k
    raw = []
    for s in molecules_like(num, seed=seed + 7919 * (k + 1), min_atoms=lo, max_atoms=hi, with_forces=True):
        raw.append(Graph(x=torch.cat([s.x, s.pos, s.forces], 1), pos=s.pos, y=s.energy.view(-1),
                         energy=s.energy, forces=s.forces))
    pcfg = json.loads(json.dumps(config))
    pcfg["Dataset"] = {"name": name, "node_features": {"name": NODE_FEATURE_NAMES, "dim": NODE_FEATURE_DIMS},
                       "graph_features": {"name": GRAPH_FEATURE_NAMES, "dim": GRAPH_FEATURE_DIMS}}
    var = pcfg["NeuralNetwork"]["Variables_of_interest"]
    var["input_node_features"] = list(range(7))  # keep every column in the store; readers select
    samples = SerializedDataLoader(pcfg).process(raw)
    tr, va, te = split_dataset(samples, config["NeuralNetwork"]["Training"]["perc_train"], False)
    w = ColumnarWriter(path, comm=COMM_SELF)  # rank 0 alone
    for lab, s in (("trainset", tr), ("valset", va), ("testset", te)):
        w.add(lab, s)
    w.add_global("pna_deg", np.asarray(_local_deg(tr)))
    w.save()


def _local_deg(samples):
    md = max(int(torch.bincount(d.edge_index[1], minlength=d.num_nodes).max()) for d in samples)
    deg = np.zeros(md + 1, dtype=np.int64)
    for d in samples:
        deg += np.bincount(torch.bincount(d.edge_index[1], minlength=d.num_nodes).numpy(), minlength=md + 1)
    return deg


def _bcast(obj):
    if dist.is_initialized():
        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]
    return obj


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--inputfile", default="gfm_multitasking.json")
    ap.add_argument("--multi_model_list", default="ANI1x,QM7-X")
    ap.add_argument("--modelname", default=None, help="single store for --adios")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--adios", dest="format", action="store_const", const="adios")
    g.add_argument("--multi", dest="format", action="store_const", const="multi")
    ap.set_defaults(format="multi")
    ap.add_argument("--ddstore", action="store_true")
    ap.add_argument("--ddstore_width", type=int, default=None)
    ap.add_argument("--shmem", action="store_true")
    ap.add_argument("--num_samples", type=int, default=None, help="per-rank train/val samples")
    ap.add_argument("--num_test_samples", type=int, default=None)
    ap.add_argument("--num_epoch", type=int, default=None)
    ap.add_argument("--batch_size", type=int, default=None)
    ap.add_argument("--log", default=None)
    ap.add_argument("--prepare_samples", type=int, default=200, help="samples per generated store")
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--hidden_dim", type=int, default=None)
    ap.add_argument("--num_conv_layers", type=int, default=None)
    ap.add_argument("--learning_rate", type=float, default=None)
    ap.add_argument("--mpnn_type", default=None)
    args = ap.parse_args(argv)
    assert not (args.shmem and args.ddstore), "Cannot use both ddstore and shmem"
    args.mpnn_type = args.global_attn_engine = args.global_attn_type = args.pe_dim = None
    config = load_config(HERE, args)
    var = config["NeuralNetwork"]["Variables_of_interest"]
    var.update(graph_feature_names=GRAPH_FEATURE_NAMES, graph_feature_dims=GRAPH_FEATURE_DIMS,
               node_feature_names=NODE_FEATURE_NAMES, node_feature_dims=NODE_FEATURE_DIMS)
    wd = os.path.abspath(args.workdir or os.getcwd())
    os.makedirs(os.path.join(wd, "dataset"), exist_ok=True)
    setup_ddp()
    world, rank = get_comm_size_and_rank()
    models = args.multi_model_list.split(",") if args.format == "multi" else [args.modelname or "GFM"]
    store = lambda m: os.path.join(wd, "dataset", f"{m}.bp")  # noqa: E731
    if rank == 0:
        for k, m in enumerate(models):
            if not os.path.isdir(store(m)):
                make_store(store(m), m, k, args.prepare_samples, config, args.seed)
    if dist.is_initialized():
        dist.barrier()
    opt = {"preload": not args.shmem}
    if args.format == "multi":
        info = None
        if rank == 0:
            nd = [ColumnarDataset(store(m), "trainset").ntotal for m in models]
            degs = [ColumnarDataset(store(m), "trainset").pna_deg.numpy() for m in models]
            info = (proportional_process_list(nd, world), merge_pna_deg(degs))
        process_list, pna_deg = _bcast(info)
        colors = [c for c, n in enumerate(process_list) for _ in range(n)]
        color = colors[rank]
        groups = [dist.new_group([r for r in range(world) if colors[r] == c]) for c in range(len(models))] \
            if dist.is_initialized() else [None]
        local_ranks = [r for r in range(world) if colors[r] == color]
        lrank, lsize = local_ranks.index(rank), len(local_ranks)
        sets = []
        for lab in ("trainset", "valset", "testset"):
            ds = ColumnarDataset(store(models[color]), lab, keys=COMMON_KEYS, var_config=var, **opt)
            rx = list(nsplit(range(len(ds)), lsize))[lrank]
            cap = args.num_test_samples if lab == "testset" and args.num_test_samples else args.num_samples
            if cap is not None:
                rx = rx[:cap]
            ds.setsubset(rx[0], rx[-1] + 1)
            sets.append(ds)
        del groups  # created on every rank (collective); the branch-local syncs use them in MultiTaskModelMP runs
    else:
        sets = [ColumnarDataset(store(models[0]), lab, keys=COMMON_KEYS, var_config=var, **opt)
                for lab in ("trainset", "valset", "testset")]
        pna_deg = sets[0].pna_deg.tolist()
    local = args.format == "multi"
    if args.ddstore:
        sets = [DistDataset(list(s), lab, ddstore_width=args.ddstore_width, var_config=None)
                for s, lab in zip(sets, ("trainset", "valset", "testset"))]
        local = False  # every rank can read every sample: shard the union
    for s in sets:
        s.pna_deg = pna_deg
    loaders = create_dataloaders(*sets, config["NeuralNetwork"]["Training"]["batch_size"], test_sampler_shuffle=False,
                                 local=local)
    cwd = os.getcwd()
    os.chdir(wd)
    try:
        model = hydragnn_amd.train_model(config, *loaders, log_name=args.log or "GFM")
        err, tasks, _, _ = test(loaders[2], model, 0, return_samples=False)
    finally:
        os.chdir(cwd)
    res = {"test_error": float(err), "task_errors": [float(t) for t in tasks], "datasets": models,
           "local_train_samples": len(sets[0])}
    if rank == 0:
        print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
