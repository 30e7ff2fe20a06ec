"""Ni-Nb EAM alloy: per-atom energy / forces / bulk modulus from CFG files (reference
``examples/eam/{eam.py, NiNb_EAM_*.json}``).

Pipeline (reference order): rank 0 generates the CFG dataset if absent
(``eam_data.write_dataset``; the reference ships LAMMPS output) -> ``CFGDataset``
(extended-CFG reader, periodic radius graphs, min-max normalisation) ->
``split_dataset`` (compositional stratification) -> ``SerializedWriter`` (``--pickle``,
default) or ``ColumnarWriter`` (``--adios``: the ADIOS2 replacement) ->
``SerializedDataset`` / ``ColumnarDataset`` -> ``create_dataloaders`` ->
``hydragnn_amd.train_model`` -> test error.  ``--preonly`` stops after writing,
``--loadexistingsplit`` skips the raw stage.

Configs: NiNb_EAM_energy (atomic energy), NiNb_EAM_multitask (energy + forces),
NiNb_EAM_bulk (bulk modulus), NiNb_EAM_bulk_multitask (all three).

Usage: python examples/eam/eam.py [--inputfile NiNb_EAM_multitask.json] [--num_samples 200]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from common import base_parser, load_config  # noqa: E402

import hydragnn_amd  # noqa: E402
from hydragnn_amd.data.datasets import (COMM_SELF, CFGDataset, ColumnarDataset, ColumnarWriter, SerializedDataset,  # noqa: E402
                                        SerializedWriter)
from hydragnn_amd.data.load_data import create_dataloaders  # noqa: E402
from hydragnn_amd.data.splitting import split_dataset  # noqa: E402
from hydragnn_amd.parallel.distributed import get_comm_size_and_rank, setup_ddp  # noqa: E402
from hydragnn_amd.train.train_validate_test import test  # noqa: E402


def main(argv=None):
    ap = base_parser(__doc__.splitlines()[0], "NiNb_EAM_energy.json")
    ap.add_argument("--loadexistingsplit", action="store_true", help="reuse the written splits")
    ap.add_argument("--preonly", action="store_true", help="preprocess and write only, no training")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--adios", dest="format", action="store_const", const="adios", help="columnar store")
    g.add_argument("--pickle", dest="format", action="store_const", const="pickle", help="serialized store")
    ap.set_defaults(format="pickle")
    args = ap.parse_args(argv)
    config = load_config(HERE, args)
    wd = os.path.abspath(args.workdir or os.getcwd())
    os.makedirs(wd, exist_ok=True)
    setup_ddp()
    world, rank = get_comm_size_and_rank()
    import torch.distributed as dist

    raw = os.path.join(wd, config["Dataset"]["path"]["total"])
    name = config["Dataset"]["name"]
    store_dir = os.path.join(wd, "dataset", f"{name}.bp" if args.format == "adios" else "serialized_dataset")
    labels = ("trainset", "valset", "testset")
    if not args.loadexistingsplit:
        if rank == 0 and not (os.path.isdir(raw) and os.listdir(raw)):
            from eam_data import write_dataset

            write_dataset(raw, args.num_samples or 200, seed=args.seed)
        if dist.is_initialized():
            dist.barrier()
        config["Dataset"]["path"] = {"total": raw}
        total = CFGDataset(config)
        splits = split_dataset(total.dataset, config["NeuralNetwork"]["Training"]["perc_train"],
                               config["Dataset"]["compositional_stratified_splitting"])
        if rank == 0:
            if args.format == "adios":
                w = ColumnarWriter(store_dir, comm=COMM_SELF)  # rank 0 alone
                for lab, s in zip(labels, splits):
                    w.add(lab, s)
                w.add_global("minmax_node_feature", total.minmax_node_feature)
                w.add_global("minmax_graph_feature", total.minmax_graph_feature)
                w.save()
            else:
                for lab, s in zip(labels, splits):
                    SerializedWriter(s, store_dir, name, lab, minmax_node_feature=total.minmax_node_feature,
                                     minmax_graph_feature=total.minmax_graph_feature)
        if dist.is_initialized():
            dist.barrier()
    if args.preonly:
        return {}
    if args.format == "adios":
        sets = [ColumnarDataset(store_dir, lab) for lab in labels]
    else:
        sets = [SerializedDataset(store_dir, name, lab) for lab in labels]
    var = config["NeuralNetwork"]["Variables_of_interest"]
    if var.get("denormalize_output"):  # reference: minmax taken from the stored train split
        var["minmax_node_feature"] = sets[0].minmax_node_feature
        var["minmax_graph_feature"] = sets[0].minmax_graph_feature
    loaders = create_dataloaders(*sets, config["NeuralNetwork"]["Training"]["batch_size"])
    cwd = os.getcwd()
    os.chdir(wd)
    try:
        model = hydragnn_amd.train_model(config, *loaders)
        err, tasks, _, _ = test(loaders[2], model, 0, return_samples=False)
    finally:
        os.chdir(cwd)
    res = {"test_error": float(err), "task_errors": [float(t) for t in tasks], "num_samples": sum(map(len, sets))}
    if rank == 0:
        print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
