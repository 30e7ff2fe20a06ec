"""LSMS alloy data, multitask (graph free energy + node charge density + magnetic moment)
through the raw-text reader (reference ``examples/lsms/{lsms.py, lsms.json}``).

The FePt LSMS dataset is not downloadable here: ``deterministic_graph_data``
writes LSMS-format text files of random BCC configurations (the reference CI
generator) into ``dataset/FePt_enthalpy``; the raw loader normalises them,
``compositional_stratified_splitting`` splits them, and PNA trains on the three
heads with min-max denormalised predictions.

Usage: python examples/lsms/lsms.py [--num_samples 500] [--num_epoch 200]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import base_parser, load_config  # noqa: E402

import hydragnn_amd  # noqa: E402
from hydragnn_amd.data.lsms import deterministic_graph_data  # noqa: E402
from hydragnn_amd.parallel.distributed import get_comm_size_and_rank, setup_ddp  # noqa: E402


def main(argv=None):
    args = base_parser(__doc__.splitlines()[0], "lsms.json").parse_args(argv)
    config = load_config(HERE, args)
    wd = os.path.abspath(args.workdir or os.getcwd())
    os.makedirs(wd, exist_ok=True)
    setup_ddp()
    _, rank = get_comm_size_and_rank()
    raw = os.path.join(wd, "dataset", "FePt_enthalpy")
    if rank == 0 and not (os.path.isdir(raw) and os.listdir(raw)):
        deterministic_graph_data(raw, number_configurations=args.num_samples or 500, seed=args.seed)
    config["Dataset"]["path"] = {"total": raw}
    os.environ["SERIALIZED_DATA_PATH"] = wd
    cwd = os.getcwd()
    os.chdir(wd)
    try:
        hydragnn_amd.run_training(config)
        error, tasks, _, _ = hydragnn_amd.run_prediction(config)
    finally:
        os.chdir(cwd)
    res = {"test_error": float(error), "task_errors": [float(t) for t in tasks]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
