"""CSCE HOMO-LUMO gap from SMILES (reference ``examples/csce/{train_gap.py, csce_gap.json}``:
PNA, hidden 200, 6 layers, element types C/F/H/N/O/S + 6 atom features = 12 inputs).

The CSCE table cannot be downloaded here: ``--csv`` reads a ``smiles,gap`` table, else
one is generated from C/F/N/O/S fragments (``examples/smiles_common.py``).

Usage: python examples/csce/train_gap.py [--num_samples 1000] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import smiles_common as sc  # noqa: E402

CSCE_NODE_TYPES = {"C": 0, "F": 1, "H": 2, "N": 3, "O": 4, "S": 5}


def main(argv=None):
    args = sc.parser(__doc__.splitlines()[0], "csce_gap.json").parse_args(argv)
    config, workdir = sc.load(HERE, args)
    path = args.csv or sc.make_table(os.path.join(workdir, "csce_gap.csv"), args.num_samples, "gap", seed=args.seed,
                                     elements=set(CSCE_NODE_TYPES))
    smiles, ys = sc.read_table(path)
    var = sc.var_config_for(config, [1], len(CSCE_NODE_TYPES) + 6)
    samples = sc.graphs_from_table(smiles, ys, CSCE_NODE_TYPES, var)
    return sc.train_and_test(config, samples, "csce_gap", seed=args.seed)


if __name__ == "__main__":
    main()
