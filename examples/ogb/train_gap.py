"""PCQM4Mv2 HOMO-LUMO gap from SMILES (reference ``examples/ogb/{train_gap.py, ogb_gap.json}``:
PNA, hidden 55, 6 layers, 31 element types + 6 RDKit-style atom features = 37 inputs).

The OGB CSV cannot be downloaded here: ``--csv`` reads a ``smiles,gap`` table, else one
is generated (``examples/smiles_common.py``).  Graphs: the RDKit-free SMILES reader
with explicit hydrogens; training through ``create_dataloaders`` -> ``train_model``.

Usage: python examples/ogb/train_gap.py [--num_samples 1000] [--num_epoch 2] [--csv gap.csv]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import smiles_common as sc  # noqa: E402

OGB_NODE_TYPES = {s: i for i, s in enumerate(
    ["H", "B", "C", "N", "O", "F", "Si", "P", "S", "Cl", "Ca", "Ge", "As", "Se", "Br", "I", "Mg", "Ti", "Ga", "Zn",
     "Ar", "Be", "He", "Al", "Kr", "V", "Na", "Li", "Cu", "Ne", "Ni"])}


def main(argv=None):
    args = sc.parser(__doc__.splitlines()[0], "ogb_gap.json").parse_args(argv)
    config, workdir = sc.load(HERE, args)
    path = args.csv or sc.make_table(os.path.join(workdir, "pcqm4m_gap.csv"), args.num_samples, "gap", seed=args.seed,
                                     elements=set(OGB_NODE_TYPES))
    smiles, ys = sc.read_table(path)
    var = sc.var_config_for(config, [1], len(OGB_NODE_TYPES) + 6)
    samples = sc.graphs_from_table(smiles, ys, OGB_NODE_TYPES, var)
    return sc.train_and_test(config, samples, "ogb_gap", seed=args.seed)


if __name__ == "__main__":
    main()
