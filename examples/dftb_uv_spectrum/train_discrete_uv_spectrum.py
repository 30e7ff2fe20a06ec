"""DFTB discrete UV spectra (reference ``examples/dftb_uv_spectrum/
{train_discrete_uv_spectrum.py, dftb_discrete_uv_spectrum.json}``: PNA, two graph heads —
excitation energies and oscillator strengths of the lowest ``--npeaks`` transitions).

Synthetic transitions from the molecules' conjugation (``examples/smiles_common.py``).

Usage: python examples/dftb_uv_spectrum/train_discrete_uv_spectrum.py [--num_samples 500] [--npeaks 4]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import smiles_common as sc  # noqa: E402

DFTB_NODE_TYPES = {"C": 0, "F": 1, "H": 2, "N": 3, "O": 4, "S": 5}


def main(argv=None):
    ap = sc.parser(__doc__.splitlines()[0], "dftb_discrete_uv_spectrum.json")
    ap.add_argument("--npeaks", type=int, default=4)
    args = ap.parse_args(argv)
    config, workdir = sc.load(HERE, args)
    config["NeuralNetwork"]["Variables_of_interest"]["output_dim"] = [args.npeaks, args.npeaks]
    path = args.csv or sc.make_table(os.path.join(workdir, "dftb_discrete.csv"), args.num_samples, "discrete",
                                     seed=args.seed, npeaks=args.npeaks, elements=set(DFTB_NODE_TYPES))
    smiles, ys = sc.read_table(path)
    var = sc.var_config_for(config, [args.npeaks, args.npeaks], len(DFTB_NODE_TYPES) + 6)
    samples = sc.graphs_from_table(smiles, ys, DFTB_NODE_TYPES, var)
    return sc.train_and_test(config, samples, "dftb_discrete_uv_spectrum", seed=args.seed)


if __name__ == "__main__":
    main()
