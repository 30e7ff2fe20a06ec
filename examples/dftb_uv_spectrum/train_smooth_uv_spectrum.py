"""DFTB UV spectra from molecular graphs (reference ``examples/dftb_uv_spectrum/
{train_smooth_uv_spectrum.py, dftb_smooth_uv_spectrum.json}``: PNA, hidden 200, 6 layers,
one graph head predicting the whole smoothed spectrum; the reference grid has 37500
points, the synthetic default 500 — ``--spectrum_dim`` sets it and the head width).

The DFTB+ outputs (smiles.pdb + spectrum files per molecule) cannot be downloaded here:
spectra are generated as Gaussian bands whose positions follow the conjugation length
(``examples/smiles_common.py``).

Usage: python examples/dftb_uv_spectrum/train_smooth_uv_spectrum.py [--num_samples 500] [--spectrum_dim 500]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import smiles_common as sc  # noqa: E402

DFTB_NODE_TYPES = {"C": 0, "F": 1, "H": 2, "N": 3, "O": 4, "S": 5}


def main(argv=None):
    ap = sc.parser(__doc__.splitlines()[0], "dftb_smooth_uv_spectrum.json")
    ap.add_argument("--spectrum_dim", type=int, default=500)
    args = ap.parse_args(argv)
    config, workdir = sc.load(HERE, args)
    config["NeuralNetwork"]["Variables_of_interest"]["output_dim"] = [args.spectrum_dim]
    path = args.csv or sc.make_table(os.path.join(workdir, "dftb_spectrum.csv"), args.num_samples, "spectrum",
                                     seed=args.seed, spectrum_dim=args.spectrum_dim, elements=set(DFTB_NODE_TYPES))
    smiles, ys = sc.read_table(path)
    var = sc.var_config_for(config, [args.spectrum_dim], len(DFTB_NODE_TYPES) + 6)
    samples = sc.graphs_from_table(smiles, ys, DFTB_NODE_TYPES, var)
    return sc.train_and_test(config, samples, "dftb_smooth_uv_spectrum", seed=args.seed)


if __name__ == "__main__":
    main()
