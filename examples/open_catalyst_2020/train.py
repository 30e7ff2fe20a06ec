"""OC20-S2EF-style adsorbate/slab energies (reference ``examples/open_catalyst_2020/train.py``
+ ``open_catalyst_energy.json``: EGNN, 3 layers, radius 10, max_neighbours 10,
edge length feature, MAE loss, batch 32).

``open_catalyst_gps.json`` is the headline benchmark configuration of this
framework (BASELINE config 4): PNAPlus + GPS (8 heads, pe_dim 16, hidden 64);
``bench.py`` times exactly that model on the HBM-resident hipGraph path.

The OC20 download is unavailable offline: ``oc20_like`` generates systems of
20-126 atoms (mean ~73, atomic numbers 1-83) at solid density with a smooth
size-extensive pseudo-energy; the target is energy per atom.

Usage: python examples/open_catalyst_2020/train.py [--inputfile open_catalyst_gps.json] [--num_samples 2000]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import base_parser, load_config, run_example, split  # noqa: E402

from hydragnn_amd.data.synthetic import oc20_like  # noqa: E402


def main(argv=None):
    args = base_parser(__doc__.splitlines()[0], "open_catalyst_energy.json").parse_args(argv)
    config = load_config(HERE, args)
    arch = config["NeuralNetwork"]["Architecture"]
    samples = oc20_like(args.num_samples or 2000, seed=args.seed, radius=arch["radius"],
                        max_neighbours=arch["max_neighbours"], pe_dim=1)
    for s in samples:  # the serialized pipeline rebuilds edges / PE from positions
        for k in ("edge_index", "edge_attr", "pe", "rel_pe", "y_loc"):
            if k in s:
                delattr(s, k)
    tr, va, te = split(samples, config["NeuralNetwork"]["Training"]["perc_train"], seed=args.seed)
    return run_example(config, tr, va, te, args.workdir)


if __name__ == "__main__":
    main()
