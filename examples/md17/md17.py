"""MD17-style molecular dynamics frames (reference ``examples/md17/{md17.py, md17.json}``).

Two configurations ship:
* ``md17.json`` — the reference's: SchNet + GPS (pe_dim 6, 6 layers), graph energy;
* ``md17_forces.json`` — BASELINE config 3: PAINN (equivariant), per-node energy head,
  ``compute_grad_energy``: trained on energies and forces = -dE/dpos.

The MD17 download is unavailable offline: ``md_trajectory`` perturbs ONE
QM9-shaped molecule (21 atoms) and labels every frame with the exact energy and
forces of a smooth pseudo-potential.

Usage: python examples/md17/md17.py [--inputfile md17_forces.json] [--num_samples 500]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import base_parser, load_config, run_example, split  # noqa: E402

from hydragnn_amd.data.synthetic import md_trajectory  # noqa: E402


def main(argv=None):
    ap = base_parser(__doc__.splitlines()[0], "md17.json")
    ap.add_argument("--num_atoms", type=int, default=21)
    args = ap.parse_args(argv)
    config = load_config(HERE, args)
    samples = md_trajectory(args.num_samples or 500, seed=args.seed, num_atoms=args.num_atoms)
    if not config["NeuralNetwork"]["Training"].get("compute_grad_energy", False):
        for s in samples:
            s.y = s.energy / s.num_nodes  # graph head: energy per atom
    tr, va, te = split(samples, config["NeuralNetwork"]["Training"]["perc_train"], seed=args.seed)
    return run_example(config, tr, va, te, args.workdir)


if __name__ == "__main__":
    main()
