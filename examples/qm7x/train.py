"""QM7-X: small organic molecules (C, N, O, S, Cl + H), non-equilibrium conformers (reference ``examples/qm7x``).

Energy (``qm7x_energy.json``) or force (``qm7x_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/qm7x/train.py [--inputfile qm7x_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("qm7x", HERE)
