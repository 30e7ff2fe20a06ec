"""ANI-1x: C/H/N/O molecules, off-equilibrium sampling (reference ``examples/ani1_x``).

Energy (``ani1_x_energy.json``) or force (``ani1_x_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/ani1_x/train.py [--inputfile ani1_x_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("ani1_x", HERE)
