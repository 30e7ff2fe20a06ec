"""Transition1x: reaction-path geometries of C/H/N/O molecules (reference ``examples/transition1x``).

Energy (``transition1x_energy.json``) or force (``transition1x_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/transition1x/train.py [--inputfile transition1x_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("transition1x", HERE)
