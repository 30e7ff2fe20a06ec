"""OMol25: molecules/complexes across the periodic table (reference ``examples/open_molecules_2025``).

Energy (``open_molecules_2025_energy.json``) or force (``open_molecules_2025_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/open_molecules_2025/train.py [--inputfile open_molecules_2025_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("open_molecules_2025", HERE)
