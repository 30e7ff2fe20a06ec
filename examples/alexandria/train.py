"""Alexandria: DFT bulk crystals (reference ``examples/alexandria``).

Energy (``alexandria_energy.json``) or force (``alexandria_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/alexandria/train.py [--inputfile alexandria_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("alexandria", HERE)
