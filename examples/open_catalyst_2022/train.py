"""OC22: oxide slabs + adsorbates, periodic in x/y (reference ``examples/open_catalyst_2022``).

Energy (``open_catalyst_2022_energy.json``) or force (``open_catalyst_2022_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/open_catalyst_2022/train.py [--inputfile open_catalyst_2022_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("open_catalyst_2022", HERE)
