"""ODAC23: metal-organic frameworks + CO2 / H2O (reference ``examples/open_direct_air_capture_2023``).

Energy (``open_direct_air_capture_2023_energy.json``) or force (``open_direct_air_capture_2023_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/open_direct_air_capture_2023/train.py [--inputfile open_direct_air_capture_2023_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("open_direct_air_capture_2023", HERE)
