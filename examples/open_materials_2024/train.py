"""OMat24: rattled / AIMD bulk inorganic structures (reference ``examples/open_materials_2024``).

Energy (``open_materials_2024_energy.json``) or force (``open_materials_2024_forces.json``) training of EGNN on
synthetic structures with the dataset's shape; see ``examples/atomistic.py``.

Usage: python examples/open_materials_2024/train.py [--inputfile open_materials_2024_forces.json] [--num_samples 600] [--num_epoch 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from atomistic import main  # noqa: E402

if __name__ == "__main__":
    main("open_materials_2024", HERE)
