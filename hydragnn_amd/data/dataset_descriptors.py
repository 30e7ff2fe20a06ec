"""Feature-column enums of the LSMS format (reference ``preprocess/dataset_descriptors.py:15-32``)."""
from enum import Enum


class AtomFeatures(Enum):
    """Node-feature column indexes of LSMS data."""

    NUM_OF_PROTONS = 0
    CHARGE_DENSITY = 1
    MAGNETIC_MOMENT = 2


class StructureFeatures(Enum):
    """Graph-feature column indexes of LSMS data."""

    FREE_ENERGY = 0
    CHARGE_DENSITY = 1
    MAGNETIC_MOMENT = 2
