"""Element symbol <-> atomic number and standard atomic weights (the subset of ase.data
the raw readers/writers need; symbols from ``utils/descriptors.py``)."""
from ..utils.descriptors import SYMBOLS

# standard atomic weights (IUPAC, conventional values; mass number of the most stable
# isotope for elements without a standard weight), Z = 1..118
ATOMIC_WEIGHTS = (
    1.008, 4.0026, 6.94, 9.0122, 10.81, 12.011, 14.007, 15.999, 18.998, 20.180,
    22.990, 24.305, 26.982, 28.085, 30.974, 32.06, 35.45, 39.948, 39.098, 40.078,
    44.956, 47.867, 50.942, 51.996, 54.938, 55.845, 58.933, 58.693, 63.546, 65.38,
    69.723, 72.630, 74.922, 78.971, 79.904, 83.798, 85.468, 87.62, 88.906, 91.224,
    92.906, 95.95, 97.0, 101.07, 102.91, 106.42, 107.87, 112.41, 114.82, 118.71,
    121.76, 127.60, 126.90, 131.29, 132.91, 137.33, 138.91, 140.12, 140.91, 144.24,
    145.0, 150.36, 151.96, 157.25, 158.93, 162.50, 164.93, 167.26, 168.93, 173.05,
    174.97, 178.49, 180.95, 183.84, 186.21, 190.23, 192.22, 195.08, 196.97, 200.59,
    204.38, 207.2, 208.98, 209.0, 210.0, 222.0, 223.0, 226.0, 227.0, 232.04,
    231.04, 238.03, 237.0, 244.0, 243.0, 247.0, 247.0, 251.0, 252.0, 257.0,
    258.0, 259.0, 262.0, 267.0, 270.0, 269.0, 270.0, 270.0, 278.0, 281.0,
    281.0, 285.0, 286.0, 289.0, 289.0, 293.0, 293.0, 294.0,
)


def atomic_number(symbol):
    s = symbol.strip()
    s = s[0].upper() + s[1:].lower()
    return SYMBOLS.index(s) + 1


def element_symbol(z):
    return SYMBOLS[int(z) - 1]


def atomic_mass(z):
    return ATOMIC_WEIGHTS[int(z) - 1]
