"""Atomic descriptors / embeddings (reference ``hydragnn/utils/descriptors_and_embeddings/
atomicdescriptors.py:12-243``).

The reference builds per-element feature vectors from ``mendeleev`` (not installed here
and not installable).  This module computes the same families of features without it:

* exact, from the atomic number alone (aufbau / IUPAC table layout): group, period,
  block (s/p/d/f one-hot), number of valence electrons;
* from an embedded table for Z = 1-36 (standard reference values: IUPAC standard atomic
  weights, Pauling electronegativities, Cordero et al. 2008 covalent radii, NIST first
  ionization energies); elements outside the table get 0 for these columns and a
  ``has_table`` flag of 0.

Parity against mendeleev is unpinned (the library is absent); the feature layout is
documented in :attr:`atomicdescriptors.feature_names`.  ``one_hot`` converts integer
properties to one-hot and real properties to 10-bin one-hot, like the reference.
SMILES / RDKit featurisation (``smiles_utils.py``, ``xyz2mol.py``) needs RDKit, which is
absent: :func:`generate_graphdata_from_smilestr` raises a clear ImportError.
"""
import json
import os

import torch
import torch.nn.functional as F

SYMBOLS = ("H He Li Be B C N O F Ne Na Mg Al Si P S Cl Ar K Ca Sc Ti V Cr Mn Fe Co Ni Cu Zn Ga Ge As Se Br Kr "
           "Rb Sr Y Zr Nb Mo Tc Ru Rh Pd Ag Cd In Sn Sb Te I Xe Cs Ba La Ce Pr Nd Pm Sm Eu Gd Tb Dy Ho Er Tm "
           "Yb Lu Hf Ta W Re Os Ir Pt Au Hg Tl Pb Bi Po At Rn Fr Ra Ac Th Pa U Np Pu Am Cm Bk Cf Es Fm Md No Lr "
           "Rf Db Sg Bh Hs Mt Ds Rg Cn Nh Fl Mc Lv Ts Og").split()

# Z: (atomic weight, Pauling electronegativity (0 = undefined), covalent radius [A], 1st ionization energy [eV])
_TABLE = {
    1: (1.008, 2.20, 0.31, 13.598), 2: (4.0026, 0.0, 0.28, 24.587), 3: (6.94, 0.98, 1.28, 5.392),
    4: (9.0122, 1.57, 0.96, 9.323), 5: (10.81, 2.04, 0.84, 8.298), 6: (12.011, 2.55, 0.76, 11.260),
    7: (14.007, 3.04, 0.71, 14.534), 8: (15.999, 3.44, 0.66, 13.618), 9: (18.998, 3.98, 0.57, 17.423),
    10: (20.180, 0.0, 0.58, 21.565), 11: (22.990, 0.93, 1.66, 5.139), 12: (24.305, 1.31, 1.41, 7.646),
    13: (26.982, 1.61, 1.21, 5.986), 14: (28.085, 1.90, 1.11, 8.152), 15: (30.974, 2.19, 1.07, 10.487),
    16: (32.06, 2.58, 1.05, 10.360), 17: (35.45, 3.16, 1.02, 12.968), 18: (39.948, 0.0, 1.06, 15.760),
    19: (39.098, 0.82, 2.03, 4.341), 20: (40.078, 1.00, 1.76, 6.113), 21: (44.956, 1.36, 1.70, 6.561),
    22: (47.867, 1.54, 1.60, 6.828), 23: (50.942, 1.63, 1.53, 6.746), 24: (51.996, 1.66, 1.39, 6.767),
    25: (54.938, 1.55, 1.39, 7.434), 26: (55.845, 1.83, 1.32, 7.902), 27: (58.933, 1.88, 1.26, 7.881),
    28: (58.693, 1.91, 1.24, 7.640), 29: (63.546, 1.90, 1.32, 7.726), 30: (65.38, 1.65, 1.22, 9.394),
    31: (69.723, 1.81, 1.22, 5.999), 32: (72.630, 2.01, 1.20, 7.899), 33: (74.922, 2.18, 1.19, 9.789),
    34: (78.971, 2.55, 1.20, 9.752), 35: (79.904, 2.96, 1.20, 11.814), 36: (83.798, 3.00, 1.16, 14.000),
}

_PERIOD_STARTS = (1, 3, 11, 19, 37, 55, 87, 119)


def period_of(z):
    for p in range(1, 8):
        if z < _PERIOD_STARTS[p]:
            return p
    return 7


def group_block_of(z):
    """IUPAC group (1-18; 3 for lanthanides/actinides) and block index (0=s,1=p,2=d,3=f)."""
    p = period_of(z)
    k = z - _PERIOD_STARTS[p - 1]  # 0-based position in the period
    if p == 1:
        return (1, 0) if z == 1 else (18, 0)
    if p in (2, 3):
        return (k + 1, 0) if k < 2 else (k + 11, 1)
    if p in (4, 5):
        if k < 2:
            return k + 1, 0
        return (k + 1, 2) if k < 12 else (k + 1, 1)
    # periods 6/7: 2 s, 14 f (group 3 by convention), 10 d, 6 p
    if k < 2:
        return k + 1, 0
    if k < 16:
        return 3, 3
    if k < 26:
        return k - 13, 2
    return k - 13, 1


def valence_electrons(z):
    g, b = group_block_of(z)
    if b == 0:
        return g if z != 2 else 2
    if b == 1:
        return g - 10
    if b == 2:
        return g
    return 3


class atomicdescriptors:
    feature_names = ["type_id", "group", "period", "block(onehot4)", "valence_electrons", "atomic_number",
                     "atomic_weight", "electronegativity", "covalent_radius", "ionization_energy", "has_table"]

    def __init__(self, embeddingfilename, overwritten=True, element_types=("C", "H", "O", "N", "F", "S"),
                 one_hot=False):
        if os.path.exists(embeddingfilename) and not overwritten:
            with open(embeddingfilename) as f:
                self.atom_embeddings = json.load(f)
            return
        syms = list(SYMBOLS) if element_types is None else [s for s in SYMBOLS if s in element_types]
        self.element_types = syms
        zs = [SYMBOLS.index(s) + 1 for s in syms]
        cols = []
        ids = torch.arange(len(zs)).view(-1, 1).float()
        gb = [group_block_of(z) for z in zs]
        group = torch.tensor([g for g, _ in gb]).view(-1, 1)
        period = torch.tensor([period_of(z) for z in zs]).view(-1, 1)
        block = F.one_hot(torch.tensor([b for _, b in gb]), 4).float()
        val = torch.tensor([valence_electrons(z) for z in zs]).view(-1, 1)
        zt = torch.tensor(zs).view(-1, 1)
        tab = torch.tensor([_TABLE.get(z, (0.0, 0.0, 0.0, 0.0)) for z in zs], dtype=torch.float32)
        has = torch.tensor([[1.0 if z in _TABLE else 0.0] for z in zs])
        if one_hot:
            ints = [self._int_onehot(t) for t in (group, period, zt, val)]
            reals = [self._real_onehot(tab[:, i:i + 1]) for i in range(4)]
            cols = [F.one_hot(ids.long().view(-1), len(zs)).float(), ints[0], ints[1], block, ints[3], ints[2]] + \
                reals + [has]
        else:
            cols = [ids, group.float(), period.float(), block, val.float(), zt.float(), tab, has]
        emb = torch.cat(cols, 1)
        self.atom_embeddings = {str(z): emb[i].tolist() for i, z in enumerate(zs)}
        with open(embeddingfilename, "w") as f:
            json.dump(self.atom_embeddings, f)

    @staticmethod
    def _int_onehot(v):
        return F.one_hot(v.view(-1) - v.min(), int(v.max() - v.min()) + 1).float()

    @staticmethod
    def _real_onehot(v, num_classes=10):
        lo, hi = float(v.min()), float(v.max())
        idx = ((v.view(-1) - lo) / max(hi - lo, 1e-12) * (num_classes - 1)).round().long()
        return F.one_hot(idx, num_classes).float()

    def get_atom_features(self, atomtype):
        return torch.tensor(self.atom_embeddings[str(int(atomtype))])


from .smiles import generate_graphdata_from_smilestr, get_node_attribute_name  # noqa: E402,F401  (RDKit-free)
