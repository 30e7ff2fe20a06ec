"""Covalent radii and the MACE distance transforms (reference
``utils/model/mace_utils/modules/radial.py:151-248``, which reads the radii from
``ase.data.covalent_radii``; ase is not available here, so the table is embedded).

Radii: B. Cordero et al., "Covalent radii revisited", Dalton Trans. 2008, 2832 (the
source of ase's table), indexed by atomic number with entry 0 (dummy "X") = 0.2;
low-spin values for Mn/Fe/Co and sp3 for C, as ase chooses; elements past Cm, which
the paper does not cover, carry ase's 0.2 placeholder.  Parity with ase itself is
unpinned (ase cannot be imported in this environment); the tests check the table's
shape/anchor values and the transforms' analytic properties.
"""
import torch
from torch import nn

_MISSING = 0.2
COVALENT_RADII = [
    _MISSING,
    0.31, 0.28,                                                              # H He
    1.28, 0.96, 0.84, 0.76, 0.71, 0.66, 0.57, 0.58,                          # Li-Ne
    1.66, 1.41, 1.21, 1.11, 1.07, 1.05, 1.02, 1.06,                          # Na-Ar
    2.03, 1.76, 1.70, 1.60, 1.53, 1.39, 1.39, 1.32, 1.26, 1.24, 1.32, 1.22,  # K-Zn
    1.22, 1.20, 1.19, 1.20, 1.20, 1.16,                                      # Ga-Kr
    2.20, 1.95, 1.90, 1.75, 1.64, 1.54, 1.47, 1.46, 1.42, 1.39, 1.45, 1.44,  # Rb-Cd
    1.42, 1.39, 1.39, 1.38, 1.39, 1.40,                                      # In-Xe
    2.44, 2.15,                                                              # Cs Ba
    2.07, 2.04, 2.03, 2.01, 1.99, 1.98, 1.98, 1.96, 1.94, 1.92, 1.92, 1.89, 1.90, 1.87, 1.87,  # La-Lu
    1.75, 1.70, 1.62, 1.51, 1.44, 1.41, 1.36, 1.36, 1.32,                    # Hf-Hg
    1.45, 1.46, 1.48, 1.40, 1.50, 1.50,                                      # Tl-Rn
    2.60, 2.21,                                                              # Fr Ra
    2.15, 2.06, 2.00, 1.96, 1.90, 1.87, 1.80, 1.69,                          # Ac-Cm
] + [_MISSING] * (118 - 96)                                                  # Bk-Og
assert len(COVALENT_RADII) == 119


class _PairTransform(nn.Module):
    """Base: per-edge r0 from the covalent radii of the two end atoms (atomic numbers Z)."""

    def __init__(self):
        super().__init__()
        self.register_buffer("covalent_radii", torch.tensor(COVALENT_RADII, dtype=torch.get_default_dtype()))

    def pair_radius(self, z_src, z_dst):
        return self.covalent_radii[z_src] + self.covalent_radii[z_dst]


class AgnesiTransform(_PairTransform):
    """y = 1 / (1 + a (x/r0)^q / (1 + (x/r0)^(q-p))),  r0 = (R_u + R_v) / 2  (ACEpotentials.jl)."""

    def __init__(self, q=0.9183, p=4.5791, a=1.0805, trainable=False):
        super().__init__()
        vals = {"q": q, "p": p, "a": a}
        for k, v in vals.items():
            t = torch.tensor(v, dtype=torch.get_default_dtype())
            if trainable:
                setattr(self, k, nn.Parameter(t))
            else:
                self.register_buffer(k, t)

    def forward(self, x, z_src, z_dst):
        u = x / (0.5 * self.pair_radius(z_src, z_dst)).view(-1, 1)
        return 1.0 / (1.0 + self.a * u.pow(self.q) / (1.0 + u.pow(self.q - self.p)))


class SoftTransform(_PairTransform):
    """y = x + tanh(-(x/r0) - a (x/r0)^b) / 2 + 1/2,  r0 = (R_u + R_v) / 4."""

    def __init__(self, a=0.2, b=3.0, trainable=False):
        super().__init__()
        for k, v in {"a": a, "b": b}.items():
            t = torch.tensor(v, dtype=torch.get_default_dtype())
            if trainable:
                setattr(self, k, nn.Parameter(t))
            else:
                self.register_buffer(k, t)

    def forward(self, x, z_src, z_dst):
        u = x / (0.25 * self.pair_radius(z_src, z_dst)).view(-1, 1)
        return x + 0.5 * torch.tanh(-u - self.a * u.pow(self.b)) + 0.5
