"""3-D periodic Ising configurations on an L^3 cubic lattice (reference
``examples/ising_model/create_configurations.py``).

Dataset definition (same Hamiltonian as the reference): spins S = f(c) of a +-1
configuration c (optionally scaled by U(0,1) per site), energy

    E = -(1/6) * sum_i S_i * (S_i + sum_{6 periodic neighbours j} S_j)

Node features per site: [c, x, y, z, S]; graph feature: [E].  For every number of down
spins the full multiset of configurations is enumerated when it is small
(binom(L^3, n_down) <= histogram_cutoff), otherwise ``histogram_cutoff`` random
permutations are drawn.  Energies are evaluated for a whole block of configurations at
once with periodic ``np.roll`` (the reference loops over sites in Python).
"""
import itertools
import math

import numpy as np


def lattice_positions(L):
    g = np.arange(L, dtype=np.float64)
    return np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)


def ising_energy(spins):
    """spins [B, L, L, L] -> E [B] (periodic 6-neighbour sum + the on-site term)."""
    nb = spins.copy()
    for ax in (1, 2, 3):
        nb += np.roll(spins, 1, axis=ax) + np.roll(spins, -1, axis=ax)
    return -(nb * spins).sum(axis=(1, 2, 3)) / 6.0


def _configs_with_downs(L, n_down, histogram_cutoff, rng):
    n = L ** 3
    if math.comb(n, n_down) > histogram_cutoff:
        base = np.ones(n)
        base[:n_down] = -1.0
        return np.stack([rng.permutation(base) for _ in range(histogram_cutoff)])
    out = []
    for downs in itertools.combinations(range(n), n_down):
        c = np.ones(n)
        c[list(downs)] = -1.0
        out.append(c)
    return np.stack(out)


def compositions(L):
    return list(range(L ** 3))


def generate(L, histogram_cutoff, n_down_list=None, spin_function=None, scale_spin=False, seed=0):
    """-> (node_features [B, L^3, 5], energies [B]) for the given down-spin counts."""
    rng = np.random.default_rng(seed)
    feats, energies = [], []
    pos = lattice_positions(L)
    for n_down in (n_down_list if n_down_list is not None else compositions(L)):
        c = _configs_with_downs(L, n_down, histogram_cutoff, rng)
        if scale_spin:
            c = c * rng.random(c.shape)
        s = spin_function(c) if spin_function is not None else c
        energies.append(ising_energy(s.reshape(-1, L, L, L)))
        f = np.empty(c.shape + (5,))
        f[..., 0] = c
        f[..., 1:4] = pos
        f[..., 4] = s
        feats.append(f)
    return np.concatenate(feats), np.concatenate(energies)


if __name__ == "__main__":
    f, e = generate(3, 10)
    print(f.shape, e.shape, e.min(), e.max())
