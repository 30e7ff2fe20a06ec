"""Synthetic FCC Ni-Nb alloy configurations with an embedded-atom (EAM) potential
(stand-in for the reference's LAMMPS-generated ``FCC_Ni_Nb`` CFG dataset of
``examples/eam``; no download is possible here).

    E_i   = 1/2 sum_j phi_ab(r_ij) - sqrt(rho_i)          (second-moment / Finnis-Sinclair)
    rho_i = sum_j xi_b^2 exp(-2 q (r_ij / r0_ab - 1)) fc(r_ij)
    phi_ab(r) = A_ab exp(-p (r / r0_ab - 1)) fc(r)
    fc(r)     = (cos(pi r / rc) + 1) / 2,  r < rc

Ni uses the Cleri-Rosato parameters (p, q, xi); the Nb-like species has a larger
r0 and xi; A is set so that each pure FCC lattice is in equilibrium at its lattice
constant (3.52 / 4.20 A), cross terms are arithmetic / geometric means.

Periodic neighbours come from ``radius_graph_pbc``; forces are exact (-dE/dpos by
autograd, fp64); the bulk modulus B = V d2E/dV2 comes from isotropic strains.
Every configuration is written as an extended CFG file (aux columns c_peratom, fx,
fy, fz) plus a ``.bulk`` file ``natoms energy bulk_modulus`` (column 2 = B in GPa).
"""
import math
import os

import numpy as np
import torch

from hydragnn_amd.data.elements import atomic_mass
from hydragnn_amd.data.lsms import write_cfg
from hydragnn_amd.data.transforms import radius_graph_pbc

Z = (28, 41)  # Ni, Nb
R0 = torch.tensor([2.489, 2.970], dtype=torch.float64)
XI = torch.tensor([1.070, 1.900], dtype=torch.float64)
A = torch.tensor([0.0376, 0.0900], dtype=torch.float64)  # re-solved for equilibrium below
P_EXP, Q_EXP, RC = 16.999, 1.189, 5.2
EV_A3_TO_GPA = 160.21766


def fcc_supercell(n, a):
    base = np.array([[0, 0, 0], [0.5, 0.5, 0], [0.5, 0, 0.5], [0, 0.5, 0.5]])
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij"), -1).reshape(-1, 3)
    frac = ((g[:, None, :] + base[None]) / n).reshape(-1, 3)
    return frac, np.eye(3) * a * n


def eam_energy(pos, cell, species):
    """pos [N,3] (may require grad), cell [3,3], species [N] in {0,1} -> per-atom energy [N]."""
    ei, sh = radius_graph_pbc(pos.detach(), cell, [True] * 3, RC, max_num_neighbors=10 ** 6)
    src, dst = ei[0], ei[1]
    vec = pos[dst] - pos[src] + sh.to(pos.dtype)
    r = vec.norm(dim=-1)
    fc = 0.5 * (torch.cos(math.pi * r / RC) + 1)
    a, b = species[dst], species[src]
    r0ab = 0.5 * (R0[a] + R0[b])
    aab = torch.sqrt(A[a] * A[b])
    phi = aab * torch.exp(-P_EXP * (r / r0ab - 1)) * fc
    f = XI[b] ** 2 * torch.exp(-2 * Q_EXP * (r / r0ab - 1)) * fc
    n = pos.shape[0]
    rho = torch.zeros(n, dtype=pos.dtype).index_add(0, dst, f)
    pair = torch.zeros(n, dtype=pos.dtype).index_add(0, dst, phi)
    return 0.5 * pair - torch.sqrt(rho)


def _equilibrate():
    """A per species so that d E / d a = 0 for the pure FCC crystal at its lattice constant."""
    for s, a0 in ((0, 3.52), (1, 4.20)):
        frac, _ = fcc_supercell(2, 1.0)
        sp = torch.full((len(frac),), s)
        h = 1e-4
        d = []
        for a in (a0 - h, a0 + h):
            cell = torch.eye(3, dtype=torch.float64) * a * 2
            pos = torch.from_numpy(frac) @ cell
            A[s] = 1.0
            e_tot = float(eam_energy(pos, cell, sp).sum())
            A[s] = 0.0
            e_emb = float(eam_energy(pos, cell, sp).sum())
            d.append((e_tot - e_emb, e_emb))
        A[s] = -(d[1][1] - d[0][1]) / (d[1][0] - d[0][0])


def sample(rng, ncell=2):
    n = 4 * ncell ** 3
    n_nb = int(rng.choice(np.arange(0, n // 2 + 1, max(1, n // 8))))  # compositions in steps of 1/8
    x_nb = n_nb / n
    frac, cell = fcc_supercell(ncell, 3.52 + 0.68 * x_nb)  # Vegard's law between 3.52 and 4.20
    species = np.zeros(n, dtype=np.int64)
    species[rng.permutation(n)[:n_nb]] = 1
    pos = frac @ cell + rng.normal(0.0, 0.05, (n, 3))
    frac = pos @ np.linalg.inv(cell)
    sp = torch.from_numpy(species)
    cell_t = torch.from_numpy(cell)
    p = torch.from_numpy(pos).requires_grad_(True)
    e_atom = eam_energy(p, cell_t, sp)
    forces = -torch.autograd.grad(e_atom.sum(), p)[0]
    # bulk modulus from isotropic strain: V d2E/dV2 = (E'' - 3E') / (9V), u = ln(scale)
    h = 5e-3
    es = []
    for u in (-h, 0.0, h):
        s = math.exp(u)
        with torch.no_grad():
            es.append(float(eam_energy(torch.from_numpy(pos * s), cell_t * s, sp).sum()))
    d1 = (es[2] - es[0]) / (2 * h)
    d2 = (es[2] - 2 * es[1] + es[0]) / h ** 2
    vol = abs(np.linalg.det(cell))
    bulk = (d2 - 3 * d1) / (9 * vol) * EV_A3_TO_GPA
    return dict(numbers=np.array([Z[s] for s in species]), masses=np.array([atomic_mass(Z[s]) for s in species]),
                frac=frac, cell=cell, c_peratom=e_atom.detach().numpy(), forces=forces.numpy(),
                energy=float(e_atom.detach().sum()), bulk=bulk)


_equilibrate()


def write_dataset(path, num, seed=0, ncell=2):
    os.makedirs(path, exist_ok=True)
    rng = np.random.default_rng(seed)
    for i in range(num):
        s = sample(rng, ncell)
        base = os.path.join(path, f"NiNb_{i:05d}")
        aux = np.concatenate([s["c_peratom"][:, None], s["forces"]], 1)
        write_cfg(base + ".cfg", s["numbers"], s["masses"], s["frac"], s["cell"], aux,
                  ("c_peratom [eV]", "fx [eV/A]", "fy [eV/A]", "fz [eV/A]"), energy=s["energy"])
        with open(base + ".bulk", "w") as f:
            f.write(f"{len(s['numbers'])} {s['energy']:.10f} {s['bulk']:.10f}\n")
