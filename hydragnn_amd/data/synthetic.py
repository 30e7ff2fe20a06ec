"""Synthetic datasets (no network access: every benchmark / test runs on generated data).

* ``oc20_like``: atomistic graphs shaped like OC20-S2EF adsorbate+slab systems
  (≈20-126 atoms, mean ≈73; random positions at solid density; atomic numbers
  1-83), radius graph with ``max_neighbours`` cap, normalised edge lengths,
  Laplacian eigenvector PE (``pe_dim``) and ``rel_pe``; graph energy target
  (+ per-atom forces).  Used by ``bench.py`` for the headline config
  (OC20 PNAPlus + GPS).
* ``deterministic_graph_data`` lives in ``data/lsms.py`` (CI dataset of the
  reference test-suite).
"""
import numpy as np
import torch

from .graph import Graph
from .transforms import laplacian_pe, radius_graph, relative_pe


def _energy(z, pos):
    # smooth, size-extensive pseudo energy: per-species reference + pair term
    e0 = -0.1 * z.sum()
    d = torch.cdist(pos, pos) + torch.eye(pos.shape[0], dtype=pos.dtype) * 1e6
    pair = (1.0 / d ** 6 - 1.0 / d ** 3).sum() * 0.5
    return float(e0 + pair)


def oc20_like(num_graphs, seed=0, min_atoms=20, max_atoms=126, radius=10.0, max_neighbours=10, pe_dim=16,
              density=0.08, with_forces=False):
    rng = np.random.default_rng(seed)
    out = []
    for g in range(num_graphs):
        n = int(rng.integers(min_atoms, max_atoms + 1))
        L = (n / density) ** (1.0 / 3.0)
        pos = torch.from_numpy(rng.uniform(0.0, L, size=(n, 3))).to(torch.float32)
        z = torch.from_numpy(rng.integers(1, 84, size=(n,))).to(torch.float32)
        # OC20's AtomsToGraphs keeps the nearest neighbours (radius_graph_pbc in fairchem)
        ei = radius_graph(pos, radius, max_num_neighbors=max_neighbours, cap_policy="nearest")
        vec = pos[ei[1]] - pos[ei[0]]
        length = torch.linalg.norm(vec, dim=-1, keepdim=True)
        edge_attr = length / radius
        x = torch.cat([z.view(-1, 1), pos], dim=1)
        pe = laplacian_pe(ei, n, pe_dim, seed=int(rng.integers(1 << 30)))
        energy = _energy(z.double(), pos.double())
        y = torch.tensor([[energy / n]], dtype=torch.float32)
        s = Graph(x=x, pos=pos, edge_index=ei, edge_attr=edge_attr, pe=pe, rel_pe=relative_pe(pe, ei), y=y,
                  y_loc=torch.tensor([[0, 1]], dtype=torch.int64), energy=y.view(1))
        if with_forces:
            s.forces = torch.from_numpy(rng.normal(size=(n, 3))).to(torch.float32)
        s.sort_edges_by_dst()
        out.append(s)
    return out


def degree_histogram(samples, max_degree=None):
    degs = [torch.bincount(s.edge_index[1], minlength=s.num_nodes) for s in samples]
    d = torch.cat(degs)
    md = int(d.max()) if max_degree is None else max_degree
    return torch.bincount(d.clamp(max=md), minlength=md + 1)


# ---------------------------------------------------------------------------- molecules
_REF_E = {1: -0.50, 6: -37.8, 7: -54.6, 8: -75.0, 9: -99.7}  # per-element reference energies (Hartree-like)


def _mol_energy(z, pos):
    """Smooth molecular pseudo-potential: element references + Morse bonds (r0 by pair)."""
    zz = torch.as_tensor(z, dtype=pos.dtype)
    e0 = sum(_REF_E.get(int(a), -1.0) for a in z)
    d = torch.cdist(pos, pos) + torch.eye(pos.shape[0], dtype=pos.dtype) * 10.0
    r0 = 0.55 + 0.09 * (zz.view(-1, 1) + zz.view(1, -1)) ** 0.5
    morse = (1.0 - torch.exp(-1.5 * (d - r0))) ** 2 - 1.0
    w = torch.exp(-((d / 3.0) ** 4))  # smooth cutoff ~3 A
    return e0 + 0.5 * (0.1 * morse * w).sum()


def _mol_geometry(rng, n, heavy=(6, 7, 8, 9), hfrac=0.45):
    """Random chain/branch molecule: heavy atoms on a self-avoiding walk (1.45 A), H caps (1.09 A)."""
    nh = max(1, int(round(n * hfrac)))
    nheavy = max(1, n - nh)
    pos = [np.zeros(3)]
    while len(pos) < nheavy:
        base = pos[int(rng.integers(max(0, len(pos) - 3), len(pos)))]
        for _ in range(20):
            v = rng.normal(size=3)
            p = base + 1.45 * v / np.linalg.norm(v)
            if min(np.linalg.norm(np.asarray(pos) - p, axis=1)) > 1.2:
                break
        pos.append(p)
    z = list(rng.choice(heavy, size=nheavy, p=[0.7, 0.12, 0.15, 0.03][:len(heavy)] if len(heavy) == 4 else None))
    for k in range(n - nheavy):
        base = pos[k % nheavy]
        for _ in range(20):
            v = rng.normal(size=3)
            p = base + 1.09 * v / np.linalg.norm(v)
            if min(np.linalg.norm(np.asarray(pos) - p, axis=1)) > 0.9:
                break
        pos.append(p)
        z.append(1)
    return np.asarray(z, dtype=np.int64), np.asarray(pos, dtype=np.float64)


def molecules_like(num_graphs, seed=0, min_atoms=5, max_atoms=29, with_forces=False):
    """QM9-shaped molecules (H/C/N/O/F, 5-29 atoms) with a smooth pseudo-energy
    (element references + Morse bonds) and, optionally, its exact forces.
    Fields: x=[Z], pos, y=[atomization energy per atom], energy=[atomization energy], forces."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(num_graphs):
        n = int(rng.integers(min_atoms, max_atoms + 1))
        z, p = _mol_geometry(rng, n)
        out.append(_mol_sample(z, p, with_forces))
    return out


def _mol_sample(z, p, with_forces):
    pos = torch.tensor(p, dtype=torch.float64, requires_grad=with_forces)
    e = _mol_energy(z, pos)
    ev = float(e.detach())
    eref = sum(_REF_E.get(int(a), -1.0) for a in z)
    # y: atomization-like energy per atom (total minus element references); energy: total
    s = Graph(x=torch.as_tensor(z, dtype=torch.float32).view(-1, 1), pos=pos.detach().to(torch.float32),
              y=torch.tensor([(ev - eref) / len(z)], dtype=torch.float32),
              energy=torch.tensor([ev - eref], dtype=torch.float32))
    if with_forces:
        (g,) = torch.autograd.grad(e, pos)
        s.forces = (-g).to(torch.float32)
    return s


def md_trajectory(num_frames, seed=0, num_atoms=21, amplitude=0.08):
    """MD17-shaped data: thermal-like perturbations of ONE molecule (fixed atoms), with
    energies and exact forces of the same pseudo-potential."""
    rng = np.random.default_rng(seed)
    z, p0 = _mol_geometry(rng, num_atoms)
    return [_mol_sample(z, p0 + amplitude * rng.normal(size=p0.shape), True) for _ in range(num_frames)]
