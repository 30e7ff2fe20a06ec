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
        ei = radius_graph(pos, radius, max_num_neighbors=max_neighbours)
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
