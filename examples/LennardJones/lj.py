"""Lennard-Jones crystals: energy + forces by automatic differentiation
(reference ``examples/LennardJones/{LennardJones.py, LJ_data.py, LJ.json}``).

Synthetic data: simple-cubic supercells (3-4 cells per axis, a = 3.8 A) with
up to 10 % random displacements, periodic boundaries, LJ(eps=1, sigma=3.4)
pair potential truncated at the graph radius.  Per-atom potentials, total
energy and analytic forces are computed in float64.  The model predicts a
per-node energy; ``Training.compute_grad_energy`` trains on the summed graph
energy and on forces = -dE/dpos (double backward through the conv stack,
reference ``Base.py:582-636``).

Usage: python examples/LennardJones/lj.py [--mpnn_type PAINN] [--num_samples 300] [--num_epoch 25]
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import base_parser, load_config, run_example, split  # noqa: E402

from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.transforms import radius_graph_pbc  # noqa: E402

LATTICE = 3.8
EPS, SIGMA = 1.0, 3.4


def lj_configuration(rng, radius, cells=(3, 5), disp=0.1):
    n = [int(rng.integers(cells[0], cells[1])) for _ in range(3)]
    grid = np.stack(np.meshgrid(*[np.arange(k) for k in n], indexing="ij"), -1).reshape(-1, 3).astype(np.float64)
    pos = (grid + disp * (rng.random(grid.shape) - 0.5)) * LATTICE
    cell = np.diag(np.asarray(n, dtype=np.float64) * LATTICE)
    ei, sh = radius_graph_pbc(torch.from_numpy(pos), torch.from_numpy(cell), [True] * 3, radius,
                              max_num_neighbors=10 ** 6)
    src, dst = ei[0].numpy(), ei[1].numpy()
    vec = pos[dst] - pos[src] + sh.numpy().astype(np.float64)  # j -> i
    r = np.linalg.norm(vec, axis=1)
    sr6 = (SIGMA / r) ** 6
    pair = 4.0 * EPS * (sr6 * sr6 - sr6)  # each unordered pair appears twice (i<-j and j<-i)
    atom_e = np.zeros(len(pos))
    np.add.at(atom_e, dst, 0.5 * pair)
    # F_i = -dE/dr_i = sum_j 24 eps (2 sr12 - sr6) / r^2 * (r_i - r_j)
    coef = 24.0 * EPS * (2.0 * sr6 * sr6 - sr6) / (r * r)
    forces = np.zeros_like(pos)
    np.add.at(forces, dst, coef[:, None] * vec)
    return pos, cell, atom_e, forces


def make_dataset(num, radius, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(num):
        pos, cell, atom_e, forces = lj_configuration(rng, radius)
        n = len(pos)
        f32 = lambda a: torch.as_tensor(a, dtype=torch.float32)  # noqa: E731
        x = torch.cat([torch.ones(n, 1), f32(atom_e).view(-1, 1), f32(forces)], 1)
        e = float(atom_e.sum())
        out.append(Graph(x=x, pos=f32(pos), cell=f32(cell), pbc=torch.ones(3, dtype=torch.bool),
                         y=torch.tensor([e], dtype=torch.float32), energy=torch.tensor([e], dtype=torch.float32),
                         forces=f32(forces)))
    return out


def main(argv=None):
    args = base_parser(__doc__.splitlines()[0], "LJ.json").parse_args(argv)
    config = load_config(HERE, args)
    arch = config["NeuralNetwork"]["Architecture"]
    samples = make_dataset(args.num_samples or 300, arch["radius"], seed=args.seed)
    tr, va, te = split(samples, config["NeuralNetwork"]["Training"]["perc_train"], seed=args.seed)
    return run_example(config, tr, va, te, args.workdir)


if __name__ == "__main__":
    main()
