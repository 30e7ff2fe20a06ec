"""Shared driver for the reference's atomistic energy / force examples whose datasets
cannot be downloaded here (reference ``examples/{qm7x, ani1_x, transition1x,
open_molecules_2025, mptrj, alexandria, open_materials_2024, open_catalyst_2022,
open_direct_air_capture_2023}/train.py``).

Each reference script reads its dataset's own format (HDF5, JSON, LMDB, ASE db),
builds ``Data(x=[Z, pos], pos, energy, forces, cell, pbc)`` samples, runs the radius
graph / PBC preprocessing and trains EGNN (hidden 50, 3 layers) on either the graph
energy (``*_energy.json``) or the node forces (``*_forces.json``), MAE loss.

Here every family is a ``Family`` record with the dataset's shape: element set, atom
count range, periodicity and cell construction.  Synthetic samples are generated with
that shape and a smooth Morse pair potential (element-dependent well depth / range),
energies and exact analytic forces in float64; periodic systems use the minimum-image
neighbour list of ``radius_graph_pbc``.  Node features are
``[Z, x, y, z, fx, fy, fz]`` (names ``atomic_number, cartesian_coordinates, forces``),
graph feature ``energy``; the configs select inputs and targets exactly as the
reference configs do.  The rest is the framework's normal path: serialized splits ->
``run_training`` (HBM-resident loader + captured step on a GPU) -> ``run_prediction``.

Usage (any family directory):  python examples/mptrj/train.py [--inputfile mptrj_forces.json]
"""
import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from common import base_parser, load_config, run_example, split  # noqa: E402

from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.synthetic import _mol_geometry  # noqa: E402
from hydragnn_amd.data.transforms import radius_graph_pbc  # noqa: E402


class Family:
    def __init__(self, name, elements, atoms, periodic, radius, max_neighbours, kind="molecule", pbc_axes=(1, 1, 1),
                 num_samples=600, notes=""):
        self.name, self.elements, self.atoms, self.periodic = name, tuple(elements), atoms, periodic
        self.radius, self.max_neighbours, self.kind = radius, max_neighbours, kind
        self.pbc_axes, self.num_samples, self.notes = tuple(bool(a) for a in pbc_axes), num_samples, notes


# dataset shapes (elements / atoms per structure / periodicity) of the reference datasets;
# radius / max_neighbours are the reference configs' values
_TM = (22, 23, 24, 25, 26, 27, 28, 29, 30)
FAMILIES = {
    "qm7x": Family("qm7x", (6, 7, 8, 16, 17), (4, 23), False, 5.0, 50,
                   notes="QM7-X: small organic molecules (C, N, O, S, Cl + H), non-equilibrium conformers"),
    "ani1_x": Family("ani1_x", (6, 7, 8), (4, 40), False, 10.0, 10,
                     notes="ANI-1x: C/H/N/O molecules, off-equilibrium sampling"),
    "transition1x": Family("transition1x", (6, 7, 8), (7, 23), False, 5.0, 50,
                           notes="Transition1x: reaction-path geometries of C/H/N/O molecules"),
    "open_molecules_2025": Family("open_molecules_2025", (5, 6, 7, 8, 9, 15, 16, 17, 35) + _TM, (4, 80), False,
                                  10.0, 10, notes="OMol25: molecules/complexes across the periodic table"),
    "mptrj": Family("mptrj", (3, 8, 11, 12, 13, 14, 15, 16) + _TM, (4, 48), True, 10.0, 10, kind="crystal",
                    notes="MPtrj: Materials Project relaxation trajectories (bulk crystals)"),
    "alexandria": Family("alexandria", (3, 5, 8, 11, 13, 14, 20, 31, 33, 38) + _TM, (2, 40), True, 10.0, 10,
                         kind="crystal", notes="Alexandria: DFT bulk crystals"),
    "open_materials_2024": Family("open_materials_2024", (8, 12, 13, 14, 20) + _TM, (4, 60), True, 10.0, 10,
                                  kind="crystal", notes="OMat24: rattled / AIMD bulk inorganic structures"),
    "open_catalyst_2022": Family("open_catalyst_2022", (1, 6, 7, 8) + _TM, (24, 120), True, 6.0, 50, kind="slab",
                                 pbc_axes=(1, 1, 0), notes="OC22: oxide slabs + adsorbates, periodic in x/y"),
    "open_direct_air_capture_2023": Family("open_direct_air_capture_2023", (1, 6, 7, 8, 29, 30), (60, 160), True,
                                           6.0, 50, kind="crystal",
                                           notes="ODAC23: metal-organic frameworks + CO2 / H2O"),
}


def _morse_params(z):
    z = np.asarray(z, dtype=np.float64)
    depth = 0.15 + 0.35 * np.abs(np.sin(0.37 * z))  # eV
    r0 = 1.1 + 0.9 * (z / (z + 10.0))  # A
    return depth, r0


def _energy_forces(z, pos, src, dst, vec):
    """Morse pair energy over the directed edge list (each pair twice) and its exact forces."""
    d, r0 = _morse_params(z)
    De = np.sqrt(d[src] * d[dst])
    re = 0.5 * (r0[src] + r0[dst])
    r = np.linalg.norm(vec, axis=1)
    ex = np.exp(-1.5 * (r - re))
    pair = De * ((1.0 - ex) ** 2 - 1.0)
    energy = 0.5 * float(pair.sum())
    dEdr = De * 2.0 * (1.0 - ex) * 1.5 * ex
    coef = (dEdr / np.maximum(r, 1e-9))[:, None]  # F_dst += -dE/dr * (r_dst - r_src)/r ... vec = p_dst - p_src
    forces = np.zeros_like(pos)
    np.add.at(forces, dst, -coef * vec)
    return energy, forces


def _periodic_structure(rng, fam):
    lo, hi = fam.atoms
    n_target = int(rng.integers(lo, hi + 1))
    a = rng.uniform(2.6, 3.6)
    reps = max(1, int(round(n_target ** (1.0 / 3.0))))
    nx = ny = reps
    nz = max(1, int(np.ceil(n_target / (nx * ny))))
    grid = np.stack(np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij"), -1).reshape(-1, 3)
    grid = grid[:n_target].astype(np.float64)
    pos = (grid + 0.08 * rng.normal(size=grid.shape)) * a
    cell = np.diag([nx * a, ny * a, nz * a])
    if fam.kind == "slab":
        cell[2, 2] += 12.0  # vacuum along z (not periodic)
    shear = rng.uniform(-0.1, 0.1) * a
    cell[1, 0] += shear
    z = rng.choice(fam.elements, size=len(pos))
    return z, pos, cell


def make_sample(rng, fam):
    if fam.periodic:
        z, pos, cell = _periodic_structure(rng, fam)
        ei, sh = radius_graph_pbc(torch.from_numpy(pos), torch.from_numpy(cell), list(fam.pbc_axes), fam.radius,
                                  max_num_neighbors=10 ** 6)
        src, dst = ei[0].numpy(), ei[1].numpy()
        vec = pos[dst] - pos[src] + sh.numpy().astype(np.float64)
    else:
        lo, hi = fam.atoms
        z, pos = _mol_geometry(rng, int(rng.integers(lo, hi + 1)), heavy=fam.elements)
        cell = None
        d = pos[:, None, :] - pos[None, :, :]
        r = np.linalg.norm(d, axis=-1)
        dst, src = np.nonzero((r < fam.radius) & (r > 0))
        vec = pos[dst] - pos[src]
    e, f = _energy_forces(z, pos, src, dst, vec)
    f32 = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32)  # noqa: E731
    x = torch.cat([f32(z).view(-1, 1), f32(pos), f32(f)], 1)
    g = Graph(x=x, pos=f32(pos), y=torch.tensor([e], dtype=torch.float32), energy=torch.tensor([e], dtype=torch.float32),
              forces=f32(f))
    if cell is not None:
        g.cell = f32(cell)
        g.pbc = torch.tensor(fam.pbc_axes, dtype=torch.bool)
    return g


def make_dataset(fam, num, seed=0):
    rng = np.random.default_rng(seed + 1009 * (sum(map(ord, fam.name)) % 97))
    return [make_sample(rng, fam) for _ in range(num)]


def family_config(fam, task):
    """The reference's ``<family>_{energy,forces}.json`` (EGNN h50 x3, MAE) for this family."""
    graph = task == "energy"
    cfg = {
        "Verbosity": {"level": 2},
        "Dataset": {
            "name": f"{fam.name}_{task}",
            "node_features": {"name": ["atomic_number", "cartesian_coordinates", "forces"], "dim": [1, 3, 3],
                              "column_index": [0, 1, 4]},
            "graph_features": {"name": ["energy"], "dim": [1], "column_index": [0]},
        },
        "NeuralNetwork": {
            "Architecture": {
                "mpnn_type": "EGNN", "equivariance": True, "radius": fam.radius, "max_neighbours": fam.max_neighbours,
                "periodic_boundary_conditions": fam.periodic, "num_gaussians": 50, "envelope_exponent": 5,
                "int_emb_size": 64, "basis_emb_size": 8, "out_emb_size": 128, "num_after_skip": 2,
                "num_before_skip": 1, "num_radial": 6, "num_spherical": 7, "num_filters": 126,
                "edge_features": ["length"], "hidden_dim": 50, "num_conv_layers": 3,
                "output_heads": ({"graph": {"num_sharedlayers": 2, "dim_sharedlayers": 50, "num_headlayers": 2,
                                            "dim_headlayers": [50, 25]}} if graph else
                                 {"node": {"num_headlayers": 2, "dim_headlayers": [200, 200], "type": "mlp"}}),
                "task_weights": [1.0],
            },
            "Variables_of_interest": {
                "input_node_features": [0],
                "output_names": ["energy" if graph else "forces"],
                "output_index": [0 if graph else 2],
                "output_dim": [1 if graph else 3],
                "type": ["graph" if graph else "node"],
            },
            "Training": {"num_epoch": 50, "EarlyStopping": True, "perc_train": 0.9, "loss_function_type": "mae",
                         "batch_size": 32, "continue": 0, "Optimizer": {"type": "AdamW", "learning_rate": 0.001}},
        },
        "Visualization": {"plot_init_solution": False, "plot_hist_solution": False, "create_plots": False},
    }
    return cfg


def write_configs(fam, directory):
    for task in ("energy", "forces"):
        with open(os.path.join(directory, f"{fam.name}_{task}.json"), "w") as f:
            json.dump(family_config(fam, task), f, indent=1)


def main(family, here, argv=None):
    fam = FAMILIES[family]
    args = base_parser(f"{family}: {fam.notes}", f"{fam.name}_energy.json").parse_args(argv)
    path = args.inputfile if os.path.isabs(args.inputfile) else os.path.join(here, args.inputfile)
    if not os.path.exists(path):
        write_configs(fam, here)
    config = load_config(here, args)
    samples = make_dataset(fam, args.num_samples or fam.num_samples, seed=args.seed)
    tr, va, te = split(samples, config["NeuralNetwork"]["Training"]["perc_train"], seed=args.seed)
    return run_example(copy.deepcopy(config), tr, va, te, args.workdir)


if __name__ == "__main__":
    name = sys.argv[1]
    main(name, os.path.join(HERE, name), sys.argv[2:])
