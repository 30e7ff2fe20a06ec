"""ZINC (subset) penalised logP regression (reference ``examples/zinc/{zinc.py, zinc.json}``:
SchNet + GPS multihead attention, pe_dim 6, graph head, MSE).

The reference loads PyG's ``ZINC(subset=True)`` (x = atom-type index, edge_attr = bond
type) and applies ``AddLaplacianEigenvectorPE(k=pe_dim)`` + ``rel_pe = |pe_i - pe_j|``
as a pre-transform.  The dataset cannot be downloaded here: molecules come from
synthetic SMILES (``examples/smiles_common.py``) read by the RDKit-free SMILES parser,
heavy atoms only like ZINC; x = ZINC-style atom-type index, edge_attr = bond-type
index.  ZINC has no coordinates while SchNet consumes positions: nodes get a
bond-graph spectral embedding (the 3 lowest non-trivial Laplacian eigenvectors,
scaled to ~1.5 A bonds) as a stand-in geometry (deviation, documented).

Usage: python examples/zinc/zinc.py [--num_samples 1000] [--num_epoch 2]
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import smiles_common as sc  # noqa: E402

from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.serialized import update_predicted_values  # noqa: E402
from hydragnn_amd.data.transforms import laplacian_pe, relative_pe  # noqa: E402
from hydragnn_amd.utils.smiles import parse_smiles  # noqa: E402

# ZINC atom dictionary (PyG ZINC): index of the atom type
ZINC_ATOMS = {"C": 0, "O": 1, "N": 2, "F": 3, "S": 5, "Cl": 6, "Br": 9, "I": 14, "P": 16}
_BOND = {1.0: 1, 1.5: 1, 2.0: 2, 3.0: 3}


def zinc_graph(smiles, y, pe_dim, seed):
    m = parse_smiles(smiles)
    n = len(m.atoms)
    src = [a for a, b, _ in m.bonds] + [b for a, b, _ in m.bonds]
    dst = [b for a, b, _ in m.bonds] + [a for a, b, _ in m.bonds]
    bt = [_BOND.get(o, 1) for _, _, o in m.bonds] * 2
    ei = torch.tensor([src, dst], dtype=torch.long).view(2, -1)
    emb = laplacian_pe(ei.numpy(), n, 3, sign_flip=False).numpy().astype(np.float64)
    if n > 1:
        L = np.linalg.norm(emb[ei[0].numpy()] - emb[ei[1].numpy()], axis=1).mean()
        emb = emb * (1.5 / max(L, 1e-6))
    pe = laplacian_pe(ei.numpy(), n, pe_dim, seed=seed)
    x = torch.tensor([ZINC_ATOMS[a.symbol] for a in m.atoms], dtype=torch.float32).view(-1, 1)
    g = Graph(x=x, pos=torch.from_numpy(emb).float(), edge_index=ei,
              edge_attr=torch.tensor(bt, dtype=torch.float32).view(-1, 1), y=torch.tensor([float(y)]).view(1),
              pe=pe, rel_pe=relative_pe(pe, ei))
    update_predicted_values(["graph"], [0], [1], [1], g)
    return g


def main(argv=None):
    args = sc.parser(__doc__.splitlines()[0], "zinc.json").parse_args(argv)
    config, workdir = sc.load(HERE, args)
    path = args.csv or sc.make_table(os.path.join(workdir, "zinc_logp.csv"), args.num_samples, "logp", seed=args.seed,
                                     elements=set(ZINC_ATOMS))
    smiles, ys = sc.read_table(path)
    pe_dim = config["NeuralNetwork"]["Architecture"]["pe_dim"]
    samples = [zinc_graph(s, y[0], pe_dim, args.seed + i) for i, (s, y) in enumerate(zip(smiles, ys))]
    return sc.train_and_test(config, samples, "zinc_test", seed=args.seed)


if __name__ == "__main__":
    main()
