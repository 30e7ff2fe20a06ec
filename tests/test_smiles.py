"""RDKit-free SMILES reader (hydragnn_amd/utils/smiles.py) vs the reference's
RDKit-based featurisation (smiles_utils.py:35-127).  RDKit is not installed, so the
expected atom / hydrogen / bond counts below are textbook chemistry, not RDKit
output; hybridisation of conjugated amide/aniline N and O is parity unpinned."""
import pytest
import torch

from hydragnn_amd.utils.smiles import generate_graphdata_from_smilestr, get_node_attribute_name, parse_smiles

TYPES = {"H": 0, "C": 1, "N": 2, "O": 3, "F": 4, "S": 5, "Cl": 6}


@pytest.mark.parametrize("smi,n_heavy,n_h", [
    ("C", 1, 4), ("CCO", 3, 6), ("c1ccccc1", 6, 6), ("C1=CC=CC=C1", 6, 6), ("CC(=O)O", 4, 4),
    ("C#N", 2, 1), ("c1ccncc1", 6, 5), ("c1cc[nH]c1", 5, 5), ("O=C=O", 3, 0), ("CS(=O)(=O)C", 5, 6),
    ("ClC(Cl)Cl", 4, 1), ("[NH4+]", 1, 4), ("C[N+](C)(C)C", 5, 12), ("[O-]C(=O)C", 4, 3),
    ("C1CC1.O", 4, 8), ("FC(F)(F)c1ccccc1", 10, 5), ("C%12CCCCC%12", 6, 12),
])
def test_counts(smi, n_heavy, n_h):
    g = generate_graphdata_from_smilestr(smi, [0.5], TYPES)
    N = n_heavy + n_h
    assert g.x.shape == (N, len(TYPES) + 6)
    assert int(g.x[:, TYPES["H"]].sum()) == n_h
    # hydrogens come after the heavy atoms (RDKit AddHs order)
    assert bool((g.x[n_heavy:, TYPES["H"]] == 1).all())
    # every bond twice, sorted by src * N + dst
    key = g.edge_index[0] * N + g.edge_index[1]
    assert bool((key[1:] > key[:-1]).all())
    # Hprop column = number of H neighbours
    hprop = torch.zeros(N).index_add_(0, g.edge_index[1], g.x[g.edge_index[0], TYPES["H"]])
    assert torch.equal(hprop, g.x[:, -1])


def test_benzene_features():
    g = generate_graphdata_from_smilestr("c1ccccc1", [1.0], TYPES)
    c = g.x[:6]
    assert torch.equal(c[:, len(TYPES)], torch.full((6,), 6.0))  # atomic number
    assert bool((c[:, len(TYPES) + 1] == 1).all())  # aromatic
    assert bool((c[:, len(TYPES) + 3] == 1).all())  # sp2
    # 6 aromatic C-C bonds (x2 directions) + 6 single C-H (x2)
    assert int(g.edge_attr[:, 3].sum()) == 12 and int(g.edge_attr[:, 0].sum()) == 12
    names, dims = get_node_attribute_name(TYPES)
    assert len(names) == g.x.shape[1] and dims == [1] * len(names)


def test_hybridisation_and_bonds():
    g = generate_graphdata_from_smilestr("C#CC=CC", [0.0], TYPES)
    sp, sp2, sp3 = (g.x[:5, len(TYPES) + k] for k in (2, 3, 4))
    assert sp.tolist() == [1, 1, 0, 0, 0]
    assert sp2.tolist() == [0, 0, 1, 1, 0]
    assert sp3.tolist() == [0, 0, 0, 0, 1]
    assert int(g.edge_attr[:, 2].sum()) == 2 and int(g.edge_attr[:, 1].sum()) == 2


def test_ring_bond_order_and_errors():
    m = parse_smiles("C=1CCCCC1")
    assert sorted(o for _, _, o in m.bonds).count(2.0) == 1
    with pytest.raises(ValueError):
        parse_smiles("C1CC")
    m = parse_smiles("[13CH3][2H]")
    assert m.atoms[0].isotope == 13 and m.num_hs[0] == 3
