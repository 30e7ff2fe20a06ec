"""SMILES -> molecular graph without RDKit (reference
``utils/descriptors_and_embeddings/smiles_utils.py:18-127``, which calls RDKit's
``MolFromSmiles`` + ``AddHs``).

RDKit is not available on this image, so this module carries its own OpenSMILES
reader covering what the reference's datasets (ogb-pcqm4m, ZINC, CSCE, DFTB UV
spectra) use:

* organic-subset atoms ``B C N O P S F Cl Br I`` and aromatic ``b c n o p s``,
  bracket atoms ``[13CH3+]``, ``[nH]``, ``[C@@H]``, ``[Na+]``, ``[O-]``, ``[2H]`` ...
* bonds ``- = # $ :`` and the stereo marks ``/ \\`` (read as single),
  branches ``( )``, ring closures ``1-9`` / ``%nn`` (with bond orders on either
  side), disconnected components ``.``;
* implicit hydrogens from the default valences of the organic subset
  (lowest allowed valence >= explicit bond-order sum, aromatic atoms counting
  one extra ring electron), then explicit H atoms appended after the heavy atoms
  in heavy-atom order, which is RDKit ``AddHs``'s atom order.

Features follow the reference exactly: ``x = [one_hot(type, len(types)),
atomic_number, aromatic, sp, sp2, sp3, num_hs]`` and a 4-way one-hot bond type
(single, double, triple, aromatic) with both directions of every bond, edges
sorted by ``src * N + dst``.  Hybridisation is derived from the bonding pattern
(aromatic or one double bond -> sp2; a triple bond or two double bonds -> sp;
otherwise sp3 for atoms with >= 2 neighbours or lone pairs; H and ions with no
bonds -> none).  RDKit additionally relabels conjugated amide / aniline N and
O as sp2; that refinement is not modelled, so those features are "parity
unpinned" against RDKit (documented in ``tests/test_smiles.py``).
"""
import torch
import torch.nn.functional as F

from ..data.graph import Graph

_ORGANIC = {"B": (3,), "C": (4,), "N": (3, 5), "O": (2,), "P": (3, 5), "S": (2, 4, 6), "F": (1,), "Cl": (1,),
            "Br": (1,), "I": (1,)}
_AROMATIC = {"b": "B", "c": "C", "n": "N", "o": "O", "p": "P", "s": "S", "se": "Se", "as": "As"}
_Z = {"H": 1, "He": 2, "Li": 3, "Be": 4, "B": 5, "C": 6, "N": 7, "O": 8, "F": 9, "Ne": 10, "Na": 11, "Mg": 12,
      "Al": 13, "Si": 14, "P": 15, "S": 16, "Cl": 17, "Ar": 18, "K": 19, "Ca": 20, "Fe": 26, "Co": 27, "Ni": 28,
      "Cu": 29, "Zn": 30, "Ga": 31, "Ge": 32, "As": 33, "Se": 34, "Br": 35, "Kr": 36, "Rb": 37, "Sr": 38,
      "Ag": 47, "Sn": 50, "Sb": 51, "Te": 52, "I": 53, "Xe": 54, "Cs": 55, "Ba": 56, "Pt": 78, "Au": 79,
      "Hg": 80, "Pb": 82, "Bi": 83}
BOND_TYPES = {"single": 0, "double": 1, "triple": 2, "aromatic": 3}
_BOND_CHARS = {"-": 1.0, "=": 2.0, "#": 3.0, "$": 4.0, ":": 1.5, "/": 1.0, "\\": 1.0}


class Atom:
    __slots__ = ("symbol", "aromatic", "charge", "hcount", "isotope", "bracket", "idx")

    def __init__(self, symbol, aromatic=False, charge=0, hcount=None, isotope=None, bracket=False):
        self.symbol, self.aromatic, self.charge = symbol, aromatic, charge
        self.hcount, self.isotope, self.bracket = hcount, isotope, bracket
        self.idx = -1


class Molecule:
    """Heavy-atom graph as parsed (``atoms``, ``bonds`` = [(i, j, order)], order 1.5 =
    aromatic) plus per-atom implicit-H counts."""

    def __init__(self, atoms, bonds):
        self.atoms = atoms
        self.bonds = bonds
        self.num_hs = [self._hydrogens(i) for i in range(len(atoms))]

    def _bond_orders(self, i):
        return [o for (a, b, o) in self.bonds if a == i or b == i]

    def _hydrogens(self, i):
        at = self.atoms[i]
        if at.bracket:
            return at.hcount or 0
        if at.symbol not in _ORGANIC:
            return 0
        orders = self._bond_orders(i)
        arom = sum(1 for o in orders if o == 1.5)
        used = sum(o for o in orders if o != 1.5) + arom
        if at.aromatic:
            used += 1  # one electron into the aromatic pi system
        for v in _ORGANIC[at.symbol]:
            if v >= used:
                return int(round(v - used))
        return 0


def _lex(s):
    """Tokenise a SMILES string."""
    i, n = 0, len(s)
    while i < n:
        c = s[i]
        if c == "[":
            j = s.index("]", i)
            yield ("bracket", s[i + 1:j])
            i = j + 1
        elif c == "%":
            yield ("ring", int(s[i + 1:i + 3]))
            i += 3
        elif c.isdigit():
            yield ("ring", int(c))
            i += 1
        elif c in "()":
            yield (c, c)
            i += 1
        elif c in _BOND_CHARS:
            yield ("bond", c)
            i += 1
        elif c == ".":
            yield ("dot", c)
            i += 1
        elif s.startswith(("Cl", "Br"), i):
            yield ("atom", s[i:i + 2])
            i += 2
        elif s.startswith(("se", "as"), i):
            yield ("atom", s[i:i + 2])
            i += 2
        elif c in "BCNOPSFI" or c in "bcnops":
            yield ("atom", c)
            i += 1
        elif c == "*":
            yield ("atom", "*")
            i += 1
        else:
            raise ValueError(f"unsupported SMILES character {c!r} at {i} in {s!r}")


def _parse_bracket(txt):
    i = 0
    iso = ""
    while i < len(txt) and txt[i].isdigit():
        iso += txt[i]
        i += 1
    if txt[i:i + 2].lower() in ("se", "as") and txt[i].islower():
        sym, aro = txt[i:i + 2], True
        i += 2
    elif txt[i].islower():
        sym, aro = txt[i], True
        i += 1
    else:
        sym = txt[i]
        i += 1
        if i < len(txt) and txt[i].islower():
            sym += txt[i]
            i += 1
        aro = False
    while i < len(txt) and txt[i] == "@":
        i += 1
    h = 0
    if i < len(txt) and txt[i] == "H":
        i += 1
        h = 1
        num = ""
        while i < len(txt) and txt[i].isdigit():
            num += txt[i]
            i += 1
        if num:
            h = int(num)
    charge = 0
    while i < len(txt) and txt[i] in "+-":
        sgn = 1 if txt[i] == "+" else -1
        i += 1
        num = ""
        while i < len(txt) and txt[i].isdigit():
            num += txt[i]
            i += 1
        charge += sgn * (int(num) if num else 1)
    symbol = _AROMATIC.get(sym, sym) if aro else sym
    return Atom(symbol, aro, charge, h, int(iso) if iso else None, bracket=True)


def parse_smiles(smiles):
    """Parse a SMILES string into a :class:`Molecule` (heavy atoms + bracket H)."""
    atoms, bonds = [], []
    stack, prev, pending = [], None, None
    rings = {}
    for kind, val in _lex(smiles.strip()):
        if kind in ("atom", "bracket"):
            if kind == "atom":
                aro = val[0].islower() and val != "*"
                at = Atom(_AROMATIC.get(val, val) if aro else val, aro)
            else:
                at = _parse_bracket(val)
            at.idx = len(atoms)
            atoms.append(at)
            if prev is not None:
                order = pending if pending is not None else (
                    1.5 if (atoms[prev].aromatic and at.aromatic) else 1.0)
                bonds.append((prev, at.idx, order))
            prev, pending = at.idx, None
        elif kind == "bond":
            pending = _BOND_CHARS[val]
        elif kind == "(":
            stack.append(prev)
        elif kind == ")":
            prev = stack.pop()
        elif kind == "dot":
            prev, pending = None, None
        elif kind == "ring":
            if val in rings:
                j, o_open = rings.pop(val)
                order = pending if pending is not None else o_open
                if order is None:
                    order = 1.5 if (atoms[j].aromatic and atoms[prev].aromatic) else 1.0
                bonds.append((j, prev, order))
            else:
                rings[val] = (prev, pending)
            pending = None
    if rings:
        raise ValueError(f"unclosed ring bond(s) {sorted(rings)} in {smiles!r}")
    return Molecule(atoms, bonds)


def _hybridisation(mol, i, heavy_nbrs):
    """(sp, sp2, sp3) flags from the bonding pattern (see module docstring)."""
    at = mol.atoms[i]
    orders = mol._bond_orders(i)
    if at.aromatic or any(o == 1.5 for o in orders):
        return 0, 1, 0
    ndouble = sum(1 for o in orders if o == 2.0)
    if any(o == 3.0 for o in orders) or ndouble >= 2:
        return 1, 0, 0
    if ndouble == 1:
        return 0, 1, 0
    degree = heavy_nbrs + mol.num_hs[i]
    if degree == 0 and at.charge != 0:
        return 0, 0, 0
    return 0, 0, 1 if degree >= 1 else 0


def get_node_attribute_name(types):
    """Feature names / dims of :func:`generate_graphdata_from_smilestr` (ref :18-32)."""
    names = ["atom" + k for k in types] + ["atomicnumber", "IsAromatic", "HSP", "HSP2", "HSP3", "Hprop"]
    return names, [1] * len(names)


def generate_graphdata_from_smilestr(smilestr, ytarget, types, var_config=None, atomicdescriptors=None):
    """SMILES -> :class:`Graph` with explicit hydrogens (ref :35-127).

    ``types``: element symbol -> type index (must contain every element present,
    including "H").  ``atomicdescriptors``: optional [N_with_H, k] tensor appended
    to ``x``."""
    mol = parse_smiles(smilestr)
    nh = len(mol.atoms)
    symbols = [a.symbol for a in mol.atoms]
    aromatic = [1 if a.aromatic else 0 for a in mol.atoms]
    edges = [(a, b, o) for (a, b, o) in mol.bonds]
    # explicit hydrogens after the heavy atoms, in heavy-atom order (RDKit AddHs order)
    for i in range(nh):
        for _ in range(mol.num_hs[i]):
            edges.append((i, len(symbols), 1.0))
            symbols.append("H")
            aromatic.append(0)
    N = len(symbols)
    heavy_deg = [0] * nh
    for a, b, _ in mol.bonds:
        heavy_deg[a] += 1
        heavy_deg[b] += 1
    hyb = [_hybridisation(mol, i, heavy_deg[i]) for i in range(nh)] + [(0, 0, 0)] * (N - nh)
    z = [_Z.get(s, 0) for s in symbols]

    def btype(o):
        return {1.0: 0, 2.0: 1, 3.0: 2, 1.5: 3}.get(o, 0)

    row, col, et = [], [], []
    for a, b, o in edges:
        row += [a, b]
        col += [b, a]
        et += [btype(o)] * 2
    ei = torch.tensor([row, col], dtype=torch.long).view(2, -1)
    etype = torch.tensor(et, dtype=torch.long)
    perm = (ei[0] * N + ei[1]).argsort()
    ei, etype = ei[:, perm], etype[perm]
    edge_attr = F.one_hot(etype, num_classes=len(BOND_TYPES)).float()
    zt = torch.tensor(z, dtype=torch.long)
    num_hs = torch.zeros(N).index_add_(0, ei[1], (zt[ei[0]] == 1).float()) if ei.numel() else torch.zeros(N)
    x1 = F.one_hot(torch.tensor([types[s] for s in symbols]), num_classes=len(types)).float()
    x2 = torch.tensor([z, aromatic, [h[0] for h in hyb], [h[1] for h in hyb], [h[2] for h in hyb]],
                      dtype=torch.float).t()
    x = torch.cat([x1, x2, num_hs.view(-1, 1)], dim=-1)
    if atomicdescriptors is not None:
        assert atomicdescriptors.shape[0] == N, "atomic descriptors need one row per atom (hydrogens included)"
        x = torch.cat([x, atomicdescriptors.float()], dim=-1)
    y = ytarget if torch.is_tensor(ytarget) else torch.tensor(ytarget, dtype=torch.float).view(-1, 1)
    data = Graph(x=x, edge_index=ei, edge_attr=edge_attr, y=y)
    if var_config is not None:
        from ..data.serialized import update_predicted_values

        update_predicted_values(var_config["type"], var_config["output_index"], var_config["graph_feature_dims"],
                                var_config["input_node_feature_dims"], data)
    return data
