"""Raw-format readers (LSMS text, CFG, XYZ) and the reference's deterministic
synthetic CI dataset.

* ``deterministic_graph_data`` re-implements the generator semantics of the
  reference test-suite (``tests/deterministic_graph_data.py:20-173``): random
  BCC supercells (2*x*y*z atoms, x,y in [1,3), z in [1,2)), node feature = a
  random type, node outputs = kNN-smoothed feature X, X^2 + feature, X^3, graph
  outputs = sum of the three and sum of X; written as LSMS-format text files.
* ``read_lsms`` parses the LSMS text format (first line: graph features; one
  line per atom: feature, index, x, y, z, nodal columns) and applies the
  charge-density update (column 1 -= column 0), as
  ``preprocess/lsms_raw_dataset_loader.py:34-106``.
* ``RawDataLoader`` walks raw directories, scales ``*_scaled_num_nodes``
  features, min-max normalises node/graph features across all splits
  (optionally all ranks) and writes the serialized split files
  (``preprocess/raw_dataset_loader.py:26-277``).
"""
import os

import numpy as np
import torch

from .graph import Graph
from .serialized import write_serialized


def _knn_smooth(positions, values, k):
    from sklearn.neighbors import KNeighborsRegressor

    knn = KNeighborsRegressor(k)
    knn.fit(positions, values)
    return torch.tensor(knn.predict(positions), dtype=torch.float32)


def deterministic_graph_data(path, number_configurations=500, configuration_start=0, unit_cell_x_range=(1, 3),
                             unit_cell_y_range=(1, 3), unit_cell_z_range=(1, 2), number_types=3, types=None,
                             number_neighbors=2, linear_only=False, seed=None):
    os.makedirs(path, exist_ok=True)
    if types is None:
        types = range(number_types)
    types = list(types)
    g = torch.Generator()
    if seed is not None:
        g.manual_seed(seed)
    else:
        g.manual_seed(torch.initial_seed())
    ux = torch.randint(unit_cell_x_range[0], unit_cell_x_range[1], (number_configurations,), generator=g)
    uy = torch.randint(unit_cell_y_range[0], unit_cell_y_range[1], (number_configurations,), generator=g)
    uz = torch.randint(unit_cell_z_range[0], unit_cell_z_range[1], (number_configurations,), generator=g)
    for c in range(number_configurations):
        _create_configuration(path, c, configuration_start, int(ux[c]), int(uy[c]), int(uz[c]), types,
                              number_neighbors, linear_only, g)


def _create_configuration(path, configuration, start, uc_x, uc_y, uc_z, types, k, linear_only, g):
    n = 2 * uc_x * uc_y * uc_z
    pos = []
    for x in range(uc_x):
        for y in range(uc_y):
            for z in range(uc_z):
                pos.append([x, y, z])
                pos.append([x + 0.5, y + 0.5, z + 0.5])
    positions = torch.tensor(pos, dtype=torch.float32)
    ids = torch.arange(n, dtype=torch.int64).view(-1, 1)
    feat = torch.randint(min(types), max(types) + 1, (n, 1), generator=g)
    if linear_only:
        ox = feat.float()
    else:
        ox = _knn_smooth(positions.numpy(), feat.numpy(), k)
    ox2 = ox ** 2 + feat
    ox3 = ox ** 3
    table = torch.cat((feat.float(), ids.float(), positions, ox, ox2, ox3), 1).numpy()
    if linear_only:
        total = float(ox.sum())
        txt = np.array2string(np.float32(total))
    else:
        total_lin = float(ox.sum())
        total = float(ox.sum() + ox2.sum() + ox3.sum())
        txt = np.array2string(np.float32(total)) + "\t" + np.array2string(np.float32(total_lin))
    for i in range(n):
        row = np.array2string(table[i], precision=2, separator="\t", suppress_small=True)
        txt += "\n" + row.lstrip("[").rstrip("]")
    with open(os.path.join(path, f"output{configuration + start}.txt"), "w") as f:
        f.write(txt)


def read_lsms(filepath, node_feature_dim, node_feature_col, graph_feature_dim, graph_feature_col):
    with open(filepath, "r", encoding="utf-8") as f:
        lines = f.readlines()
    gl = lines[0].split(None, 2)
    gf = []
    for item in range(len(graph_feature_dim)):
        for ic in range(graph_feature_dim[item]):
            gf.append(float(gl[graph_feature_col[item] + ic].strip()))
    pos, xs = [], []
    for line in lines[1:]:
        if not line.strip():
            continue
        nf = line.split(None, 11)
        pos.append([float(nf[2]), float(nf[3]), float(nf[4])])
        row = []
        for item in range(len(node_feature_dim)):
            for ic in range(node_feature_dim[item]):
                row.append(float(nf[node_feature_col[item] + ic].strip()))
        xs.append(row)
    d = Graph(y=torch.tensor(gf, dtype=torch.float32), pos=torch.tensor(pos, dtype=torch.float32),
              x=torch.tensor(xs, dtype=torch.float32))
    # charge density update for LSMS: x[:, 1] -= x[:, 0]
    if d.x.shape[1] > 1:
        d.x[:, 1] = d.x[:, 1] - d.x[:, 0]
    return d


def read_cfg(filepath, node_feature_dim, node_feature_col, graph_feature_dim, graph_feature_col):
    """AtomEye extended-CFG reader (reference ``utils/datasets/cfgdataset.py:31-89`` via
    ``ase.io.cfg.read_cfg``; ase is not available here, the format is parsed directly).

    Layout: ``Number of particles = N``; ``A = <scale> Angstrom``; ``H0(i,j) = v``;
    ``.NO_VELOCITY.``; ``entry_count``; ``auxiliary[k] = name``; then per species a mass
    line, a symbol line and that species' rows ``s1 s2 s3 aux...`` (reduced coordinates).
    Returns x = [Z, mass, aux columns...] (the reference's node matrix ``numbers, masses,
    c_peratom, fx, fy, fz``), cartesian ``pos = s @ (A * H0)``, the cell, and ``y`` from
    the sibling ``.bulk`` file's graph columns when it exists (else the ``# energy``
    comment, else empty)."""
    from .elements import atomic_number

    if not filepath.endswith(".cfg"):
        return None  # companion files (.bulk) and anything else in the directory
    with open(filepath) as f:
        lines = [l.strip() for l in f if l.strip()]
    n = None
    scale = 1.0
    H = np.zeros((3, 3))
    n_aux = 0
    energy = None
    mass, z = 0.0, 0
    rows = []
    for l in lines:
        key = l.split("=")[0].strip()
        if key.startswith("Number of particles"):
            n = int(l.split("=")[1].split()[0])
        elif key == "A":
            scale = float(l.split("=")[1].split()[0])
        elif key.startswith("H0("):
            i, j = int(key[3]) - 1, int(key[5]) - 1
            H[i, j] = float(l.split("=")[1].split()[0])
        elif key.startswith("auxiliary["):
            n_aux += 1
        elif key in ("entry_count", "R", "eta") or key.startswith((".", "Transform(")):
            continue
        elif l.startswith("#"):
            if "energy" in l.lower() and "=" in l:
                energy = float(l.split("=")[-1])
        else:
            tok = l.split()
            if len(tok) == 1:
                try:
                    mass = float(tok[0])
                except ValueError:
                    z = atomic_number(tok[0])
                continue
            if len(tok) >= 3 + n_aux:
                rows.append([float(z), mass] + [float(v) for v in tok[:3 + n_aux]])
    assert n is not None and len(rows) == n, f"{filepath}: expected {n} atoms, parsed {len(rows)}"
    arr = np.asarray(rows, dtype=np.float64)
    cell = H * scale
    pos = arr[:, 2:5] @ cell
    x = np.concatenate([arr[:, :2], arr[:, 5:]], 1)
    bulk = os.path.splitext(filepath)[0] + ".bulk"
    gf = []
    if os.path.exists(bulk):
        with open(bulk) as f:
            vals = f.readline().split()
        for item in range(len(graph_feature_dim)):
            for ic in range(graph_feature_dim[item]):
                gf.append(float(vals[graph_feature_col[item] + ic]))
    elif energy is not None:
        gf = [energy]
    return Graph(x=torch.tensor(x, dtype=torch.float32), pos=torch.tensor(pos, dtype=torch.float32),
                 y=torch.tensor(gf, dtype=torch.float32), cell=torch.tensor(cell, dtype=torch.float32),
                 pbc=torch.tensor([True, True, True]))


def write_cfg(filepath, numbers, masses, frac, cell, aux=None, aux_names=(), energy=None):
    """Write an extended CFG file (species-grouped, reduced coordinates) that ``read_cfg``
    and AtomEye/ase read; ``aux`` [N, K] per-atom auxiliary columns."""
    from .elements import element_symbol

    numbers = np.asarray(numbers)
    aux = np.zeros((len(numbers), 0)) if aux is None else np.asarray(aux)
    with open(filepath, "w") as f:
        f.write(f"Number of particles = {len(numbers)}\n")
        if energy is not None:
            f.write(f"# energy = {energy:.10f}\n")
        f.write("A = 1.0 Angstrom (basic length-scale)\n")
        for i in range(3):
            for j in range(3):
                f.write(f"H0({i + 1},{j + 1}) = {cell[i][j]:.10f} A\n")
        f.write(".NO_VELOCITY.\n")
        f.write(f"entry_count = {3 + aux.shape[1]}\n")
        for k, name in enumerate(aux_names):
            f.write(f"auxiliary[{k}] = {name}\n")
        for zz in sorted(set(numbers.tolist())):
            sel = np.nonzero(numbers == zz)[0]
            f.write(f"{float(masses[sel[0]]):.6f}\n{element_symbol(int(zz))}\n")
            for i in sel:
                f.write(" ".join(f"{v:.10f}" for v in list(frac[i]) + list(aux[i])) + "\n")


def read_xyz(filepath, node_feature_dim=(), node_feature_col=(), graph_feature_dim=(1,), graph_feature_col=(0,)):
    """Extended-XYZ reader: line 1 = atom count, line 2 = graph values, then "Z x y z ..." rows."""
    with open(filepath) as f:
        lines = [l for l in f if l.strip()]
    n = int(lines[0])
    gvals = [float(v) for v in lines[1].split()]
    gf = []
    for item in range(len(graph_feature_dim)):
        for ic in range(graph_feature_dim[item]):
            gf.append(gvals[graph_feature_col[item] + ic])
    rows = [l.split() for l in lines[2:2 + n]]
    from .elements import atomic_number

    z = [atomic_number(r[0]) if not r[0].lstrip("-").isdigit() else int(r[0]) for r in rows]
    pos = [[float(r[1]), float(r[2]), float(r[3])] for r in rows]
    cols = [[float(zz), 0.0] + p + [float(v) for v in r[4:]] for zz, p, r in zip(z, pos, rows)]
    cols = np.array(cols)
    xs = []
    for item in range(len(node_feature_dim)):
        for ic in range(node_feature_dim[item]):
            xs.append(cols[:, node_feature_col[item] + ic])
    x = np.stack(xs, 1) if xs else cols[:, :1]
    return Graph(x=torch.tensor(x, dtype=torch.float32), pos=torch.tensor(pos, dtype=torch.float32),
                 y=torch.tensor(gf, dtype=torch.float32))


READERS = {"LSMS": read_lsms, "unit_test": read_lsms, "CFG": read_cfg, "XYZ": read_xyz}


def check_same_count_across_ranks(n, what=""):
    """All-reduce MIN and MAX of a host count over the host (gloo) group; raise if ranks disagree."""
    import torch
    import torch.distributed as dist

    from ..parallel.distributed import host_group

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return n
    t = torch.tensor([n, -n], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=host_group())
    if int(t[0]) != n or int(-t[1]) != n:
        raise RuntimeError(f"rank {dist.get_rank()} sees {n} files in {what}; ranks disagree "
                           f"(min {int(-t[1])}, max {int(t[0])})")
    return n


class RawDataLoader:
    """Raw directories -> normalised serialized split files (``raw_dataset_loader.py:26-277``)."""

    def __init__(self, dataset_config, dist=False):
        c = dataset_config
        self.node_feature_name = c["node_features"]["name"]
        self.node_feature_dim = c["node_features"]["dim"]
        self.node_feature_col = c["node_features"]["column_index"]
        self.graph_feature_name = c["graph_features"]["name"]
        self.graph_feature_dim = c["graph_features"]["dim"]
        self.graph_feature_col = c["graph_features"]["column_index"]
        self.raw_dataset_name = c["name"]
        self.data_format = c["format"]
        self.path_dictionary = c["path"]
        assert len(self.node_feature_name) == len(self.node_feature_dim) == len(self.node_feature_col)
        assert len(self.graph_feature_name) == len(self.graph_feature_dim) == len(self.graph_feature_col)
        self.dist = dist
        self.dataset_list = []
        self.serial_data_name_list = []

    def _read(self, fp):
        r = READERS[self.data_format]
        return r(fp, self.node_feature_dim, self.node_feature_col, self.graph_feature_dim, self.graph_feature_col)

    def load_raw_data(self, out_dir=None):
        import torch.distributed as dist

        out_dir = out_dir or os.path.join(os.environ.get("SERIALIZED_DATA_PATH", os.getcwd()), "serialized_dataset")
        os.makedirs(out_dir, exist_ok=True)
        for split, raw_path in self.path_dictionary.items():
            if not os.path.isabs(raw_path):
                raw_path = os.path.join(os.getcwd(), raw_path)
            if not os.path.exists(raw_path):
                raise ValueError("Folder not found: ", raw_path)
            files = sorted(os.listdir(raw_path))
            assert files, f"No data files provided in {raw_path}!"
            if self.dist and dist.is_initialized():
                import random

                from ..parallel.distributed import nsplit

                random.seed(43)
                random.shuffle(files)
                # C16 (``raw_dataset_loader.py:115-118``): every rank must see the same directory
                # listing before splitting it, or the per-rank shards overlap / drop files
                check_same_count_across_ranks(len(files), raw_path)
                files = list(nsplit(files, dist.get_world_size()))[dist.get_rank()]
            dataset = []
            for name in files:
                if name == ".DS_Store":
                    continue
                full = os.path.join(raw_path, name)
                if os.path.isfile(full):
                    dataset.append(self._read(full))
                elif os.path.isdir(full):
                    for sub in sorted(os.listdir(full)):
                        if os.path.isfile(os.path.join(full, sub)):
                            dataset.append(self._read(os.path.join(full, sub)))
            dataset = [d for d in dataset if d is not None]  # readers skip files of other kinds
            dataset = self.scale_features_by_num_nodes(dataset)
            fname = self.raw_dataset_name + (".pkl" if split == "total" else f"_{split}.pkl")
            self.dataset_list.append(dataset)
            self.serial_data_name_list.append(fname)
        self.normalize_dataset()
        for fname, ds in zip(self.serial_data_name_list, self.dataset_list):
            write_serialized(os.path.join(out_dir, fname), ds, self.minmax_node_feature, self.minmax_graph_feature)

    def scale_features_by_num_nodes(self, dataset):
        gi = [i for i, n in enumerate(self.graph_feature_name) if "_scaled_num_nodes" in n]
        ni = [i for i, n in enumerate(self.node_feature_name) if "_scaled_num_nodes" in n]
        for d in dataset:
            if d.y is not None and gi:
                d.y[gi] = d.y[gi] / d.num_nodes
            if d.x is not None and ni:
                d.x[:, ni] = d.x[:, ni] / d.num_nodes
        return dataset

    def normalize_dataset(self):
        ng, nn_ = len(self.graph_feature_dim), len(self.node_feature_dim)
        mg = np.full((2, ng), np.inf)
        mn = np.full((2, nn_), np.inf)
        mg[1] *= -1
        mn[1] *= -1
        for ds in self.dataset_list:
            for d in ds:
                s = 0
                for f in range(ng):
                    e = s + self.graph_feature_dim[f]
                    mg[0, f] = min(float(d.y[s:e].min()), mg[0, f])
                    mg[1, f] = max(float(d.y[s:e].max()), mg[1, f])
                    s = e
                s = 0
                for f in range(nn_):
                    e = s + self.node_feature_dim[f]
                    mn[0, f] = min(float(d.x[:, s:e].min()), mn[0, f])
                    mn[1, f] = max(float(d.x[:, s:e].max()), mn[1, f])
                    s = e
        if self.dist:
            from ..parallel.distributed import comm_reduce
            import torch.distributed as dist

            if dist.is_initialized():
                mg[0] = comm_reduce(torch.from_numpy(mg[0].copy()), dist.ReduceOp.MIN).numpy()
                mg[1] = comm_reduce(torch.from_numpy(mg[1].copy()), dist.ReduceOp.MAX).numpy()
                mn[0] = comm_reduce(torch.from_numpy(mn[0].copy()), dist.ReduceOp.MIN).numpy()
                mn[1] = comm_reduce(torch.from_numpy(mn[1].copy()), dist.ReduceOp.MAX).numpy()
        self.minmax_graph_feature, self.minmax_node_feature = mg, mn

        def _div(a, b):
            return torch.where(torch.tensor(b != 0), a / (b if b != 0 else 1.0), torch.zeros_like(a))

        for ds in self.dataset_list:
            for d in ds:
                s = 0
                for f in range(ng):
                    e = s + self.graph_feature_dim[f]
                    d.y[s:e] = _div(d.y[s:e] - mg[0, f], mg[1, f] - mg[0, f])
                    s = e
                s = 0
                for f in range(nn_):
                    e = s + self.node_feature_dim[f]
                    d.x[:, s:e] = _div(d.x[:, s:e] - mn[0, f], mn[1, f] - mn[0, f])
                    s = e
