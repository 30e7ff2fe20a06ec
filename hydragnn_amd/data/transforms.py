"""Per-sample graph transforms (host reference implementations).

Replaces the PyG transforms used by the reference preprocessing
(``preprocess/serialized_dataset_loader.py:110-212``,
``preprocess/graph_samples_checks_and_updates.py:109-413``):
``RadiusGraph`` / ``RadiusGraphPBC`` (radius graph with ``max_num_neighbors``
cap), ``Distance`` (edge length, optionally normalised), ``Spherical``,
``PointPairFeatures``, ``NormalizeRotation``, ``AddLaplacianEigenvectorPE``
and ``rel_pe``.  Batched GPU versions live in ``ops/graph.py`` (HIP cell-list
radius graph, batched Jacobi eigensolver); these host versions are the
oracles and the fallback for CPU preprocessing.
"""
import math

import numpy as np
import torch


def radius_graph(pos, r, batch=None, max_num_neighbors=32, loop=False, cap_policy="index"):
    """Edges (j -> i) with ||pos_i - pos_j|| <= r within the same graph.

    ``cap_policy``: "nearest" keeps the closest ``max_num_neighbors`` sources per
    receiver (``RadiusGraphPBC._limit_neighbors`` semantics); "index" keeps the
    first found in index order (torch_cluster semantics).  Returns
    ``edge_index`` [2, E] sorted by destination then distance/index.
    """
    pos = torch.as_tensor(pos, dtype=torch.float64)
    n = pos.shape[0]
    if batch is None:
        batch = torch.zeros(n, dtype=torch.long)
    d = torch.cdist(pos, pos)
    same = batch.view(-1, 1) == batch.view(1, -1)
    mask = (d <= r) & same
    if not loop:
        mask.fill_diagonal_(False)
    if n == 0:
        return torch.zeros(2, 0, dtype=torch.long)
    if cap_policy == "nearest":
        key = torch.where(mask, d, torch.full_like(d, float("inf")))
        k = min(max_num_neighbors, n)
        vals, nb = torch.topk(key, k, dim=1, largest=False, sorted=True)
        ok = torch.isfinite(vals)
        # keep index order inside each receiver's list (stable & deterministic)
        nb = torch.where(ok, nb, torch.full_like(nb, n))
        nb, _ = torch.sort(nb, dim=1)
        ok = nb < n
    else:
        # first-found in index order (torch_cluster semantics)
        csum = torch.cumsum(mask.to(torch.long), dim=1)
        keep = mask & (csum <= max_num_neighbors)
        idx = torch.arange(n).view(1, -1).expand(n, n)
        nb = torch.where(keep, idx, torch.full_like(idx, n))
        nb, _ = torch.sort(nb, dim=1)
        nb = nb[:, :max_num_neighbors] if n > max_num_neighbors else nb
        ok = nb < n
    dst = torch.arange(n).view(-1, 1).expand_as(nb)[ok]
    src = nb[ok]
    return torch.stack([src, dst], 0)


def radius_graph_pbc(pos, cell, pbc, r, max_num_neighbors=32, loop=False):
    """Periodic radius graph over the 27 (or fewer, per non-periodic axis) image
    cells; returns (edge_index [2,E], edge_shifts [E,3]) with
    ``pos[dst] - pos[src] + shift`` the minimum-image-consistent vector, nearest
    ``max_num_neighbors`` kept per receiver (``RadiusGraphPBC``, reference
    ``graph_samples_checks_and_updates.py:141-343``)."""
    pos = torch.as_tensor(pos, dtype=torch.float64)
    cell = torch.as_tensor(cell, dtype=torch.float64).view(3, 3)
    pbc = [bool(p) for p in torch.as_tensor(pbc).view(-1).tolist()]
    n = pos.shape[0]
    # number of images needed per axis: r / (plane spacing)
    vol = torch.abs(torch.det(cell))
    reps = []
    for a in range(3):
        if not pbc[a]:
            reps.append(0)
            continue
        b, c = cell[(a + 1) % 3], cell[(a + 2) % 3]
        h = vol / torch.linalg.norm(torch.cross(b, c, dim=0))
        reps.append(int(math.ceil(r / float(h))))
    rng = [torch.arange(-k, k + 1, dtype=torch.float64) for k in reps]
    grid = torch.stack(torch.meshgrid(*rng, indexing="ij"), -1).view(-1, 3)
    shifts = grid @ cell  # [S,3]
    # vec[i, j, s] = pos[i] - (pos[j] + shift_s)  -> edge j(+s) -> i with shift = -shift_s
    srcs, dsts, shs, ds = [], [], [], []
    for s in range(shifts.shape[0]):
        diff = pos.view(n, 1, 3) - (pos.view(1, n, 3) + shifts[s])
        d = torch.linalg.norm(diff, dim=-1)
        m = d <= r
        if not loop and bool((grid[s] == 0).all()):
            m.fill_diagonal_(False)
        ii, jj = torch.nonzero(m, as_tuple=True)
        dsts.append(ii)
        srcs.append(jj)
        shs.append((-shifts[s]).expand(ii.numel(), 3) * -1.0)
        ds.append(d[ii, jj])
    dst = torch.cat(dsts)
    src = torch.cat(srcs)
    sh = torch.cat(shs)
    dist = torch.cat(ds)
    # cap per receiver: nearest first
    order = torch.argsort(dst * (dist.max() + 1.0 if dist.numel() else 1.0) + dist)
    dst, src, sh, dist = dst[order], src[order], sh[order], dist[order]
    keep = torch.ones_like(dst, dtype=torch.bool)
    if dst.numel():
        first = torch.ones_like(dst, dtype=torch.bool)
        first[1:] = dst[1:] != dst[:-1]
        idx = torch.arange(dst.numel())
        start = torch.cummax(torch.where(first, idx, torch.zeros_like(idx)), 0).values
        keep = (idx - start) < max_num_neighbors
    ei = torch.stack([src[keep], dst[keep]], 0)
    # shift convention: vec = pos[dst] - pos[src] + shift  -> shift = -(image shift of the source)
    return ei, sh[keep].to(torch.float32) * -1.0


def missing_receivers(edge_index, num_nodes):
    """Nodes that receive no edge."""
    dst = torch.as_tensor(edge_index)[1]
    has = torch.zeros(int(num_nodes), dtype=torch.bool)
    if dst.numel():
        has[dst] = True
    return (~has).nonzero().view(-1)


def ensure_connected(edge_index, edge_shifts, num_nodes, seed=None):
    """Give every receiver-less node one artificial incoming edge from a random other node
    with zero cell shift (reference ``RadiusGraphPBC._ensure_connected``,
    ``graph_samples_checks_and_updates.py:284-307``).  Returns (edge_index, edge_shifts,
    number of edges added)."""
    miss = missing_receivers(edge_index, num_nodes)
    if miss.numel() == 0:
        return edge_index, edge_shifts, 0
    print(f"WARNING: {miss.numel()} node(s) receive no edge; adding artificial edges", flush=True)
    rng = np.random.default_rng(seed)
    src = []
    for m in miss.tolist():
        if num_nodes > 1:
            s = int(rng.integers(num_nodes - 1))
            src.append(s + (s >= m))  # uniform over the other nodes
        else:
            src.append(0)
    add = torch.stack([torch.tensor(src, dtype=edge_index.dtype), miss.to(edge_index.dtype)], 0)
    ei = torch.cat([edge_index, add], 1)
    sh = None if edge_shifts is None else torch.cat([edge_shifts, edge_shifts.new_zeros(miss.numel(), 3)], 0)
    return ei, sh, int(miss.numel())


def radius_graph_pbc_robust(pos, cell, pbc, r, max_num_neighbors=32, loop=False, multiplier=1.25, max_attempts=3,
                            seed=None):
    """``radius_graph_pbc`` with the reference's failure handling (``RadiusGraphPBC.__call__``,
    ``graph_samples_checks_and_updates.py:161-222``): while some node receives no edge the
    cutoff grows by ``multiplier`` (at most ``max_attempts`` builds), then any node still
    without a receiver edge gets an artificial one (``ensure_connected``).  Returns
    (edge_index, edge_shifts, cutoff used)."""
    n = int(torch.as_tensor(pos).shape[0])
    cutoff = float(r)
    for attempt in range(max_attempts):
        ei, sh = radius_graph_pbc(pos, cell, pbc, cutoff, max_num_neighbors, loop)
        if missing_receivers(ei, n).numel() == 0:
            return ei, sh, cutoff
        if attempt < max_attempts - 1:
            print(f"Not all nodes receive an edge, expanding radius from {cutoff} -> {cutoff * multiplier}",
                  flush=True)
            cutoff *= multiplier
    ei, sh, _ = ensure_connected(ei, sh, n, seed)
    return ei, sh, cutoff


def local_cartesian(pos, edge_index, shifts=None, norm=True, interval=(0.0, 1.0), cat=False, edge_attr=None):
    """PyG ``LocalCartesian`` / reference ``PBCLocalCartesian`` (``:379-413``): relative
    Cartesian offset pos[src] - pos[dst] (- shift), optionally scaled per receiver by its
    largest |component| into ``interval``."""
    row, col = edge_index[0], edge_index[1]
    cart = pos[row] - pos[col]
    if shifts is not None:
        cart = cart - shifts
    if norm and cart.numel():
        n = pos.shape[0]
        mx = torch.zeros(n, dtype=cart.dtype).scatter_reduce(0, col, cart.abs().max(dim=-1).values, "amax",
                                                              include_self=True)
        length = interval[1] - interval[0]
        center = (interval[0] + interval[1]) / 2
        cart = length * cart / (2 * mx[col].clamp_min(1e-9).view(-1, 1)) + center
    if cat and edge_attr is not None:
        return torch.cat([edge_attr.view(edge_attr.shape[0], -1), cart.to(edge_attr.dtype)], dim=-1)
    return cart


def pbc_distance(pos, edge_index, shifts, norm=True, max_value=None, cat=False, edge_attr=None):
    """Reference ``PBCDistance`` (``:346-376``): ``distance`` with the periodic shift added."""
    return distance(pos, edge_index, shifts=shifts, norm=norm, max_value=max_value, cat=cat, edge_attr=edge_attr)


def distance(pos, edge_index, shifts=None, norm=True, max_value=None, cat=False, edge_attr=None):
    """PyG ``Distance``: edge length, optionally divided by max (global max if given)."""
    vec = pos[edge_index[1]] - pos[edge_index[0]]
    if shifts is not None:
        vec = vec + shifts
    d = torch.linalg.norm(vec, dim=-1, keepdim=True)
    if norm and d.numel() > 0:
        d = d / (d.max() if max_value is None else max_value)
    if cat and edge_attr is not None:
        return torch.cat([edge_attr.view(edge_attr.shape[0], -1), d.to(edge_attr.dtype)], dim=-1)
    return d


def laplacian_pe(edge_index, num_nodes, k, seed=None, sign_flip=True):
    """PyG ``AddLaplacianEigenvectorPE(k, is_undirected=True)``: eigenvectors 1..k of the
    symmetric-normalised Laplacian (ascending eigenvalues, trivial one skipped),
    zero-padded when the graph is smaller than k+1, random sign per vector."""
    n = int(num_nodes)
    A = np.zeros((n, n), dtype=np.float64)
    ei = np.asarray(edge_index)
    if ei.size:
        A[ei[1], ei[0]] = 1.0
        A[ei[0], ei[1]] = 1.0
    deg = A.sum(1)
    dinv = np.where(deg > 0, 1.0 / np.sqrt(np.maximum(deg, 1e-12)), 0.0)
    L = np.eye(n) - dinv[:, None] * A * dinv[None, :]
    w, V = np.linalg.eigh(L)
    V = V[:, np.argsort(w)]
    pe = np.zeros((n, k), dtype=np.float32)
    m = min(k, max(n - 1, 0))
    if m > 0:
        pe[:, :m] = V[:, 1:m + 1]
    if sign_flip:
        rng = np.random.default_rng(seed)
        pe *= (-1.0 + 2.0 * rng.integers(0, 2, size=(1, k))).astype(np.float32)
    return torch.from_numpy(pe)


def relative_pe(pe, edge_index):
    return torch.abs(pe[edge_index[0]] - pe[edge_index[1]])


def normalize_rotation(pos, max_points=-1, sort=False):
    """PyG ``NormalizeRotation``: rotate onto the principal axes (PCA via SVD)."""
    pos = torch.as_tensor(pos)
    p = pos[:max_points] if max_points > 0 else pos
    p = p - p.mean(dim=0, keepdim=True)
    C = p.t() @ p
    e, v = torch.linalg.eigh(C)
    if sort:
        idx = e.argsort(descending=True)
        v = v[:, idx]
    return (pos - pos.mean(dim=0, keepdim=True)) @ v


def spherical(pos, edge_index, norm=True, max_value=None):
    """PyG ``Spherical``: (rho, theta, phi) per edge."""
    vec = pos[edge_index[1]] - pos[edge_index[0]]
    rho = torch.linalg.norm(vec, dim=-1, keepdim=True)
    theta = torch.atan2(vec[:, 1], vec[:, 0]).view(-1, 1)
    theta = theta + (theta < 0).to(theta.dtype) * (2 * math.pi)
    phi = torch.acos((vec[:, 2] / rho.view(-1).clamp(min=1e-12)).clamp(-1, 1)).view(-1, 1)
    if norm:
        rho = rho / (rho.max() if max_value is None else max_value)
        theta = theta / (2 * math.pi)
        phi = phi / math.pi
    return torch.cat([rho, theta, phi], dim=-1)


def point_pair_features(pos, normal, edge_index):
    """PyG ``PointPairFeatures`` (needs per-node normals)."""
    d = pos[edge_index[0]] - pos[edge_index[1]]
    n1, n2 = normal[edge_index[1]], normal[edge_index[0]]

    def ang(v1, v2):
        return torch.atan2(torch.linalg.norm(torch.cross(v1, v2, dim=1), dim=1), (v1 * v2).sum(1))

    return torch.stack([torch.linalg.norm(d, dim=1), ang(n1, d), ang(n2, d), ang(n1, n2)], dim=1)


def laplacian_pe_batch(samples, k, seed=None, device=None, max_sweeps=30, tol=1e-7):
    """``laplacian_pe`` for a list of samples at once.  On a GPU device (and graphs of
    <= 128 nodes) the batched Jacobi HIP kernel (``csrc/spectral.hip``, one workgroup per
    graph, matrices in LDS) diagonalises every Laplacian in one launch; otherwise the
    per-graph host path.  Returns a list of [n_i, k] tensors (CPU)."""
    from .graph import collate

    dev = torch.device(device) if device is not None else None
    if dev is None or dev.type != "cuda" or not samples or max(s.num_nodes for s in samples) > 128:
        rng = np.random.default_rng(seed)
        return [laplacian_pe(s.edge_index, s.num_nodes, k, seed=int(rng.integers(1 << 30))) for s in samples]
    from .. import _native

    b = collate([type(s)(edge_index=s.edge_index, x=torch.zeros(s.num_nodes, 1)) for s in samples])
    rng = np.random.default_rng(seed)
    signs = torch.from_numpy((-1.0 + 2.0 * rng.integers(0, 2, size=(len(samples), k))).astype(np.float32))
    ei = b.edge_index.to(dev)
    pe, _ = _native.ops().laplacian_pe(ei, b.dst_si.rowptr.to(dev), b.ptr.to(dev, torch.int32), int(k),
                                       signs.to(dev), int(max_sweeps), float(tol))
    pe = pe.cpu()
    return [pe[int(b.ptr[g]):int(b.ptr[g + 1])] for g in range(len(samples))]


def build_radius_graphs_gpu(samples, r, max_num_neighbors, pbc=False, device="cuda"):
    """Radius graphs of a whole dataset in ONE batched launch of the cell-list HIP builder
    (``ops.radius.radius_graph_cells``) instead of one host ``cdist`` per sample.  Periodic
    samples use the "nearest" cap (RadiusGraphPBC) and then the reference's retry /
    connectivity repair per sample (``radius_graph_pbc_robust``); non-periodic samples the
    torch_cluster "index" cap.  Returns a list of (edge_index, edge_shifts or None) on the CPU."""
    from ..ops.radius import radius_graph_cells

    dev = torch.device(device)
    n = [int(s.num_nodes) for s in samples]
    pos = torch.cat([s.pos.to(torch.float32) for s in samples]).to(dev)
    batch = torch.repeat_interleave(torch.arange(len(samples)), torch.tensor(n)).to(dev)
    cell = None
    if pbc:
        cell = torch.stack([torch.as_tensor(s.cell, dtype=torch.float32).view(3, 3) for s in samples]).to(dev)
    cap = None if max_num_neighbors is None else int(max_num_neighbors)
    policy = "nearest" if pbc else "index"
    native_cap = cap if (cap is not None and cap <= 64) else None
    ei, sh = radius_graph_cells(pos, batch, r, native_cap, cap_policy=policy, cell=cell)
    if cap is not None and native_cap is None:  # wide caps: uncapped build, cap per receiver here
        if policy == "nearest":
            vec = pos[ei[1]] - pos[ei[0]] + (sh if sh is not None else 0.0)
            d = vec.norm(dim=1)
            order = torch.argsort(ei[1].double() * (float(d.max()) + 1.0 if d.numel() else 1.0) + d.double(),
                                  stable=True)
            ei = ei[:, order]
            sh = sh[order] if sh is not None else None
        dst = ei[1]
        first = torch.ones_like(dst, dtype=torch.bool)
        first[1:] = dst[1:] != dst[:-1]
        idx = torch.arange(dst.numel(), device=dev)
        start = torch.cummax(torch.where(first, idx, torch.zeros_like(idx)), 0).values
        keep = (idx - start) < cap
        ei = ei[:, keep]
        sh = sh[keep] if sh is not None else None
    ei, sh = ei.cpu(), (sh.cpu() if sh is not None else None)
    off = np.concatenate([[0], np.cumsum(n)])
    bounds = torch.searchsorted(ei[1].contiguous(), torch.as_tensor(off, dtype=torch.long))
    out = []
    for g, s in enumerate(samples):
        a, b = int(bounds[g]), int(bounds[g + 1])
        e = ei[:, a:b] - int(off[g])
        shg = sh[a:b] if sh is not None else None
        if pbc and missing_receivers(e, n[g]).numel():
            e, shg, _ = radius_graph_pbc_robust(s.pos, s.cell, s.get("pbc", [True, True, True]), r,
                                                cap if cap is not None else 1 << 30)
        out.append((e, shg))
    return out
