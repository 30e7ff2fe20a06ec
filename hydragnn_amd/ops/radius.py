"""In-forward radius graphs on the device (reference ``RadiusInteractionGraph`` used by
SchNet, ``SCFStack.py:57-61``, and torch_cluster ``radius_graph``).

Batch-aware and chunked over receivers so memory stays O(chunk x N); edges come
out sorted by destination (CSR-ready) with a stable by-source permutation, so the
result plugs straight into the segment ops.  Cap policy follows torch_cluster: the
first ``max_num_neighbors`` sources in index order.
"""
import os

import torch

from .segment import SegIndex


def _graph_ptr(batch, n):
    """node->graph ids (contiguous graphs) -> (node_graph int32, gptr int32 [G+1])."""
    b = batch.to(torch.int32)
    G = int(batch.max()) + 1 if n else 0
    counts = torch.bincount(batch.long(), minlength=G)
    gptr = torch.zeros(G + 1, dtype=torch.int32, device=batch.device)
    gptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return b, gptr


def pbc_reps(cell, pbc, r):
    """Periodic image extents per graph: ceil(r / lattice-plane spacing) on periodic axes.
    cell [G, 3, 3] (rows = lattice vectors), pbc [G, 3] bool -> int32 [G, 3]."""
    cell = cell.double().view(-1, 3, 3)
    vol = torch.det(cell).abs()
    reps = []
    for a in range(3):
        b, c = cell[:, (a + 1) % 3], cell[:, (a + 2) % 3]
        h = vol / torch.linalg.norm(torch.cross(b, c, dim=1), dim=1)
        reps.append(torch.ceil(r / h))
    out = torch.stack(reps, 1).to(torch.int32)
    return out * torch.as_tensor(pbc, device=out.device).view(-1, 3).to(torch.int32)


def radius_graph_device(pos, batch, r, max_num_neighbors=32, loop=False, cap_policy="index", cell=None,
                        reps=None):
    """HIP radius graph (``csrc/graph.hip``): (edge_index [2, E], shifts [E, 3] or None).

    ``cell`` [G, 3, 3] / ``reps`` [G, 3] enable periodic images per graph; ``cap_policy``
    "index" (torch_cluster: first sources in index order) or "nearest" (RadiusGraphPBC)."""
    from .. import _native

    n = pos.shape[0]
    if batch is None:
        batch = torch.zeros(n, dtype=torch.long, device=pos.device)
    node_graph, gptr = _graph_ptr(batch.to(pos.device), n)
    k = -1 if max_num_neighbors is None else int(max_num_neighbors)
    ei, sh = _native.ops().radius_graph(pos.detach(), node_graph, gptr, float(r), k, bool(loop),
                                        cap_policy == "nearest", cell, reps)
    return ei, (sh if cell is not None else None)


def radius_edges(pos, batch, r, max_num_neighbors=32, loop=False, chunk=4096):
    """edge_index [2, E] (row 0 = source j, row 1 = receiver i), sorted by receiver."""
    n = pos.shape[0]
    dev = pos.device
    if n == 0:
        return torch.zeros(2, 0, dtype=torch.long, device=dev)
    if pos.is_cuda:  # HIP two-pass builder; same cap semantics as the torch path below
        return radius_graph_device(pos, batch, r, max_num_neighbors, loop)[0]
    if batch is None:
        batch = torch.zeros(n, dtype=torch.long, device=dev)
    batch = batch.to(dev).long()
    k = int(max_num_neighbors) if max_num_neighbors is not None else n
    srcs, dsts = [], []
    p = pos.detach()
    ar = torch.arange(n, device=dev)
    for i0 in range(0, n, chunk):
        i1 = min(n, i0 + chunk)
        d2 = torch.cdist(p[i0:i1], p)
        m = (d2 <= r) & (batch[i0:i1].view(-1, 1) == batch.view(1, -1))
        if not loop:
            m[torch.arange(i1 - i0, device=dev), ar[i0:i1]] = False
        keep = m & (torch.cumsum(m.to(torch.int32), dim=1) <= k)
        rows, cols = keep.nonzero(as_tuple=True)  # row-major: receiver-sorted, sources ascending
        dsts.append(rows + i0)
        srcs.append(cols)
    return torch.stack([torch.cat(srcs), torch.cat(dsts)], 0)


def csr_views(edge_index, n):
    """(dst_si, src_si) SegIndex views of a receiver-sorted edge list."""
    src, dst = edge_index[0], edge_index[1]
    dst_si = SegIndex.from_index(dst, n, sorted_=True)
    src_si = SegIndex.from_index(src, n, sorted_=False)
    return dst_si, src_si


def interaction_graph(pos, batch, r, max_num_neighbors=32):
    ei = radius_edges(pos, batch, r, max_num_neighbors)
    return csr_views(ei, pos.shape[0])


def interaction_graph_static(pos, data, r, max_num_neighbors=None):
    """In-forward radius graph of a statically padded batch with FIXED shapes and no host
    synchronisation (capturable; csrc/graph.hip ``radius_static_*``): each valid receiver
    keeps the first ``max_num_neighbors`` sources of its graph within ``r`` (index order,
    torch_cluster semantics); the edge list has capacity ``N * cap``, unused slots are
    self-edges of the last (padding) node.  Returns (dst_si, src_si)."""
    from .. import _native

    N = pos.shape[0]
    cap = 32 if max_num_neighbors is None else int(max_num_neighbors)
    Ecap = N * cap
    mask = data.get("node_mask")
    mask = None if mask is None else mask.view(-1).bool()
    batch, ptr = data.batch.long(), data.ptr.long()
    dummy = N - 1
    p = pos.detach()
    nmax = data.get("max_graph_nodes")
    if p.is_cuda and nmax and os.environ.get("HYDRA_RS_GRAPHS", "1") == "1":
        # one workgroup per graph, two launches (csrc/graph.hip rg_*): the dataset's largest
        # graph (a host int the store keeps) sizes the LDS edge list, fixed for a captured
        # bucket; a graph above it gets no edges and sets the "radius_graph_size" flag
        from . import devcheck

        out = _native.ops().radius_static_graphs(p, ptr, mask, float(r), cap, Ecap, dummy, int(nmax),
                                                 devcheck.flag(p.device, "radius_graph_size"))
        devcheck.debug_check("radius_graph_size", p.device)
        if out:
            src, dst, drp, limit, srp, sperm = out
            return SegIndex(dst, drp, None, N, limit), SegIndex(src, srp, sperm, N, limit)
    if p.is_cuda and os.environ.get("HYDRA_RS_SMALL", "1") == "1":
        # small batches: the whole builder (both CSR views) in one workgroup, one launch
        out = _native.ops().radius_static_small(p, batch, ptr, mask, float(r), cap, Ecap, dummy)
        if out:
            src, dst, drp, limit, srp, sperm = out
            return SegIndex(dst, drp, None, N, limit), SegIndex(src, srp, sperm, N, limit)
    if p.is_cuda:
        counts = _native.ops().radius_static_count(p, batch, ptr, mask, float(r), cap)
        rowptr = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0, dtype=torch.int32)])
        src, dst = _native.ops().radius_static_fill(p, batch, ptr, mask, float(r), cap, rowptr, Ecap, dummy)
    else:  # CPU twin (padded_step tests): identical edge order
        d = torch.cdist(p.float(), p.float())
        m = (d <= r) & (batch.view(-1, 1) == batch.view(1, -1))
        m.fill_diagonal_(False)
        if mask is not None:
            m &= mask.view(-1, 1) & mask.view(1, -1)
        keep = m & (torch.cumsum(m.to(torch.int32), dim=1) <= cap)
        dst_v, src_v = keep.nonzero(as_tuple=True)
        counts = keep.sum(1).to(torch.int32)
        rowptr = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0, dtype=torch.int32)])
        E = dst_v.numel()
        src = torch.full((Ecap,), dummy, dtype=torch.int32)
        dst = torch.full((Ecap,), dummy, dtype=torch.int32)
        src[:E], dst[:E] = src_v.int(), dst_v.int()
    drp = rowptr.clone()
    drp[N:].fill_(Ecap)  # the padding slots belong to the last (padding) receiver (device fill: capturable)
    # rowptr[N] = the real edge count: CSR positions past it are the slack (self-edges of the
    # padding node, last in both views); the native segment sums stop there instead of
    # walking the whole slack in one row (it was 30% of the QM9 SchNet step)
    limit = rowptr[N:N + 1]
    scnt = torch.zeros(N, dtype=torch.int32, device=src.device).index_add_(
        0, src.long(), torch.ones(Ecap, dtype=torch.int32, device=src.device))
    srp = torch.cat([scnt.new_zeros(1), torch.cumsum(scnt, 0, dtype=torch.int32)])
    sperm = torch.sort(src, stable=True).indices.to(torch.int32)
    return SegIndex(dst, drp, None, N, limit), SegIndex(src, srp, sperm, N, limit)


def radius_graph_cells(pos, batch, r, max_num_neighbors=None, loop=False, cap_policy="index", cell=None):
    """Cell-list (binned) HIP radius graph (``csrc/graph.hip`` ``radius_graph_cells``): O(N) for
    large structures, same output as ``radius_graph_device`` (edge set, cap policies, CSR order
    by receiver, shifts convention).  ``cell`` [G, 3, 3] (fully periodic graphs) or None.
    Returns (edge_index [2, E], shifts [E, 3] or None)."""
    from .. import _native

    dev = pos.device
    n = pos.shape[0]
    if batch is None:
        batch = torch.zeros(n, dtype=torch.long, device=dev)
    batch = batch.to(dev).long()
    node_graph, gptr = _graph_ptr(batch, n)
    G = gptr.numel() - 1
    p = pos.detach().to(torch.float32)
    k = -1 if max_num_neighbors is None else int(max_num_neighbors)
    if cell is not None:
        cellf = torch.as_tensor(cell, dtype=torch.float64, device=dev).view(-1, 3, 3)
        inv = torch.linalg.inv(cellf)
        vol = torch.abs(torch.linalg.det(cellf))
        h = torch.stack([vol / torch.linalg.norm(torch.cross(cellf[:, (a + 1) % 3], cellf[:, (a + 2) % 3], dim=1),
                                                 dim=1) for a in range(3)], 1)  # plane spacings [G, 3]
        nb = torch.clamp(torch.floor(h / r), min=1, max=512)
        st = torch.ceil(r / (h / nb) - 1e-9).clamp(min=1)
        rep = torch.ceil(r / h)
        lo = torch.zeros(G, 3, dtype=torch.float64, device=dev)
        geo = torch.cat([inv.reshape(G, 9), cellf.reshape(G, 9), lo], 1)
    else:
        lo = torch.full((G, 3), float("inf"), dtype=torch.float32, device=dev).scatter_reduce(
            0, batch.view(-1, 1).expand(-1, 3), p, "amin", include_self=True)
        hi = torch.full((G, 3), float("-inf"), dtype=torch.float32, device=dev).scatter_reduce(
            0, batch.view(-1, 1).expand(-1, 3), p, "amax", include_self=True)
        ext = (hi - lo).clamp(min=0)
        nb = torch.clamp(torch.floor(ext / r) + 1, min=1, max=1024).double()
        st = torch.ones_like(nb)
        rep = torch.zeros_like(nb)
        z9 = torch.zeros(G, 9, dtype=torch.float64, device=dev)
        geo = torch.cat([z9, z9, lo.double()], 1)
    grid = torch.cat([nb, st, rep], 1).to(torch.int32).contiguous()
    cells = nb.prod(1).long()
    off = torch.zeros(G + 1, dtype=torch.long, device=dev)
    off[1:] = torch.cumsum(cells, 0)
    ei, sh = _native.ops().radius_graph_cells(p, node_graph, grid, geo.to(torch.float32).contiguous(), off, float(r),
                                              k, bool(loop), cap_policy == "nearest", cell is not None)
    return ei, (sh if cell is not None else None)
