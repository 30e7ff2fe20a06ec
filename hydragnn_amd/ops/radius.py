"""In-forward radius graphs on the device (reference ``RadiusInteractionGraph`` used by
SchNet, ``SCFStack.py:57-61``, and torch_cluster ``radius_graph``).

Batch-aware and chunked over receivers so memory stays O(chunk x N); edges come
out sorted by destination (CSR-ready) with a stable by-source permutation, so the
result plugs straight into the segment ops.  Cap policy follows torch_cluster: the
first ``max_num_neighbors`` sources in index order.
"""
import torch

from .segment import SegIndex


def radius_edges(pos, batch, r, max_num_neighbors=32, loop=False, chunk=4096):
    """edge_index [2, E] (row 0 = source j, row 1 = receiver i), sorted by receiver."""
    n = pos.shape[0]
    dev = pos.device
    if n == 0:
        return torch.zeros(2, 0, dtype=torch.long, device=dev)
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
