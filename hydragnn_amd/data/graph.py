"""Graph sample / mini-batch containers (replaces PyG ``Data``/``Batch``).

Schema follows the reference's use of PyG ``Data``:
``x [n,F]``, ``pos [n,3]``, ``edge_index [2,E]`` (row 0 = source j, row 1 =
destination i, PyG flow source_to_target), ``edge_attr [E,d]``,
``edge_shifts [E,3]``, ``y`` (packed targets) + ``y_loc [1,H+1]``,
``pe [n,k]``, ``rel_pe [E,k]``, ``dataset_name [1,1]``, ``energy``, ``forces``...

Collation mirrors PyG semantics (every tensor concatenated along dim 0,
``edge_index`` along dim -1 with a node-offset increment) and additionally
makes the batch **CSR-ready**: edges are sorted by destination inside every
sample, so the concatenated edge list is globally sorted by destination and
every aggregation is a contiguous, atomic-free segment reduce.  The
source-side permutation (for deterministic backward of source gathers) and
the node->graph CSR (``ptr``) are built once here.
"""
import numbers

import numpy as np
import torch

from .. import _native
from ..ops.segment import SegIndex

# keys whose leading dim is the edge count
EDGE_KEYS_PREFIX = ("edge_",)
EDGE_KEYS = {"rel_pe"}
INDEX_KEYS = {"edge_index"}


def is_edge_key(k):
    return (k.startswith(EDGE_KEYS_PREFIX) and k not in INDEX_KEYS) or k in EDGE_KEYS


class Graph:
    """Dictionary-backed graph sample with attribute access (PyG ``Data``-like)."""

    _std_keys = ("x", "pos", "edge_index", "edge_attr", "y", "batch", "pe", "rel_pe", "edge_shifts")

    def __init__(self, **kwargs):
        object.__setattr__(self, "_store", {})
        for k, v in kwargs.items():
            if v is not None:
                self._store[k] = v

    def __getattr__(self, k):
        store = object.__getattribute__(self, "_store")
        if k in store:
            return store[k]
        if k in Graph._std_keys:
            return None
        raise AttributeError(k)

    def __setattr__(self, k, v):
        if v is None:
            self._store.pop(k, None)
        else:
            self._store[k] = v

    def __delattr__(self, k):
        self._store.pop(k, None)

    def __contains__(self, k):
        return k in self._store

    def __getitem__(self, k):
        return self._store[k]

    def __setitem__(self, k, v):
        self._store[k] = v

    def get(self, k, default=None):
        return self._store.get(k, default)

    def keys(self):
        return list(self._store.keys())

    def items(self):
        return self._store.items()

    @property
    def num_nodes(self):
        s = self._store
        if "num_nodes" in s:
            return int(s["num_nodes"])
        for k in ("x", "pos", "pe"):
            if k in s and torch.is_tensor(s[k]):
                return s[k].shape[0]
        if "edge_index" in s and s["edge_index"].numel() > 0:
            return int(s["edge_index"].max()) + 1
        return 0

    @num_nodes.setter
    def num_nodes(self, n):
        self._store["num_nodes"] = int(n)

    @property
    def num_edges(self):
        ei = self._store.get("edge_index")
        return 0 if ei is None else ei.shape[1]

    def clone(self):
        return Graph(**{k: (v.clone() if torch.is_tensor(v) else v) for k, v in self._store.items()})

    def to(self, device, non_blocking=False):
        for k, v in list(self._store.items()):
            if torch.is_tensor(v):
                self._store[k] = v.to(device, non_blocking=non_blocking)
        return self

    def sort_edges_by_dst(self):
        """Stable sort of the sample's edges by destination (idempotent)."""
        ei = self._store.get("edge_index")
        if ei is None or ei.shape[1] < 2:
            return self
        dst = ei[1]
        if bool((dst[1:] >= dst[:-1]).all()):
            return self
        perm = torch.argsort(dst, stable=True)
        E = ei.shape[1]
        for k, v in list(self._store.items()):
            if k == "edge_index":
                self._store[k] = v[:, perm]
            elif is_edge_key(k) and torch.is_tensor(v) and v.dim() > 0 and v.shape[0] == E:
                self._store[k] = v[perm]
        return self

    def __repr__(self):
        parts = []
        for k, v in self._store.items():
            parts.append(f"{k}={list(v.shape)}" if torch.is_tensor(v) else f"{k}={v!r}")
        return "Graph(" + ", ".join(parts) + ")"


class GraphBatch(Graph):
    """A collated, CSR-ready mini-batch.

    Extra members: ``batch`` [N] (int64), ``ptr`` [G+1], ``num_graphs``, and
    three :class:`SegIndex` views: ``dst_si`` (edges -> destination nodes,
    sorted, no permutation), ``src_si`` (edges -> source nodes, with a stable
    permutation) and ``graph_si`` (nodes -> graphs, sorted).
    """

    def __init__(self, **kwargs):
        super().__init__(**kwargs)

    @property
    def num_graphs(self):
        return int(self._store["num_graphs"])

    def build_csr(self):
        s = self._store
        N = self.num_nodes
        G = int(s["num_graphs"])
        ptr = s["ptr"]
        s["graph_si"] = SegIndex(s["batch"].to(torch.int32), ptr.to(torch.int32), None, G)
        ei = s.get("edge_index")
        if ei is not None and ei.device.type == "cpu" and _native.available():
            drow, srow, sperm = _native.ops().csr_from_edges(ei[0], ei[1], N)
            s["dst_si"] = SegIndex(ei[1].to(torch.int32), drow, None, N)
            s["src_si"] = SegIndex(ei[0].to(torch.int32), srow, sperm, N)
        elif ei is not None:
            src, dst = ei[0], ei[1]
            dev = ei.device
            cnt = torch.bincount(dst, minlength=N)
            rowptr = torch.zeros(N + 1, dtype=torch.int32, device=dev)
            rowptr[1:] = torch.cumsum(cnt, 0)
            s["dst_si"] = SegIndex(dst.to(torch.int32), rowptr, None, N)
            scnt = torch.bincount(src, minlength=N)
            srowptr = torch.zeros(N + 1, dtype=torch.int32, device=dev)
            srowptr[1:] = torch.cumsum(scnt, 0)
            sperm = torch.argsort(src, stable=True).to(torch.int32)
            s["src_si"] = SegIndex(src.to(torch.int32), srowptr, sperm, N)
        return self

    def to(self, device, non_blocking=False):
        for k, v in list(self._store.items()):
            if torch.is_tensor(v):
                self._store[k] = v.to(device, non_blocking=non_blocking)
            elif isinstance(v, SegIndex):
                self._store[k] = v.to(device)
        return self

    def pin_memory(self):
        for k, v in list(self._store.items()):
            if torch.is_tensor(v):
                self._store[k] = v.pin_memory()
            elif isinstance(v, SegIndex):
                p = None if v.perm is None else v.perm.pin_memory()
                self._store[k] = SegIndex(v.index.pin_memory(), v.rowptr.pin_memory(), p, v.num_segments)
        return self

    def to_data_list(self):
        """Split back into per-sample Graphs (node/edge-level tensors only)."""
        s = self._store
        ptr = s["ptr"].tolist()
        out = []
        eptr = s.get("eptr")
        eptr = eptr.tolist() if eptr is not None else None
        for g in range(self.num_graphs):
            n0, n1 = ptr[g], ptr[g + 1]
            d = {}
            for k in ("x", "pos", "pe", "forces"):
                if k in s:
                    d[k] = s[k][n0:n1]
            if eptr is not None and "edge_index" in s:
                e0, e1 = eptr[g], eptr[g + 1]
                d["edge_index"] = s["edge_index"][:, e0:e1] - n0
                for k, v in s.items():
                    if is_edge_key(k) and torch.is_tensor(v):
                        d[k] = v[e0:e1]
            out.append(Graph(**d))
        return out


def collate(samples, build_csr=True):
    """Collate a list of :class:`Graph` into a CSR-ready :class:`GraphBatch`."""
    G = len(samples)
    assert G > 0, "cannot collate an empty list"
    nn = [s.num_nodes for s in samples]
    ne = [s.num_edges for s in samples]
    ptr = torch.zeros(G + 1, dtype=torch.long)
    ptr[1:] = torch.cumsum(torch.tensor(nn, dtype=torch.long), 0)
    eptr = torch.zeros(G + 1, dtype=torch.long)
    eptr[1:] = torch.cumsum(torch.tensor(ne, dtype=torch.long), 0)
    keys = []
    seen = set()
    for s in samples:
        for k in s.keys():
            if k not in seen:
                seen.add(k)
                keys.append(k)
    out = {}
    for k in keys:
        vals = [s.get(k) for s in samples]
        if any(v is None for v in vals):
            continue
        v0 = vals[0]
        if k == "edge_index":
            for s in samples:
                s.sort_edges_by_dst()
            vals = [s.get(k) for s in samples]
            if _native.available() and all(v.device.type == "cpu" for v in vals):
                out[k] = _native.ops().collate_edges(vals, torch.tensor(nn, dtype=torch.long))
            else:
                off = ptr[:-1].tolist()
                out[k] = torch.cat([v + o for v, o in zip(vals, off)], dim=1) if G > 1 else vals[0].clone()
        elif torch.is_tensor(v0):
            if v0.dim() == 0:
                out[k] = torch.stack(vals)
            else:
                out[k] = torch.cat(vals, dim=0)
        elif isinstance(v0, numbers.Number) and not isinstance(v0, bool):
            out[k] = torch.tensor(vals)
        elif isinstance(v0, np.ndarray):
            out[k] = torch.from_numpy(np.concatenate([np.atleast_1d(v) for v in vals]))
        else:
            out[k] = vals
    # edge-level tensors were sorted inside each sample by sort_edges_by_dst();
    # re-fetch them so the permuted versions are used.
    for k in keys:
        if is_edge_key(k) and torch.is_tensor(samples[0].get(k)):
            vals = [s.get(k) for s in samples]
            out[k] = torch.cat(vals, dim=0)
    N = int(ptr[-1])
    out.pop("num_nodes", None)
    b = GraphBatch(**out)
    b._store["num_nodes"] = N
    b._store["num_graphs"] = G
    b._store["ptr"] = ptr
    b._store["eptr"] = eptr
    b._store["batch"] = torch.repeat_interleave(torch.arange(G, dtype=torch.long), torch.tensor(nn, dtype=torch.long))
    if build_csr:
        b.build_csr()
    return b


# PyG-compatible alias
Data = Graph
Batch = GraphBatch


def head_targets(batch, head_types, head_dims):
    """Unpack the packed ``y``/``y_loc`` of a collated batch into per-head targets
    ([G, d] for graph heads, [N, d] for node heads), vectorised — replaces the
    reference's per-batch host index loops (``train_validate_test.py:316-379``)."""
    y = batch.y.reshape(-1)
    yl = batch.y_loc.to(y.device).long()
    G = yl.shape[0]
    total = yl[:, -1]
    start = torch.cumsum(total, 0) - total
    out = []
    ptr = batch.ptr.to(y.device).long()
    nnodes = ptr[1:] - ptr[:-1]
    for ih, (t, d) in enumerate(zip(head_types, head_dims)):
        base = start + yl[:, ih]
        if t == "graph":
            idx = base.view(-1, 1) + torch.arange(d, device=y.device).view(1, -1)
            out.append(y[idx.reshape(-1)].view(G, d))
        else:
            bnode = torch.repeat_interleave(torch.arange(G, device=y.device), nnodes)
            local = torch.arange(bnode.numel(), device=y.device) - ptr[bnode]
            idx = (base[bnode] + local * d).view(-1, 1) + torch.arange(d, device=y.device).view(1, -1)
            out.append(y[idx.reshape(-1)].view(-1, d))
    return out


def get_head_indices(head_types, head_dims, batch):
    """Reference-compatible flat indices into ``batch.y`` per head."""
    y = batch.y.reshape(-1)
    yl = batch.y_loc.long()
    G = yl.shape[0]
    if len(head_types) == 1:
        return [torch.arange(y.numel())]
    total = yl[:, -1]
    start = torch.cumsum(total, 0) - total
    out = []
    for ih in range(len(head_types)):
        s = start + yl[:, ih]
        e = start + yl[:, ih + 1]
        out.append(torch.cat([torch.arange(int(a), int(b)) for a, b in zip(s, e)]))
    return out
