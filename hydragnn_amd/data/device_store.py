"""HBM-resident graph dataset with host-indexed GPU batch assembly.

MI355X design (SURVEY §7.1 decision 3): with 288 GB of HBM per GPU an entire
training shard lives on the device.  Every per-sample tensor is concatenated
once into a field-major pool (node fields [sum n, F], edge fields [sum e, F],
graph fields [S, F]); per-sample offsets are kept on the HOST.  Building a
mini-batch then needs no device->host synchronisation:

1. ``plan()`` (host, numpy, ~100 us): from offsets alone it computes the node /
   edge row lists, destination CSR (edges are pre-sorted by destination inside
   every sample), source CSR (per-sample stable source permutations are
   precomputed at load time and concatenated with edge offsets), ``batch`` /
   ``ptr`` and the attention segments, packed into ONE int32 array;
2. that array travels in ONE pinned asynchronous H2D copy;
3. ``assemble()`` (device only) gathers the feature rows out of the HBM pool.

This replaces the reference's CPU DataLoader + PyG ``Batch.from_data_list`` +
per-step H2D of every feature tensor (``train_validate_test.py:514``) and the
host-side ``get_head_indices`` loops (``:316-379``): per-head targets come out
as ready [G, d] / [N, d] tensors.

Static padding (``Np``/``Ep``/``Gp``) produces fixed-shape batches so that
``assemble`` + forward + backward + optimizer can be captured once in a hipGraph
and replayed (``train/step.py``): padded nodes form an extra dummy graph (and an
extra attention segment), padded edges are spread over the padded nodes
(bounded degree, no self-loops), padded nodes sit at distinct finite positions
(no zero-length edges), the model zeroes padded node rows after every layer,
and the device scalars ``num_valid`` / ``num_graphs_valid`` drive the masked
reductions.
"""
import functools
import os
import time

import numpy as np
import torch

from ..ops.segment import SegIndex
from .graph import GraphBatch

NODE_KEYS = ("x", "pos", "pe", "forces")
EDGE_KEYS = ("edge_attr", "rel_pe", "edge_shifts")

_PLAN_FIELDS = ("node_rows", "edge_rows", "src", "dst", "sperm", "rowptr", "srowptr", "batch", "gptr",
                "aseg_id", "aseg_ptr", "sample_idx", "scalars")


class Layout:
    """Static sizes of one packed batch plan."""

    __slots__ = ("Np", "Ep", "Gp", "padded", "attn_scope", "sizes", "total")

    def __init__(self, Np, Ep, Gp, padded, attn_scope):
        self.Np, self.Ep, self.Gp, self.padded, self.attn_scope = Np, Ep, Gp, padded, attn_scope
        na = 3 if attn_scope == "batch" else Gp + 1
        self.sizes = [Np, Ep, Ep, Ep, Ep, Np + 1, Np + 1, Np, Gp + 1, Np, na, Gp, 4]
        self.total = int(sum(self.sizes))

    def key(self):
        return (self.Np, self.Ep, self.Gp, self.padded, self.attn_scope)


class DeviceGraphStore:
    def __init__(self, samples, device, head_types=None, head_dims=None, node_keys=NODE_KEYS, edge_keys=EDGE_KEYS,
                 graph_keys=("energy",), dtype=torch.float32, attn_scope="batch"):
        self.device = torch.device(device)
        self.attn_scope = attn_scope
        S = len(samples)
        self.num_samples = S
        nn_ = np.array([s.num_nodes for s in samples], dtype=np.int64)
        ne = np.array([s.num_edges for s in samples], dtype=np.int64)
        self.n_nodes, self.n_edges = nn_, ne
        self.max_graph_nodes = int(nn_.max()) if S else 0  # static bound for per-graph kernels
        self.node_off = np.zeros(S + 1, dtype=np.int64)
        self.node_off[1:] = np.cumsum(nn_)
        self.edge_off = np.zeros(S + 1, dtype=np.int64)
        self.edge_off[1:] = np.cumsum(ne)
        for s in samples:
            s.sort_edges_by_dst()
        self.src_local = np.concatenate([s.edge_index[0].numpy() for s in samples]).astype(np.int64)
        self.dst_local = np.concatenate([s.edge_index[1].numpy() for s in samples]).astype(np.int64)
        self.sperm_local = np.concatenate(
            [np.argsort(s.edge_index[0].numpy(), kind="stable") for s in samples]).astype(np.int64)
        self.node_keys = [k for k in node_keys if all(k in s for s in samples)]
        self.edge_keys = [k for k in edge_keys if all(k in s for s in samples)]
        self.graph_keys = [k for k in graph_keys if all(k in s for s in samples)]
        self.fields = {}
        for k in self.node_keys + self.edge_keys:
            self.fields[k] = torch.cat([s[k].reshape(s[k].shape[0], -1).to(dtype) for s in samples], 0).to(self.device)
        for k in self.graph_keys:
            self.fields[k] = torch.stack([s[k].reshape(-1).to(dtype) for s in samples], 0).to(self.device)
        self.head_types = list(head_types) if head_types is not None else None
        self.head_dims = list(head_dims) if head_dims is not None else None
        self.targets_graph, self.targets_node = {}, {}
        if self.head_types is not None and all("y" in s for s in samples):
            for ih, (t, d) in enumerate(zip(self.head_types, self.head_dims)):
                vals = []
                for s in samples:
                    yl = s["y_loc"].view(-1)
                    vals.append(s["y"].view(-1)[int(yl[ih]):int(yl[ih + 1])].view(-1, d).to(dtype))
                tgt = torch.cat(vals, 0).to(self.device)
                (self.targets_graph if t == "graph" else self.targets_node)[ih] = tgt
        self.dataset_name = None
        if all("dataset_name" in s for s in samples):
            self.dataset_name = np.array([int(s["dataset_name"].view(-1)[0]) for s in samples], dtype=np.int64)
            self.dataset_name_dev = torch.from_numpy(self.dataset_name).to(self.device)
        self._ring = []
        self._ring_pos = 0
        self.slot_wait_s = 0.0  # host seconds spent waiting for a pinned plan slot (the GPU is behind)
        self.phase_s = {}  # host seconds per upload phase (plan, copy call incl. event record)

    def __len__(self):
        return self.num_samples

    def memory_bytes(self):
        return sum(t.numel() * t.element_size() for t in self.fields.values())

    # ------------------------------------------------------------------ host side
    def sizes_of(self, indices):
        idx = np.asarray(indices, dtype=np.int64)
        return int(self.n_nodes[idx].sum()), int(self.n_edges[idx].sum())

    def layout(self, indices, Np=None, Ep=None, Gp=None):
        N, E = self.sizes_of(indices)
        G = len(indices)
        padded = Np is not None
        if padded:
            Np = max(Np, N + 2)
            Ep = max(Ep if Ep is not None else E, E)
            Gp = max(Gp if Gp is not None else G + 1, G + 1)
        else:
            Np, Ep, Gp = N, E, G
        return Layout(Np, Ep, Gp, padded, self.attn_scope)

    def triplet_cap(self, G, Ep=None):
        """Upper bound on the DimeNet triplet count (k -> j -> i, k != i) of any batch of at
        most ``G`` graphs (and at most ``Ep`` edges): the smaller of the sum of the ``G``
        largest per-graph counts and ``Ep`` x the largest per-graph triplets-per-edge ratio,
        rounded up to 256.  A padded batch carries it (``triplet_cap``) so the model can build
        its triplets on the device with a fixed capacity (models/dimenet.triplets_static)."""
        cs = getattr(self, "_tri_cum", None)
        if cs is None:
            S = self.num_samples
            e_sample = np.repeat(np.arange(S), self.n_edges)
            gs = self.src_local + self.node_off[:-1][e_sample]
            gd = self.dst_local + self.node_off[:-1][e_sample]
            Ntot = int(self.node_off[-1])
            indeg = np.bincount(gd, minlength=Ntot)
            per_edge = indeg[gs].astype(np.int64)
            # minus the in-edges k -> j of j whose source is i (the back edges of j -> i)
            key = gs * Ntot + gd
            rkey = gd * Ntot + gs
            uk, uc = np.unique(key, return_counts=True)
            pos = np.searchsorted(uk, rkey)
            pos_c = np.minimum(pos, max(uk.size - 1, 0))
            back = np.where((uk.size > 0) & (uk[pos_c] == rkey), uc[pos_c], 0) if uk.size else np.zeros_like(rkey)
            per_edge -= back
            t = np.bincount(e_sample, weights=per_edge, minlength=S).astype(np.int64)
            cs = self._tri_cum = np.concatenate([[0], np.cumsum(np.sort(t)[::-1])])
            ne = self.n_edges
            self._tri_ratio = float(np.max(t[ne > 0] / ne[ne > 0])) if (ne > 0).any() else 0.0
        G = max(0, min(int(G), cs.size - 1))
        cap = int(cs[G])
        if Ep is not None:  # T = sum_g r_g E_g <= max_g r_g * Ep
            cap = min(cap, int(np.ceil(self._tri_ratio * int(Ep))) + 1)
        return int(max(256, -(-cap // 256) * 256))

    def _native_plan_args(self):
        t = getattr(self, "_plan_t", None)
        if t is None:
            c = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64))  # noqa: E731
            t = self._plan_t = (c(self.n_nodes), c(self.n_edges), c(self.node_off), c(self.edge_off),
                                c(self.src_local), c(self.dst_local), c(self.sperm_local))
        return t

    def plan(self, indices, lay, out=None):
        """Fill the packed int32 plan for ``indices`` (numpy view ``out`` of size lay.total):
        native C++ (``csrc/collate.cpp`` store_plan) when the library is loaded, else the
        numpy reference ``plan_numpy`` (identical values; tests/test_store_plan.py)."""
        from .. import _native

        if out is None:
            out = np.empty(lay.total, dtype=np.int32)
        if _native.available():
            idx = torch.from_numpy(np.ascontiguousarray(indices, dtype=np.int64))
            _native.ops().store_plan(idx, *self._native_plan_args(), torch.from_numpy(out), lay.Np, lay.Ep, lay.Gp,
                                     bool(lay.padded), lay.attn_scope == "batch")
            return out
        return self.plan_numpy(indices, lay, out)

    # ------------------------------------------------------------------ device-side plan
    def device_plan_ok(self, lay):
        """The captured step can expand the plan on the device (csrc/assemble.hip
        store_plan_expand) from the sample ids alone."""
        from .. import _native

        return (self.device.type == "cuda" and lay.Gp <= 4096 and _native.available()
                and os.environ.get("HYDRA_DEVICE_PLAN", "1") == "1")

    def _dev_plan_tabs(self):
        t = getattr(self, "_dplan", None)
        if t is None:
            S = self.num_samples
            i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(self.device)  # noqa: E731
            Ntot, Etot = int(self.node_off[-1]), int(self.edge_off[-1])
            e_sample = np.repeat(np.arange(S), self.n_edges)
            n_sample = np.repeat(np.arange(S), self.n_nodes)
            # per-sample local CSR row starts: every earlier sample's edges come first globally
            gd = self.dst_local + self.node_off[:-1][e_sample]
            gs = self.src_local + self.node_off[:-1][e_sample]
            dc = np.zeros(Ntot + 1, dtype=np.int64)
            np.cumsum(np.bincount(gd, minlength=Ntot), out=dc[1:])
            sc = np.zeros(Ntot + 1, dtype=np.int64)
            np.cumsum(np.bincount(gs, minlength=Ntot), out=sc[1:])
            base = self.edge_off[:-1][n_sample]
            t = self._dplan = [i32(self.n_nodes), i32(self.n_edges), i32(self.node_off[:-1]), i32(self.edge_off[:-1]),
                               i32(self.src_local), i32(self.dst_local), i32(self.sperm_local), i32(dc[:-1] - base),
                               i32(sc[:-1] - base)]
            assert Etot == self.src_local.size
        return t

    def seed(self, indices, lay, out):
        """Host part of the device-side plan: out[0] = G, out[1 + g] = sample id (int32 view of
        ``lay.Gp + 1`` entries); the layout must hold the batch (as for ``plan``)."""
        idx = np.asarray(indices, dtype=np.int64)
        G = idx.size
        N, E = self.sizes_of(idx)
        if N > lay.Np or E > lay.Ep or G > lay.Gp or (lay.padded and (N + 2 > lay.Np or G + 1 > lay.Gp)):
            raise ValueError("seed: batch exceeds the layout")
        if G and (idx.min() < 0 or idx.max() >= self.num_samples):
            raise ValueError("seed: sample index out of range")
        out[0] = G
        out[1:1 + G] = idx
        out[1 + G:] = 0
        return out

    def plan_device(self, seed, lay, out, rng=None):
        """Expand ``seed`` (device int32, see ``seed``) into the packed plan ``out`` on the device:
        the same values as ``plan`` (tests/test_device_plan_gpu.py).  ``rng``: an int64 device
        counter the launch also advances by one (the step's dropout counter)."""
        from .. import _native

        _native.ops().store_plan_expand(seed, self._dev_plan_tabs(), out, lay.Np, lay.Ep, lay.Gp, bool(lay.padded),
                                        lay.attn_scope == "batch", rng)
        return out

    def plan_numpy(self, indices, lay, out=None):
        """numpy reference of ``plan`` (the oracle of the native builder)."""
        idx = np.asarray(indices, dtype=np.int64)
        G = idx.size
        n = self.n_nodes[idx]
        e = self.n_edges[idx]
        N, E = int(n.sum()), int(e.sum())
        Np, Ep, Gp = lay.Np, lay.Ep, lay.Gp
        ptr = np.zeros(G + 1, dtype=np.int64)
        ptr[1:] = np.cumsum(n)
        eptr = np.zeros(G + 1, dtype=np.int64)
        eptr[1:] = np.cumsum(e)
        edge_rows = _ranges(self.edge_off[idx], e)
        nbase_e = np.repeat(ptr[:-1], e)
        if out is None:
            out = np.empty(lay.total, dtype=np.int32)
        views = []
        o = 0
        for sz in lay.sizes:
            views.append(out[o:o + sz])
            o += sz
        (node_rows, erows, src, dst, sperm, rowptr, srowptr, batch, gptr, aseg_id, aseg_ptr, sidx, scal) = views
        node_rows[:N] = _ranges(self.node_off[idx], n)
        erows[:E] = edge_rows
        src[:E] = self.src_local[edge_rows] + nbase_e
        dst[:E] = self.dst_local[edge_rows] + nbase_e
        sperm[:E] = self.sperm_local[edge_rows] + np.repeat(eptr[:-1], e)
        batch[:N] = np.repeat(np.arange(G), n)
        gptr[:G + 1] = ptr
        sidx[:G] = idx
        if lay.padded:
            node_rows[N:] = -1
            erows[E:] = -1
            # padded edges spread evenly over the padded nodes (bounded degrees keep the
            # dummy rows numerically tame), never self-loops, destination-sorted
            pn, pe = Np - N, Ep - E
            if pe:
                k = np.arange(pe)
                pd = (k * pn) // pe
                ps = (pd + 1) % pn
                dst[E:] = N + pd
                src[E:] = N + ps
                sperm[E:] = E + np.argsort(ps, kind="stable")
            batch[N:] = G
            gptr[G + 1:] = Np
            sidx[G:] = 0
        cnt = np.bincount(dst, minlength=Np)
        rowptr[0] = 0
        np.cumsum(cnt, out=rowptr[1:])
        scnt = np.bincount(src, minlength=Np)
        srowptr[0] = 0
        np.cumsum(scnt, out=srowptr[1:])
        if lay.attn_scope == "batch":
            aseg_id[:N] = 0
            aseg_id[N:] = 1
            aseg_ptr[:] = (0, N, Np)
        else:
            aseg_id[:] = batch
            aseg_ptr[:] = gptr
        scal[:] = (N, G, E, 0)
        return out

    def _slot(self, n, ring=4):
        cuda = self.device.type == "cuda"
        if len(self._ring) < ring:
            self._ring.append([None, None])
            slot = self._ring[-1]
        else:
            slot = self._ring[self._ring_pos % ring]
            self._ring_pos += 1
        if slot[1] is not None:
            t0 = time.perf_counter()
            slot[1].synchronize()  # the async copy that last read this pinned buffer is done
            self.slot_wait_s += time.perf_counter() - t0
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(max(n, 1 << 16), dtype=torch.int32, pin_memory=cuda)
        slot[1] = torch.cuda.Event() if cuda else None
        return slot

    def upload(self, indices, lay, dev_buf=None):
        """plan() into a pinned buffer and copy it (async) to ``dev_buf`` (or a new device tensor)."""
        slot = self._slot(lay.total)
        host = slot[0][:lay.total]
        t0 = time.perf_counter()
        self.plan(indices, lay, host.numpy())
        t1 = time.perf_counter()
        if self.device.type == "cuda":
            if dev_buf is None:
                dev_buf = host.to(self.device, non_blocking=True)
            else:
                dev_buf[:lay.total].copy_(host, non_blocking=True)
            slot[1].record()
        else:
            if dev_buf is None:
                dev_buf = host.clone()
            else:
                dev_buf[:lay.total].copy_(host)
        ph = self.phase_s
        ph["plan"] = ph.get("plan", 0.0) + (t1 - t0)
        ph["copy"] = ph.get("copy", 0.0) + (time.perf_counter() - t1)
        return dev_buf

    # ------------------------------------------------------------------ device side
    def _assemble_native(self, dev_buf, lay):
        """One HIP launch (``csrc/assemble.hip``) for every per-batch tensor."""
        from .. import _native

        offs, o = [], 0
        for sz in lay.sizes:
            offs.append(o)
            o += sz
        th = [(ih, t) for ih, t in enumerate(self.head_types or [])]
        node_t = [ih for ih, t in th if t != "graph" and ih in self.targets_node]
        graph_t = [ih for ih, t in th if t == "graph" and ih in self.targets_graph]
        node_src = [self.fields[k] for k in self.node_keys] + [self.targets_node[ih] for ih in node_t]
        edge_src = [self.fields[k] for k in self.edge_keys]
        graph_src = [self.fields[k] for k in self.graph_keys] + [self.targets_graph[ih] for ih in graph_t]
        pos_field = self.node_keys.index("pos") if (lay.padded and "pos" in self.node_keys) else -1
        outs = _native.ops().store_assemble(dev_buf, lay.Np, lay.Ep, lay.Gp, lay.padded, offs, node_src, edge_src,
                                            graph_src, pos_field)
        nn_, ne, ng = len(node_src), len(edge_src), len(graph_src)
        fields = {}
        for k, t in zip(self.node_keys, outs[:len(self.node_keys)]):
            fields[k] = t
        tn = dict(zip(node_t, outs[len(self.node_keys):nn_]))
        for k, t in zip(self.edge_keys, outs[nn_:nn_ + ne]):
            fields[k] = t
        gout = outs[nn_ + ne:nn_ + ne + ng]
        for k, t in zip(self.graph_keys, gout[:len(self.graph_keys)]):
            fields[k] = t
        tg = dict(zip(graph_t, gout[len(self.graph_keys):]))
        targets = [tg[ih] if ih in tg else tn[ih] for ih, _ in th if ih in tg or ih in tn]
        edge_index, batch_l, ptr_l, nmask, gmask = outs[nn_ + ne + ng:]
        return fields, targets, edge_index, batch_l, ptr_l, nmask, gmask

    def assemble(self, dev_buf, lay, host_ids=None, branch_sorted=False):
        """Build a GraphBatch from a packed device plan (device ops only; graph-capturable).
        ``branch_sorted``: the sample indices were ordered by ``branch_order`` (graphs, and so
        nodes, grouped by branch id, padding last): enables branch-grouped decoding."""
        if dev_buf.is_cuda:
            views = []
            o = 0
            for sz in lay.sizes:
                views.append(dev_buf[o:o + sz])
                o += sz
            (_, _, src, dst, sperm, rowptr, srowptr, batch, gptr, aseg_id, aseg_ptr, _, scal) = views
            fields, targets, edge_index, batch_l, ptr_l, nmask, gmask = self._assemble_native(dev_buf, lay)
            b = GraphBatch(**fields)
            s = b._store
            s["edge_index"] = edge_index
            s["num_nodes"] = lay.Np
            s["num_graphs"] = lay.Gp
            s["batch"] = batch_l
            s["ptr"] = ptr_l
            s["dst_si"] = SegIndex(dst, rowptr, None, lay.Np)
            s["src_si"] = SegIndex(src, srowptr, sperm, lay.Np)
            s["graph_si"] = SegIndex(batch, gptr, None, lay.Gp)
            s["attn_seg_id"] = aseg_id
            s["attn_seg_ptr"] = aseg_ptr
            s["targets"] = targets
            if lay.padded:
                s["num_valid"] = scal[0]
                s["max_graph_nodes"] = self.max_graph_nodes
                s["graph_mask"] = gmask
                s["node_mask"] = nmask
                s["triplet_cap"] = functools.partial(self.triplet_cap, lay.Gp - 1, lay.Ep)  # host int, computed on demand
            self._branch_fields(s, views[11], gmask if lay.padded else None, host_ids, branch_sorted)
            return b
        return self._assemble_torch(dev_buf, lay, host_ids, branch_sorted)

    def _branch_fields(self, s, sidx, gmask, host_ids, branch_sorted):
        """Multi-branch batches: per-graph dataset ids (-1 on padding graphs), two launches."""
        if self.dataset_name is None:
            return
        dn = self.dataset_name_dev.index_select(0, sidx)
        if gmask is not None:
            dn = torch.where(gmask, dn, -1)
        s["dataset_name"] = dn.view(-1, 1)
        s["branch_sorted"] = bool(branch_sorted)
        if host_ids is not None:
            s["dataset_ids_host"] = host_ids

    def _assemble_torch(self, dev_buf, lay, host_ids=None, branch_sorted=False):
        """Plain-torch assembly: the CPU path, multi-branch batches, and the oracle of the
        native kernel's tests."""
        views = []
        o = 0
        for sz in lay.sizes:
            views.append(dev_buf[o:o + sz])
            o += sz
        (node_rows, erows, src, dst, sperm, rowptr, srowptr, batch, gptr, aseg_id, aseg_ptr, sidx, scal) = views
        Np, Ep, Gp = lay.Np, lay.Ep, lay.Gp
        out = {}
        nrow = node_rows.clamp(min=0).long() if lay.padded else node_rows.long()
        erow = erows.clamp(min=0).long() if lay.padded else erows.long()
        sid = sidx.long()
        nvalid = scal[0]
        gvalid = scal[1]
        if lay.padded:
            nmask = (node_rows >= 0).unsqueeze(1)
            emask = (erows >= 0).unsqueeze(1)
        for k in self.node_keys:
            v = self.fields[k].index_select(0, nrow)
            if lay.padded:
                v = v * nmask.to(v.dtype)
                if k == "pos":
                    # padded nodes at distinct finite positions: padded edges never have zero length
                    r = torch.arange(Np, device=v.device, dtype=v.dtype) - nvalid.to(v.dtype)
                    padpos = torch.stack([2.0 * (r + 1.0), torch.zeros_like(r), torch.zeros_like(r)], 1)
                    v = v + padpos * (~nmask).to(v.dtype)
            out[k] = v
        for k in self.edge_keys:
            v = self.fields[k].index_select(0, erow)
            if lay.padded:
                v = v * emask.to(v.dtype)
            out[k] = v
        gmask = None
        if lay.padded:
            gmask = torch.arange(Gp, device=dev_buf.device) < gvalid
        for k in self.graph_keys:
            v = self.fields[k].index_select(0, sid)
            if lay.padded:
                v = v * gmask.view(-1, *([1] * (v.dim() - 1))).to(v.dtype)
            out[k] = v
        targets = []
        if self.head_types is not None:
            for ih, t in enumerate(self.head_types):
                if t == "graph" and ih in self.targets_graph:
                    v = self.targets_graph[ih].index_select(0, sid)
                    if lay.padded:
                        v = v * gmask.unsqueeze(1).to(v.dtype)
                    targets.append(v)
                elif ih in self.targets_node:
                    v = self.targets_node[ih].index_select(0, nrow)
                    if lay.padded:
                        v = v * nmask.to(v.dtype)
                    targets.append(v)
        b = GraphBatch(**out)
        s = b._store
        s["edge_index"] = torch.stack([src.long(), dst.long()], 0)
        s["num_nodes"] = Np
        s["num_graphs"] = Gp
        s["batch"] = batch.long()
        s["ptr"] = gptr.long()
        s["dst_si"] = SegIndex(dst, rowptr, None, Np)
        s["src_si"] = SegIndex(src, srowptr, sperm, Np)
        s["graph_si"] = SegIndex(batch, gptr, None, Gp)
        s["attn_seg_id"] = aseg_id
        s["attn_seg_ptr"] = aseg_ptr
        s["targets"] = targets
        if lay.padded:
            s["num_valid"] = nvalid
            s["max_graph_nodes"] = self.max_graph_nodes
            s["graph_mask"] = gmask
            s["node_mask"] = nmask.view(-1)
            s["triplet_cap"] = functools.partial(self.triplet_cap, lay.Gp - 1, lay.Ep)  # host int, computed on demand
        self._branch_fields(s, sid, gmask, host_ids, branch_sorted)
        return b

    def branch_order(self, indices):
        """Stable-sort a batch's sample indices by ``dataset_name`` and return
        (indices, [(ID, g0, g1)], [(ID, n0, n1)]): every branch's graphs (and their
        nodes) become one contiguous range, known on the host (multi-branch decode
        without masks / host syncs)."""
        idx = np.asarray(indices, dtype=np.int64)
        dn = self.dataset_name[idx]
        order = np.argsort(dn, kind="stable")
        idx, dn = idx[order], dn[order]
        nn_ = self.n_nodes[idx]
        gr, nr = [], []
        g0, n0 = 0, 0
        for ID in np.unique(dn):
            c = int((dn == ID).sum())
            m = int(nn_[g0:g0 + c].sum())
            gr.append((int(ID), g0, g0 + c))
            nr.append((int(ID), n0, n0 + m))
            g0, n0 = g0 + c, n0 + m
        return idx.tolist(), gr, nr

    def batch(self, indices, Np=None, Ep=None, Gp=None):
        host_ids, ranges = None, None
        if self.dataset_name is not None:
            indices, gr, nr = self.branch_order(indices)
            host_ids = [g[0] for g in gr]
            ranges = (gr, nr)
        lay = self.layout(indices, Np, Ep, Gp)
        dev = self.upload(indices, lay)
        b = self.assemble(dev, lay, host_ids, branch_sorted=True)
        if ranges is not None:
            b._store["branch_graph_ranges"], b._store["branch_node_ranges"] = ranges
        return b


def _ranges(starts, counts):
    """Concatenate arange(s, s+c) for every (s, c) without a Python loop."""
    counts = np.asarray(counts, dtype=np.int64)
    tot = int(counts.sum())
    if tot == 0:
        return np.zeros(0, dtype=np.int64)
    shift = np.asarray(starts, dtype=np.int64) - np.concatenate([[0], np.cumsum(counts)[:-1]])
    return np.repeat(shift, counts) + np.arange(tot, dtype=np.int64)
