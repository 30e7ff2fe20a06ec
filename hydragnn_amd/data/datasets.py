"""Dataset containers (reference ``hydragnn/utils/datasets/*``).

* :class:`AbstractBaseDataset` — ``get``/``len`` protocol, ``dataset_name`` branch id
  attached in ``__getitem__`` (``abstractbasedataset.py:6-60``; the reference's
  hard-coded 6-name map is the default, any map can be passed).
* :class:`SimplePickleWriter` / :class:`SimplePickleDataset` — one file per sample
  plus a ``<label>-meta`` file, optional sub-directories of ``nmax_persubdir``
  (``pickledataset.py:14-182``).  Same directory layout, but every file is a
  torch-serialised dict of tensors loaded with ``weights_only=True``: nothing in a
  dataset file can execute code on load.
* :class:`SerializedWriter` / :class:`SerializedDataset` — one file per split and
  rank (``serializeddataset.py:10-87``).
* :class:`ColumnarWriter` / :class:`ColumnarDataset` — the ADIOS2 replacement
  (``adiosdataset.py:91-976``, N15): per key ONE concatenated ``.npy`` array plus
  per-sample counts/offsets, memory-mapped on read (``preload``/``subset`` like
  ``AdiosDataset``).  ``AdiosWriter``/``AdiosDataset`` are aliases.
* :class:`DistDataset` — the DDStore replacement (``distdataset.py:22-183``, N14):
  each rank serialises its shard into a node-local POSIX shared-memory segment
  (C++ ``csrc/shm_store.cpp``); an index of (owner, offset, nbytes) is
  all-gathered once and any rank reads any sample by a memcpy from the owner's
  segment.  Single-node scope (the MI355X target: 8 GPUs share host memory).
"""
import atexit
import io
import json
import os

import numpy as np
import torch
import torch.distributed as dist

from .graph import Graph

DEFAULT_DATASET_IDS = {"ani1x": 0, "qm7x": 1, "mptrj": 2, "alexandria": 3, "transition1x": 4, "omat24": 5}


COMM_SELF = "self"  # the MPI.COMM_SELF analogue: a writer/reader used by one rank alone


def _rank_world(group=None):
    if group == COMM_SELF:
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _allgather_obj(obj, group=None):
    if group == COMM_SELF or not (dist.is_available() and dist.is_initialized()):
        return [obj]
    from ..parallel.distributed import host_group

    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group or host_group())
    return out


def _barrier(group=None):
    if group != COMM_SELF and dist.is_available() and dist.is_initialized():
        from ..parallel.distributed import host_group

        dist.barrier(group=group or host_group())


def sample_to_dict(data):
    return {k: v for k, v in data.items() if torch.is_tensor(v)}


def sample_to_bytes(data):
    buf = io.BytesIO()
    torch.save(sample_to_dict(data), buf)
    return buf.getvalue()


def sample_from_bytes(b):
    if isinstance(b, torch.Tensor):
        b = b.numpy().tobytes()
    return Graph(**torch.load(io.BytesIO(b), map_location="cpu", weights_only=True))


class AbstractBaseDataset(torch.utils.data.Dataset):
    """Base dataset: subclasses implement ``get(idx)`` and ``len()``."""

    dataset_name = None
    dataset_ids = DEFAULT_DATASET_IDS

    def __init__(self):
        super().__init__()
        self.dataset = []

    def get(self, idx):
        return self.dataset[idx]

    def len(self):
        return len(self.dataset)

    def apply(self, func):
        for d in self.dataset:
            func(d)

    def map(self, func):
        self.dataset = [func(d) for d in self.dataset]

    def __len__(self):
        return self.len()

    def __getitem__(self, idx):
        obj = self.get(idx)
        if self.dataset_name is not None:
            obj.dataset_name = torch.tensor([[self.dataset_ids[self.dataset_name]]])
        return obj

    def __iter__(self):
        for i in range(self.len()):
            yield self[i]


# ------------------------------------------------------------------------------ pickle layout
class SimplePickleWriter:
    def __init__(self, dataset, basedir, label="total", minmax_node_feature=None, minmax_graph_feature=None,
                 use_subdir=False, nmax_persubdir=10_000, comm=None, attrs=None):
        if not isinstance(dataset, list):
            raise TypeError("SimplePickleWriter expects a list of samples")
        rank, _ = _rank_world(comm)
        ns = _allgather_obj(len(dataset), comm)
        noffset, ntotal = sum(ns[:rank]), sum(ns)
        if rank == 0:
            os.makedirs(basedir, exist_ok=True)
            meta = {"minmax_node_feature": minmax_node_feature, "minmax_graph_feature": minmax_graph_feature,
                    "ntotal": ntotal, "use_subdir": use_subdir, "nmax_persubdir": nmax_persubdir,
                    "attrs": {k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in (attrs or {}).items()}}
            with open(os.path.join(basedir, f"{label}-meta.json"), "w") as f:
                json.dump(meta, f, default=lambda o: np.asarray(o).tolist())
        _barrier(comm)
        for i, data in enumerate(dataset):
            k = noffset + i
            d = os.path.join(basedir, str(k // nmax_persubdir)) if use_subdir else basedir
            os.makedirs(d, exist_ok=True)
            torch.save(sample_to_dict(data), os.path.join(d, f"{label}-{k}.pkl"))
        _barrier(comm)


class SimplePickleDataset(AbstractBaseDataset):
    def __init__(self, basedir, label, subset=None, preload=False, var_config=None):
        super().__init__()
        self.basedir, self.label, self.var_config = basedir, label, var_config
        with open(os.path.join(basedir, f"{label}-meta.json")) as f:
            meta = json.load(f)
        self.minmax_node_feature = meta["minmax_node_feature"]
        self.minmax_graph_feature = meta["minmax_graph_feature"]
        self.ntotal = meta["ntotal"]
        self.use_subdir = meta["use_subdir"]
        self.nmax_persubdir = meta["nmax_persubdir"]
        for k, v in meta["attrs"].items():  # e.g. pna_deg
            setattr(self, k, torch.tensor(v) if isinstance(v, list) else v)
        self.subset = list(range(self.ntotal)) if subset is None else list(subset)
        self.preload = preload
        if preload:
            self.dataset = [self.read(k) for k in self.subset]

    def len(self):
        return len(self.subset)

    def setsubset(self, subset):
        self.subset = list(subset)

    def read(self, k):
        d = os.path.join(self.basedir, str(k // self.nmax_persubdir)) if self.use_subdir else self.basedir
        s = Graph(**torch.load(os.path.join(d, f"{self.label}-{k}.pkl"), map_location="cpu", weights_only=True))
        return self.update_data_object(s)

    def get(self, i):
        return self.dataset[i] if self.preload else self.read(self.subset[i])

    def update_data_object(self, data):
        """Optional input-feature column selection (``var_config["input_node_features"]``)."""
        if self.var_config is not None and "input_node_features" in self.var_config and data.get("x") is not None:
            data.x = data.x[:, self.var_config["input_node_features"]]
        return data


# ------------------------------------------------------------------------------ per-split serialized
class SerializedWriter:
    """One torch-serialised file per split (and per rank when ``dist``):
    ``<basedir>/<datasetname>-<label>[-<rank>].pt``."""

    def __init__(self, dataset, basedir, datasetname, label="total", minmax_node_feature=None,
                 minmax_graph_feature=None, dist=False):
        from .serialized import write_serialized

        rank, _ = _rank_world()
        suffix = f"-{rank}" if dist else ""
        write_serialized(os.path.join(basedir, f"{datasetname}-{label}{suffix}.pt"), list(dataset),
                         minmax_node_feature, minmax_graph_feature)


class SerializedDataset(AbstractBaseDataset):
    def __init__(self, basedir, datasetname, label, dist=False):
        from .serialized import read_serialized

        super().__init__()
        rank, _ = _rank_world()
        suffix = f"-{rank}" if dist else ""
        self.minmax_node_feature, self.minmax_graph_feature, self.dataset = read_serialized(
            os.path.join(basedir, f"{datasetname}-{label}{suffix}.pt"))


# ------------------------------------------------------------------------------ columnar (ADIOS2 replacement)
class ColumnarWriter:
    """``ColumnarWriter(path)``; ``add(label, samples)`` (any number of times, any rank);
    ``add_global(name, array)``; ``save()``.  Layout: ``<path>/<label>/<key>.npy``
    (all samples' rows concatenated), ``<key>.count.npy`` (rows per sample) and
    ``meta.json`` ({keys, dtypes, trailing shapes, ntotal}); globals in ``<path>/globals``."""

    def __init__(self, filename, comm=None):
        self.path = filename
        self.comm = comm
        self.data = {}
        self.globals = {}

    def add_global(self, vname, arr):
        self.globals[vname] = np.asarray(arr)

    def add(self, label, data):
        self.data.setdefault(label, []).extend(data if isinstance(data, list) else [data])

    def save(self):
        rank, world = _rank_world(self.comm)
        for label, samples in self.data.items():
            shard = [sample_to_dict(s) for s in samples]
            allsh = _allgather_obj(len(shard), self.comm)
            # rank-ordered concatenation: every rank writes its own part file, rank 0 merges
            d = os.path.join(self.path, label)
            os.makedirs(d, exist_ok=True)
            keys = sorted({k for s in shard for k in s})
            keys = sorted(set().union(*_allgather_obj(keys, self.comm)))
            part = {}
            for k in keys:
                rows = [s[k].numpy() if k in s else None for s in shard]
                if any(r is None for r in rows):
                    continue
                nd = max([r.ndim for r in rows] + [1])
                shp = np.asarray([list(r.shape) + [1] * (nd - r.ndim) for r in rows], dtype=np.int64).reshape(-1, nd)
                cnt = np.asarray([r.size for r in rows], dtype=np.int64)
                arr = np.concatenate([r.reshape(-1) for r in rows]) if rows else np.zeros((0,), dtype=np.float32)
                part[k] = (arr, cnt, shp)
            np.savez(os.path.join(d, f"part-{rank}.npz"), **{k: v[0] for k, v in part.items()},
                     **{f"{k}.count": v[1] for k, v in part.items()}, **{f"{k}.shape": v[2] for k, v in part.items()})
            _barrier(self.comm)
            if rank == 0:
                parts = [np.load(os.path.join(d, f"part-{r}.npz")) for r in range(world)]
                meta = {"ntotal": int(sum(allsh)), "keys": {}}
                for k in keys:
                    if not all(k in p for p in parts):
                        continue
                    arr = np.concatenate([p[k] for p in parts])
                    np.save(os.path.join(d, f"{k}.npy"), arr)
                    np.save(os.path.join(d, f"{k}.count.npy"), np.concatenate([p[f"{k}.count"] for p in parts]))
                    np.save(os.path.join(d, f"{k}.shape.npy"), np.concatenate([p[f"{k}.shape"] for p in parts]))
                    meta["keys"][k] = {"dtype": str(arr.dtype)}
                with open(os.path.join(d, "meta.json"), "w") as f:
                    json.dump(meta, f)
                for r in range(world):
                    os.remove(os.path.join(d, f"part-{r}.npz"))
            _barrier(self.comm)
        if rank == 0 and self.globals:
            g = os.path.join(self.path, "globals")
            os.makedirs(g, exist_ok=True)
            for k, v in self.globals.items():
                np.save(os.path.join(g, f"{k}.npy"), v)
        _barrier(self.comm)


class ColumnarDataset(AbstractBaseDataset):
    """Memory-mapped reader of a :class:`ColumnarWriter` store (``AdiosDataset`` API subset:
    ``preload``, ``subset_istart/iend``, ``keys``, ``setsubset``, globals as attributes)."""

    def __init__(self, filename, label, comm=None, preload=False, var_config=None, subset_istart=None,
                 subset_iend=None, keys=None, **_unused):
        super().__init__()
        self.path, self.label, self.var_config = filename, label, var_config
        d = os.path.join(filename, label)
        with open(os.path.join(d, "meta.json")) as f:
            meta = json.load(f)
        self.ntotal = meta["ntotal"]
        self.keys = [k for k in meta["keys"] if keys is None or k in keys]
        self.arr, self.off, self.shape = {}, {}, {}
        for k in self.keys:
            self.arr[k] = np.load(os.path.join(d, f"{k}.npy"), mmap_mode=None if preload else "r")
            cnt = np.load(os.path.join(d, f"{k}.count.npy"))
            self.off[k] = np.concatenate([[0], np.cumsum(cnt)])
            self.shape[k] = np.load(os.path.join(d, f"{k}.shape.npy"))
        g = os.path.join(filename, "globals")
        if os.path.isdir(g):
            for fn in os.listdir(g):
                setattr(self, fn[:-4], torch.from_numpy(np.load(os.path.join(g, fn))))
        self.setsubset(subset_istart, subset_iend)

    def setsubset(self, subset_istart=None, subset_iend=None, preload=False):
        a = 0 if subset_istart is None else subset_istart
        b = self.ntotal if subset_iend is None else subset_iend
        self.subset = range(a, b)

    def len(self):
        return len(self.subset)

    def get(self, i):
        k0 = self.subset[i]
        s = {}
        for k in self.keys:
            o0, o1 = self.off[k][k0], self.off[k][k0 + 1]
            s[k] = torch.from_numpy(np.array(self.arr[k][o0:o1]).reshape(tuple(self.shape[k][k0])))
        g = Graph(**s)
        if self.var_config is not None and "input_node_features" in self.var_config and g.get("x") is not None:
            g.x = g.x[:, self.var_config["input_node_features"]]
        return g


AdiosWriter = ColumnarWriter
AdiosDataset = ColumnarDataset


# ------------------------------------------------------------------------------ DDStore replacement
_OWNED_SEGMENTS = []


@atexit.register
def _cleanup_segments():
    from .. import _native

    if _OWNED_SEGMENTS and _native.load():
        for name in _OWNED_SEGMENTS:
            _native.ops().shm_store_unlink(name)


class DistDataset(AbstractBaseDataset):
    """``DistDataset(data, label, comm=None, ddstore_width=None, local=False)``.

    ``data``: this rank's local shard (list of samples).  After construction every
    rank can ``get`` any global index: local hits are served from the segment of the
    rank itself, remote ones by a read-only mapping of the owner's segment.
    ``ddstore_width`` splits the world into independent stores of that many ranks
    (reference ``distdataset.py:43``)."""

    def __init__(self, data, label, comm=None, ddstore_width=None, local=False, var_config=None, tag=None):
        super().__init__()
        from .. import _native

        self.ops = _native.ops()
        self.label, self.var_config = label, var_config
        rank, world = _rank_world(comm)
        width = ddstore_width or world
        self.store_id = rank // width
        blobs = [sample_to_bytes(s) for s in data]
        sizes = np.asarray([len(b) for b in blobs], dtype=np.int64)
        offs = np.concatenate([[0], np.cumsum(sizes)]) if len(sizes) else np.zeros(1, dtype=np.int64)
        tag = tag or f"{os.getpid() if world == 1 else _allgather_obj(os.getpid(), comm)[0]}"
        self.segname = f"hydra_dd_{tag}_{label}_{rank}"
        self.h_local = self.ops.shm_store_create(self.segname, int(offs[-1]))
        _OWNED_SEGMENTS.append(self.segname)
        for b, o in zip(blobs, offs[:-1]):
            self.ops.shm_store_write(self.h_local, int(o), torch.frombuffer(bytearray(b), dtype=torch.uint8))
        entries = _allgather_obj((rank, self.segname, offs[:-1].tolist(), sizes.tolist()), comm)
        _barrier(comm)
        # global index over the ranks of this store (rank order), like DDStore's
        self.index = []
        for r, name, o, s in entries:
            if r // width != self.store_id:
                continue
            self.index.extend((name, oo, ss) for oo, ss in zip(o, s))
        self.handles = {self.segname: self.h_local}
        self.local = local

    def len(self):
        return len(self.index)

    def _handle(self, name):
        h = self.handles.get(name)
        if h is None:
            h = self.ops.shm_store_attach(name)
            self.handles[name] = h
        return h

    def get(self, idx):
        name, off, nb = self.index[idx]
        s = sample_from_bytes(self.ops.shm_store_read(self._handle(name), int(off), int(nb)))
        if self.var_config is not None and "input_node_features" in self.var_config and s.get("x") is not None:
            s.x = s.x[:, self.var_config["input_node_features"]]
        return s

    def epoch_begin(self):
        """Start of a data epoch (reference DDStore ``epoch_begin``: opens the MPI one-sided
        access epoch).  Shared-memory segments need no fence; remote segments are mapped
        lazily on first access."""
        self.epochs = getattr(self, "epochs", 0) + 1

    def epoch_end(self):
        """End of a data epoch (DDStore ``epoch_end``): unmap the other ranks' segments so
        the mappings (and their page-cache residency in this process) do not accumulate
        across epochs; the local segment stays."""
        for name in [n for n in self.handles if n != self.segname]:
            self.ops.shm_store_close(self.handles.pop(name))

    def close(self):
        for name, h in list(self.handles.items()):
            self.ops.shm_store_close(h)
        self.handles = {}
        if self.segname in _OWNED_SEGMENTS:
            self.ops.shm_store_unlink(self.segname)
            _OWNED_SEGMENTS.remove(self.segname)


# ------------------------------------------------------------------------------ raw datasets (P35)
class AbstractRawDataset(AbstractBaseDataset):
    """In-memory raw dataset (``abstractrawdataset.py:29-405``): read every raw file of
    ``config["Dataset"]["path"]`` with the format reader, scale ``*_scaled_num_nodes``
    features, min-max normalise (all ranks), then build edges / descriptors / PE and pack
    targets exactly like the serialized pipeline (``SerializedDataLoader.process``)."""

    format = None

    def __init__(self, config, dist=False, sampling=None):
        super().__init__()
        from .lsms import RawDataLoader
        from .serialized import SerializedDataLoader

        ds = dict(config["Dataset"])
        if self.format is not None:
            ds["format"] = self.format
        loader = RawDataLoader(ds, dist=dist)
        self._collect(loader)
        loader.normalize_dataset()
        self.minmax_node_feature = loader.minmax_node_feature
        self.minmax_graph_feature = loader.minmax_graph_feature
        proc = SerializedDataLoader(config, dist=dist)
        samples = [s for part in loader.dataset_list for s in part]
        if sampling is not None:
            rng = np.random.default_rng(0)
            samples = [samples[i] for i in sorted(rng.choice(len(samples), int(len(samples) * sampling),
                                                             replace=False))]
        self.dataset = proc.process(samples)

    @classmethod
    def from_samples(cls, samples, config, dist=False):
        """Raw samples already in memory (a generator's output: ``x`` = all node feature
        columns, ``y`` = all graph feature columns, ``pos``) -> the same normalise + process
        pipeline as raw files (the reference's in-script ``transform_input_to_data_object_base``
        datasets, e.g. ``examples/ising_model/train_ising.py``).  With ``dist`` each rank
        passes its own shard and the min/max normalisation is reduced over ranks."""
        from .lsms import RawDataLoader
        from .serialized import SerializedDataLoader

        self = cls.__new__(cls)
        AbstractBaseDataset.__init__(self)
        ds = dict(config["Dataset"])
        ds.setdefault("format", "unit_test")
        ds.setdefault("path", {})
        loader = RawDataLoader(ds, dist=dist)
        loader.dataset_list = [loader.scale_features_by_num_nodes(list(samples))]
        loader.normalize_dataset()
        self.minmax_node_feature = loader.minmax_node_feature
        self.minmax_graph_feature = loader.minmax_graph_feature
        self.dataset = SerializedDataLoader(config, dist=dist).process(loader.dataset_list[0])
        return self

    @staticmethod
    def _collect(loader):
        for split, raw_path in loader.path_dictionary.items():
            files = sorted(f for f in os.listdir(raw_path) if f != ".DS_Store")
            ds = [loader._read(os.path.join(raw_path, f)) for f in files
                  if os.path.isfile(os.path.join(raw_path, f))]
            ds = [d for d in ds if d is not None]
            loader.dataset_list.append(loader.scale_features_by_num_nodes(ds))
            loader.serial_data_name_list.append(split)


class LSMSDataset(AbstractRawDataset):
    format = "LSMS"


class CFGDataset(AbstractRawDataset):
    format = "CFG"


class XYZDataset(AbstractRawDataset):
    format = "XYZ"
