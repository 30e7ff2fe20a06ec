"""Mini-batch loaders (reference ``preprocess/load_data.py:93-326``).

``GraphDataLoader``: host path — sampler (DistributedSampler / RandomSampler /
shuffle, same semantics as the reference ``create_dataloaders``) -> CSR-ready
collation (``data.graph.collate``) in a background prefetch thread -> pinned
memory.  ``HYDRAGNN_NUM_WORKERS`` sets the number of collation threads
(reference env var).

``DeviceGraphLoader``: MI355X fast path — the whole split lives in HBM
(``DeviceGraphStore``); each batch is assembled on the GPU from index lists,
with per-head targets precomputed (no host ``get_head_indices``).
Both yield objects with the same attribute interface (``GraphBatch``).
"""
import os
import queue
import threading

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DistributedSampler, RandomSampler

from .graph import collate


class _ShuffleSampler:
    def __init__(self, n, shuffle=True, seed=0):
        self.n, self.shuffle, self.seed, self.epoch = n, shuffle, seed, 0

    def set_epoch(self, e):
        self.epoch = e

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            return iter(torch.randperm(self.n, generator=g).tolist())
        return iter(range(self.n))

    def __len__(self):
        return self.n


def make_sampler(dataset, shuffle=True, group=None, oversampling=False, num_samples=None):
    n = len(dataset)
    if dist.is_available() and dist.is_initialized():
        if oversampling:
            assert num_samples is not None
            return RandomSampler(range(n), replacement=False, num_samples=num_samples)
        group = group or dist.group.WORLD
        return DistributedSampler(range(n), num_replicas=dist.get_world_size(group), rank=dist.get_rank(group),
                                  shuffle=shuffle)
    return _ShuffleSampler(n, shuffle)


class GraphDataLoader:
    def __init__(self, dataset, batch_size=32, shuffle=True, sampler=None, num_workers=None, pin_memory=True,
                 drop_last=False, prefetch=4, group=None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = sampler if sampler is not None else make_sampler(dataset, shuffle, group)
        nw = num_workers if num_workers is not None else int(os.environ.get("HYDRAGNN_NUM_WORKERS", "0"))
        self.num_workers = max(nw, 0)
        self.pin_memory = pin_memory and torch.cuda.is_available()
        self.drop_last = drop_last
        self.prefetch = prefetch

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _batches(self):
        idx = list(iter(self.sampler))
        for i in range(0, len(idx), self.batch_size):
            b = idx[i:i + self.batch_size]
            if self.drop_last and len(b) < self.batch_size:
                break
            yield b

    def _make(self, b):
        batch = collate([self.dataset[j].clone() for j in b])
        if self.pin_memory:
            batch.pin_memory()
        return batch

    def __iter__(self):
        nw = self.num_workers
        if nw == 0 and os.environ.get("HYDRAGNN_CUSTOM_DATALOADER", "0") == "1":
            nw = 1  # the reference's HydraDataLoader: threaded prefetch even without workers
        if nw == 0:
            for b in self._batches():
                yield self._make(b)
            return
        # nw collate threads, worker w builds batches w, w + nw, ...; consumed in order
        batches = list(self._batches())
        qs = [queue.Queue(maxsize=max(1, self.prefetch // nw + 1)) for _ in range(nw)]

        def worker(w):
            apply_worker_affinity(w)
            for k in range(w, len(batches), nw):
                qs[w].put(self._make(batches[k]))

        ts = [threading.Thread(target=worker, args=(w,), daemon=True) for w in range(nw)]
        for t in ts:
            t.start()
        for k in range(len(batches)):
            yield qs[k % nw].get()
        for t in ts:
            t.join()


def parse_omp_places(places):
    """CPU list of an ``OMP_PLACES`` string such as ``{0:4},{8:4}`` or ``{0,1,2},{5}``."""
    cpus = []
    for part in (places or "").replace("},", "}|").split("|"):
        part = part.strip().strip("{}")
        if not part:
            continue
        if ":" in part:
            start, n = part.split(":")[:2]
            cpus += list(range(int(start), int(start) + int(n)))
        else:
            cpus += [int(c) for c in part.split(",") if c.strip()]
    return cpus


def apply_worker_affinity(wid):
    """Pin the calling loader thread to its core window (reference ``HydraDataLoader.worker_init``,
    ``load_data.py:118-150``): ``HYDRAGNN_AFFINITY_WIDTH`` cores (default 2) starting at
    ``HYDRAGNN_AFFINITY_OFFSET + width * wid`` of the process's allowed set (or of
    ``OMP_PLACES`` with ``HYDRAGNN_AFFINITY=OMP``).  Only when HYDRAGNN_AFFINITY is set;
    returns the applied set (None when unchanged)."""
    mode = os.environ.get("HYDRAGNN_AFFINITY")
    if mode is None or not hasattr(os, "sched_setaffinity"):
        return None
    width = int(os.environ.get("HYDRAGNN_AFFINITY_WIDTH", "2"))
    offset = int(os.environ.get("HYDRAGNN_AFFINITY_OFFSET", "0"))
    cpus = parse_omp_places(os.environ.get("OMP_PLACES")) if mode == "OMP" else sorted(os.sched_getaffinity(0))
    mask = set(cpus[width * wid + offset:width * (wid + 1) + offset])
    if not mask:
        return None
    os.sched_setaffinity(0, mask)  # tid 0 = this thread
    return mask


class DeviceGraphLoader:
    """Iterates device-assembled batches of an HBM-resident split."""

    def __init__(self, dataset, store, batch_size=32, shuffle=True, sampler=None, group=None, drop_last=False,
                 pad=None):
        self.dataset = dataset
        self.store = store
        self.batch_size = batch_size
        self.sampler = sampler if sampler is not None else make_sampler(dataset, shuffle, group)
        self.drop_last = drop_last
        self.pad = pad

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def index_batches(self):
        idx = list(iter(self.sampler))
        for i in range(0, len(idx), self.batch_size):
            b = idx[i:i + self.batch_size]
            if self.drop_last and len(b) < self.batch_size:
                break
            yield b

    def __iter__(self):
        for b in self.index_batches():
            yield self.store.batch(b)
