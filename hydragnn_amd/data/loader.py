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
        if self.num_workers == 0:
            for b in self._batches():
                yield self._make(b)
            return
        q = queue.Queue(maxsize=self.prefetch)
        stop = object()

        def worker(chunks):
            for b in chunks:
                q.put(self._make(b))
            q.put(stop)

        batches = list(self._batches())
        t = threading.Thread(target=worker, args=(batches,), daemon=True)
        t.start()
        while True:
            item = q.get()
            if item is stop:
                break
            yield item
        t.join()


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
