"""Dataset containers (reference ``hydragnn/utils/datasets/*`` and
``tests/test_datasetclass_inheritance.py``): pickle layout round trip (incl. subdirs and
attrs such as ``pna_deg``), per-split serialized files, the columnar (ADIOS2-free)
mmap store, the shared-memory DistDataset (DDStore replacement, native C++ segment
store) on 1 and 2 ranks, and an LSMS raw dataset feeding a training run."""
import os

import pytest
import torch

from hydragnn_amd.data.datasets import (ColumnarDataset, ColumnarWriter, DistDataset, LSMSDataset, SerializedDataset,
                                        SerializedWriter, SimplePickleDataset, SimplePickleWriter)
from hydragnn_amd.data.synthetic import oc20_like
from test_distributed import run_ranks


def _same(a, b):
    assert set(k for k, v in a.items() if torch.is_tensor(v)) == set(k for k, v in b.items() if torch.is_tensor(v))
    for k, v in a.items():
        if torch.is_tensor(v):
            assert torch.equal(v, b[k]), k


def _samples(n=7, seed=0):
    return oc20_like(n, seed=seed, min_atoms=5, max_atoms=12, radius=5.0, max_neighbours=6, pe_dim=2)


@pytest.mark.parametrize("use_subdir", [False, True])
def test_pickle_roundtrip(tmp_path, use_subdir):
    s = _samples()
    SimplePickleWriter(s, str(tmp_path), "trainset", use_subdir=use_subdir, nmax_persubdir=3,
                       attrs={"pna_deg": torch.tensor([0, 3, 5])})
    ds = SimplePickleDataset(str(tmp_path), "trainset")
    assert len(ds) == 7 and ds.pna_deg.tolist() == [0, 3, 5]
    for a, b in zip(s, ds):
        _same(a, b)
    ds2 = SimplePickleDataset(str(tmp_path), "trainset", subset=[2, 5], preload=True,
                              var_config={"input_node_features": [0]})
    assert len(ds2) == 2 and ds2[1].x.shape[1] == 1


def test_serialized_writer_dataset(tmp_path):
    s = _samples()
    SerializedWriter(s, str(tmp_path), "oc", "valset")
    ds = SerializedDataset(str(tmp_path), "oc", "valset")
    for a, b in zip(s, ds):
        _same(a, b)


def test_columnar_store(tmp_path):
    s = _samples(9)
    w = ColumnarWriter(str(tmp_path / "store"))
    w.add("trainset", s[:6])
    w.add("trainset", s[6:])
    w.add_global("pna_deg", [1, 2, 3])
    w.save()
    ds = ColumnarDataset(str(tmp_path / "store"), "trainset")
    assert len(ds) == 9 and ds.pna_deg.tolist() == [1, 2, 3]
    for a, b in zip(s, ds):
        _same(a, b)
    ds.setsubset(3, 5)
    assert len(ds) == 2
    _same(ds[0], s[3])


def test_dist_dataset_single_rank():
    s = _samples(5)
    dd = DistDataset(s, "unit", tag="t1")
    assert len(dd) == 5
    for a, b in zip(s, dd):
        _same(a, b)
    dd.close()


def _dd_body(rank, world):
    s = _samples(3 + rank, seed=rank)
    dd = DistDataset(s, "two", tag="t2")
    assert len(dd) == 3 + 4
    mine = list(range(0, 3)) if rank == 0 else list(range(3, 7))
    other = list(range(3, 7)) if rank == 0 else list(range(0, 3))
    for k, i in enumerate(mine):
        _same(dd[i], s[k])
    ref = _samples(4 if rank == 0 else 3, seed=1 - rank)
    for k, i in enumerate(other):
        _same(dd[i], ref[k])  # remote gets through the owner's shm segment
    torch.distributed.barrier()
    dd.close()


def test_dist_dataset_two_ranks():
    run_ranks("test_datasets:_dd_body")


def test_lsms_raw_dataset(tmp_path):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    from ci_configs import ci
    from hydragnn_amd.data.lsms import deterministic_graph_data

    raw = tmp_path / "raw"
    deterministic_graph_data(str(raw), number_configurations=20, seed=3)
    cfg = ci("ci")
    cfg["Dataset"]["path"] = {"total": str(raw)}
    ds = LSMSDataset(cfg)
    assert len(ds) == 20
    d = ds[0]
    assert d.edge_index.shape[0] == 2 and d.y.shape[1] == 1 and d.x.shape[1] == 1
    assert float(d.edge_attr.max()) <= 1.0 + 1e-6
