"""Host-native batch assembly (csrc/collate.cpp) against the plain torch path it replaces:
offset-concatenated edge_index, dst/src CSR row pointers and the stable src permutation."""
import pytest
import torch

from hydragnn_amd import _native
from hydragnn_amd.data.graph import Graph, collate

pytestmark = pytest.mark.skipif(not _native.available(), reason="native library not built")


def _samples(G=48, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(G):
        n = int(torch.randint(1, 30, (1,), generator=g))
        e = int(torch.randint(0, 120, (1,), generator=g))
        ei = torch.randint(0, n, (2, e), generator=g)
        out.append(Graph(x=torch.randn(n, 3, generator=g), edge_index=ei, edge_attr=torch.randn(e, 2, generator=g)))
    return out


def test_native_collate_matches_torch():
    b = collate(_samples())
    ei, N = b.edge_index, b.num_nodes
    src, dst = ei[0], ei[1]
    ptr = b.ptr
    # every edge stays inside its own graph and the batch is dst-sorted
    gs, gd = b.batch[src], b.batch[dst]
    assert torch.equal(gs, gd)
    assert bool((dst[1:] >= dst[:-1]).all())
    assert int(ei.min()) >= 0 and int(ei.max()) < int(ptr[-1])
    rp = torch.zeros(N + 1, dtype=torch.int32)
    rp[1:] = torch.cumsum(torch.bincount(dst, minlength=N), 0)
    srp = torch.zeros(N + 1, dtype=torch.int32)
    srp[1:] = torch.cumsum(torch.bincount(src, minlength=N), 0)
    assert torch.equal(b.dst_si.rowptr, rp)
    assert torch.equal(b.src_si.rowptr, srp)
    assert torch.equal(b.src_si.perm, torch.argsort(src, stable=True).to(torch.int32))


def test_native_collate_edges_offsets_and_bounds():
    ops = _native.ops()
    e0 = torch.tensor([[0, 1], [1, 0]])
    e1 = torch.tensor([[2], [0]])
    out = ops.collate_edges([e0, e1], torch.tensor([2, 3]))
    assert out.tolist() == [[0, 1, 4], [1, 0, 2]]
    with pytest.raises(RuntimeError, match="outside"):
        ops.collate_edges([torch.tensor([[0], [5]])], torch.tensor([2]))
    with pytest.raises(RuntimeError, match="outside"):
        ops.csr_from_edges(torch.tensor([0]), torch.tensor([3]), 2)


def test_native_collate_empty_edges():
    gs = [Graph(x=torch.randn(3, 2), edge_index=torch.zeros(2, 0, dtype=torch.long)) for _ in range(3)]
    b = collate(gs)
    assert b.edge_index.shape == (2, 0)
    assert b.dst_si.rowptr.tolist() == [0] * 10
    assert b.src_si.perm.numel() == 0
