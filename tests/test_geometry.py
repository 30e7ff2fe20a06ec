"""Geometry / graph-construction tests (reference ``tests/test_periodic_boundary_conditions.py``
and ``tests/test_rotational_invariance.py``):

* periodic radius graph: H2 in a 3 A box -> 1 neighbour per atom (2 with self loops);
  BCC Cr 5x5x5 supercell (a = 3.6 A) at r = 5 A -> 14 neighbours (15); every
  ``|pos[dst] - pos[src] + shift| <= r``;
* the radius graph and edge lengths are invariant under ``normalize_rotation``;
* HIP builders (``csrc/graph.hip``, GPU-marked): radius graph (index / nearest cap,
  periodic) and DimeNet triplets == the CPU reference implementations.
"""
import numpy as np
import pytest
import torch

from hydragnn_amd.data.transforms import normalize_rotation, radius_graph, radius_graph_pbc


def _bcc_cr(n=5, a=3.6):
    basis = np.array([[0, 0, 0], [0.5, 0.5, 0.5]])
    g = np.stack(np.meshgrid(*[np.arange(n)] * 3, indexing="ij"), -1).reshape(-1, 3)
    pos = ((g[:, None, :] + basis[None]) * a).reshape(-1, 3)
    return torch.tensor(pos, dtype=torch.float64), torch.eye(3, dtype=torch.float64) * a * n


def _check_pbc(pos, cell, r, per_atom, per_atom_loops):
    n = pos.shape[0]
    ei, sh = radius_graph_pbc(pos, cell, [True] * 3, r, max_num_neighbors=100, loop=False)
    assert ei.shape[1] == per_atom * n
    ei2, _ = radius_graph_pbc(pos, cell, [True] * 3, r, max_num_neighbors=100, loop=True)
    assert ei2.shape[1] == per_atom_loops * n
    vec = pos[ei[1]] - pos[ei[0]] + sh.double()
    d = vec.norm(dim=-1)
    assert bool(((d <= r + 1e-6) & (d > 0)).all())


def test_periodic_h2():
    pos = torch.tensor([[1.0, 1.0, 1.0], [1.43, 1.43, 1.43]], dtype=torch.float64)
    _check_pbc(pos, torch.eye(3, dtype=torch.float64) * 3.0, 1.0, 1, 2)


def test_periodic_bcc_large():
    pos, cell = _bcc_cr()
    _check_pbc(pos, cell, 5.0, 14, 15)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.float64, 1e-12)])
def test_rotational_invariance(dtype, tol):
    torch.manual_seed(0)
    pos = torch.rand(30, 3, dtype=dtype) * 4
    q, _ = torch.linalg.qr(torch.randn(3, 3, dtype=torch.float64))
    rot = pos @ q.to(dtype).T
    a, b = normalize_rotation(pos), normalize_rotation(rot)
    ea = radius_graph(a, 1.5, max_num_neighbors=100)
    eb = radius_graph(b, 1.5, max_num_neighbors=100)
    assert torch.equal(ea, eb)
    la = (a[ea[1]] - a[ea[0]]).norm(dim=-1)
    lb = (b[eb[1]] - b[eb[0]]).norm(dim=-1)
    assert float((la - lb).abs().max()) < tol


# ---------------------------------------------------------------------------- HIP builders
def _batch(seed=0, G=6):
    rng = np.random.default_rng(seed)
    pos, batch = [], []
    for g in range(G):
        n = int(rng.integers(5, 40))
        pos.append(torch.tensor(rng.uniform(0, 6, size=(n, 3)), dtype=torch.float32))
        batch.append(torch.full((n,), g))
    return torch.cat(pos), torch.cat(batch)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [4, 16, 1000])
def test_radius_graph_hip_index_policy(k):
    from hydragnn_amd.ops.radius import radius_edges

    pos, batch = _batch()
    ref = radius_edges(pos, batch, 2.5, k)  # CPU torch path (torch_cluster semantics)
    out = radius_edges(pos.cuda(), batch.cuda(), 2.5, k).cpu()
    assert torch.equal(out, ref)


@pytest.mark.gpu
def test_radius_graph_hip_nearest_policy():
    from hydragnn_amd.ops.radius import radius_graph_device

    pos, batch = _batch(1)
    ei, _ = radius_graph_device(pos.cuda(), batch.cuda(), 3.0, 6, cap_policy="nearest")
    ei = ei.cpu()
    ptr = torch.cat([torch.zeros(1, dtype=torch.long), torch.bincount(batch).cumsum(0)])
    for g in range(len(ptr) - 1):
        a, b = int(ptr[g]), int(ptr[g + 1])
        ref = radius_graph(pos[a:b], 3.0, max_num_neighbors=6, cap_policy="nearest") + a
        m = (ei[1] >= a) & (ei[1] < b)
        got = ei[:, m]
        key = lambda e: sorted(zip(e[1].tolist(), e[0].tolist()))  # noqa: E731
        assert key(got) == key(ref)


@pytest.mark.gpu
def test_radius_graph_hip_periodic_bcc():
    from hydragnn_amd.ops.radius import pbc_reps, radius_graph_device

    pos, cell = _bcc_cr()
    reps = pbc_reps(cell.view(1, 3, 3), torch.ones(1, 3, dtype=torch.bool), 5.0)
    ei, sh = radius_graph_device(pos.float().cuda(), None, 5.0, 100, cap_policy="index",
                                 cell=cell.float().view(1, 3, 3).cuda(), reps=reps.cuda())
    ei, sh = ei.cpu(), sh.cpu()
    assert ei.shape[1] == 14 * pos.shape[0]
    d = (pos[ei[1]] - pos[ei[0]] + sh.double()).norm(dim=-1)
    assert bool(((d <= 5.0 + 1e-4) & (d > 0)).all())
    ref, rsh = radius_graph_pbc(pos, cell, [True] * 3, 5.0, max_num_neighbors=100)
    key = lambda e, s: sorted(zip(e[1].tolist(), e[0].tolist(), [tuple(np.round(v, 3)) for v in s.tolist()]))  # noqa
    assert key(ei, sh) == key(ref, rsh)


@pytest.mark.gpu
def test_triplets_hip():
    from hydragnn_amd.data.graph import collate
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.models.dimenet import triplets_csr

    b = collate(oc20_like(5, seed=2, min_atoms=6, max_atoms=15, radius=5.0, max_neighbours=8, pe_dim=1))
    kj, ji = triplets_csr(b.dst_si, b.src_si, b.num_nodes)
    g = b.to("cuda")
    kj2, ji2 = triplets_csr(g.dst_si, g.src_si, g.num_nodes)
    assert torch.equal(kj2.cpu(), kj) and torch.equal(ji2.cpu(), ji)


def _lap(ei, n):
    A = torch.zeros(n, n, dtype=torch.float64)
    A[ei[1], ei[0]] = 1.0
    A[ei[0], ei[1]] = 1.0
    d = A.sum(1)
    di = torch.where(d > 0, d.clamp(min=1e-12).rsqrt(), torch.zeros_like(d))
    return torch.eye(n, dtype=torch.float64) - di[:, None] * A * di[None, :]


def test_laplacian_pe_host():
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.data.transforms import laplacian_pe

    s = oc20_like(1, seed=1, min_atoms=12, max_atoms=12, radius=5.0, max_neighbours=6, pe_dim=1)[0]
    pe = laplacian_pe(s.edge_index, s.num_nodes, 4, seed=0).double()
    L = _lap(s.edge_index, s.num_nodes)
    lam = torch.linalg.eigvalsh(L)[1:5]
    for c in range(4):
        v = pe[:, c]
        torch.testing.assert_close(L @ v, lam[c] * v, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
def test_laplacian_pe_hip_jacobi():
    """Batched Jacobi eigenvectors: unit norm, L v = lambda v with the eigenvalues of the
    host solver (subspace-exact for degenerate eigenvalues), zero padding for tiny graphs."""
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.data.transforms import laplacian_pe_batch

    samples = oc20_like(12, seed=4, min_atoms=2, max_atoms=126, radius=6.0, max_neighbours=8, pe_dim=1)
    k = 6
    pes = laplacian_pe_batch(samples, k, seed=0, device="cuda")
    for s, pe in zip(samples, pes):
        n = s.num_nodes
        L = _lap(s.edge_index, n)
        lam = torch.linalg.eigvalsh(L)
        pe = pe.double()
        for c in range(k):
            v = pe[:, c]
            if c + 1 >= n:
                assert float(v.abs().max()) == 0.0
                continue
            assert abs(float(v.norm()) - 1.0) < 1e-3
            lv = float(v @ L @ v)
            assert abs(lv - float(lam[c + 1])) < 1e-3, (n, c, lv, float(lam[c + 1]))
            assert float((L @ v - lv * v).norm()) < 5e-3


def test_pbc_radius_retry_expands_cutoff():
    """Reference RadiusGraphPBC: when a node receives no edge the cutoff grows x1.25 (<= 3 builds)."""
    from hydragnn_amd.data.transforms import missing_receivers, radius_graph_pbc_robust

    cell = torch.eye(3) * 10.0
    pos = torch.tensor([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [5.0, 5.0, 5.0]])
    ei, sh, cutoff = radius_graph_pbc_robust(pos, cell, [True] * 3, 4.0, max_num_neighbors=10)
    # atom 2 is 5*sqrt(3)-ish = 7.8 A away from the pair in the minimum image: 4 -> 5 -> 6.25 fails twice,
    # then the artificial edge is added
    assert missing_receivers(ei, 3).numel() == 0
    assert abs(cutoff - 6.25) < 1e-9
    ei2, _, c2 = radius_graph_pbc_robust(pos, cell, [True] * 3, 7.0, max_num_neighbors=10)
    assert abs(c2 - 8.75) < 1e-9 and missing_receivers(ei2, 3).numel() == 0


def test_ensure_connected_adds_one_edge_per_isolated_node():
    from hydragnn_amd.data.transforms import ensure_connected

    ei = torch.tensor([[0, 1], [1, 0]])
    sh = torch.zeros(2, 3)
    ei2, sh2, added = ensure_connected(ei, sh, 4, seed=0)
    assert added == 2 and ei2.shape[1] == 4 and sh2.shape == (4, 3)
    assert sorted(ei2[1, 2:].tolist()) == [2, 3]
    assert all(int(s) != int(d) for s, d in zip(ei2[0, 2:], ei2[1, 2:]))


def test_pbc_descriptors():
    from hydragnn_amd.data.transforms import local_cartesian, pbc_distance

    pos = torch.tensor([[0.0, 0.0, 0.0], [9.5, 0.0, 0.0]])
    ei = torch.tensor([[1], [0]])
    sh = torch.tensor([[10.0, 0.0, 0.0]])  # vec = pos[dst] - pos[src] + shift = 0.5
    d = pbc_distance(pos, ei, sh, norm=False)
    assert torch.allclose(d, torch.tensor([[0.5]]))
    c = local_cartesian(pos, ei, sh, norm=False)
    assert torch.allclose(c, torch.tensor([[-0.5, 0.0, 0.0]]))
    cn = local_cartesian(pos, ei, sh, norm=True)
    assert torch.allclose(cn, torch.tensor([[0.0, 0.5, 0.5]]))


def test_radius_graph_default_cap_is_index_order():
    """Non-PBC default follows torch_cluster (first sources in index order), not nearest."""
    pos = torch.tensor([[0.0, 0, 0], [0.9, 0, 0], [0.1, 0, 0], [0.2, 0, 0]])
    ei = radius_graph(pos, 1.0, max_num_neighbors=1)
    first = {int(d): int(s) for s, d in zip(ei[0], ei[1])}
    assert first[0] == 1  # index order keeps node 1 although node 2 is nearer


@pytest.mark.gpu
@pytest.mark.parametrize("policy,cap", [("index", 12), ("nearest", 12), ("index", None)])
def test_cell_list_radius_graph_matches_brute_force(policy, cap):
    """Cell-list HIP builder == the brute-force HIP builder (edge set AND order), batched
    non-periodic graphs of different extents."""
    from hydragnn_amd.ops.radius import radius_graph_cells, radius_graph_device

    torch.manual_seed(0)
    sizes = [50, 300, 7, 1200]
    pos = torch.cat([torch.rand(n, 3) * (n ** (1 / 3)) * 1.6 for n in sizes]).cuda()
    batch = torch.cat([torch.full((n,), g, dtype=torch.long) for g, n in enumerate(sizes)]).cuda()
    a, _ = radius_graph_cells(pos, batch, 2.1, cap, cap_policy=policy)
    b, _ = radius_graph_device(pos, batch, 2.1, cap if cap is not None else None, cap_policy=policy)
    assert torch.equal(a.cpu(), b.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["index", "nearest"])
def test_cell_list_radius_graph_periodic_triclinic(policy):
    from hydragnn_amd.ops.radius import pbc_reps, radius_graph_cells, radius_graph_device

    torch.manual_seed(1)
    cells = [torch.tensor([[6.0, 0, 0], [1.5, 5.5, 0], [0.7, 0.4, 7.0]]), torch.eye(3) * 2.5,
             torch.tensor([[12.0, 0, 0], [0, 9.0, 0], [2.0, 0, 10.0]])]
    counts = [40, 5, 300]
    pos = torch.cat([torch.rand(n, 3) @ c for n, c in zip(counts, cells)]).cuda()
    batch = torch.cat([torch.full((n,), g, dtype=torch.long) for g, n in enumerate(counts)]).cuda()
    cell = torch.stack(cells).cuda()
    reps = pbc_reps(cell, torch.ones(3, 3, dtype=torch.bool), 3.1)
    a, sa = radius_graph_cells(pos, batch, 3.1, 16, cap_policy=policy, cell=cell)
    b, sb = radius_graph_device(pos, batch, 3.1, 16, cap_policy=policy, cell=cell, reps=reps)
    assert torch.equal(a.cpu(), b.cpu())
    torch.testing.assert_close(sa.cpu(), sb.cpu(), rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_cell_list_radius_graph_large_structure_linear_time():
    """A 100k-atom structure (the O(N) case): edges agree with a host reference on a sample
    of receivers, and the build is fast."""
    import time

    from hydragnn_amd.ops.radius import radius_graph_cells

    torch.manual_seed(2)
    n = 100_000
    L = (n / 0.08) ** (1 / 3)
    pos = (torch.rand(n, 3) * L).cuda()
    radius_graph_cells(pos[:1000], None, 3.0)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    ei, _ = radius_graph_cells(pos, None, 3.0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    assert dt < 2.0, dt
    p = pos.cpu().double()
    ei = ei.cpu()
    for i in (0, 12345, 99999):
        want = ((p - p[i]).norm(dim=1) <= 3.0).nonzero().view(-1)
        want = want[want != i]
        got = ei[0][ei[1] == i].sort().values
        assert torch.equal(got, want.sort().values)


@pytest.mark.gpu
@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("small_kernel", ["1", "0"])
@pytest.mark.parametrize("per_graph", ["1", "0"])
def test_static_radius_graph_gpu_matches_cpu_twin(big, small_kernel, per_graph, monkeypatch):
    """Capturable in-forward radius graph (csrc/graph.hip radius_static_*, the one-workgroup
    builder and the multi-launch one): same edges, CSR views (stable source order), limit
    and padding layout as the CPU twin, no host sync (fixed capacity)."""
    from hydragnn_amd.ops.radius import interaction_graph_static

    monkeypatch.setenv("HYDRA_RS_SMALL", small_kernel)
    monkeypatch.setenv("HYDRA_RS_GRAPHS", per_graph)
    g = torch.Generator().manual_seed(3)
    sizes = [7, 12, 1, 9] if not big else [int(x) for x in torch.randint(1, 30, (120,), generator=g)]
    pos = torch.cat([torch.rand(n, 3, generator=g) * 3 for n in sizes] + [torch.zeros(3, 3)])
    batch = torch.cat([torch.full((n,), i) for i, n in enumerate(sizes)] + [torch.full((3,), len(sizes))])
    ptr = torch.tensor([0] + list(np.cumsum(sizes + [3])))
    mask = torch.cat([torch.ones(sum(sizes), dtype=torch.bool), torch.zeros(3, dtype=torch.bool)])

    class D(dict):
        def get(self, k, d=None):
            return dict.get(self, k, d)

    def data(dev):
        d = D(node_mask=mask.to(dev), max_graph_nodes=max(sizes))
        d.batch, d.ptr = batch.to(dev), ptr.to(dev)
        return d

    a_dst, a_src = interaction_graph_static(pos, data("cpu"), 1.5, 4)
    b_dst, b_src = interaction_graph_static(pos.cuda(), data("cuda"), 1.5, 4)
    for x, y in [(a_dst.index, b_dst.index), (a_dst.rowptr, b_dst.rowptr), (a_src.index, b_src.index),
                 (a_src.rowptr, b_src.rowptr), (a_src.perm, b_src.perm), (a_dst.limit, b_dst.limit)]:
        assert torch.equal(x, y.cpu())
    assert a_dst.index.numel() == pos.shape[0] * 4


@pytest.mark.gpu
def test_static_radius_graph_per_graph_size_bound_flags():
    """A graph above the store's ``max_graph_nodes`` bound gets no edges in the per-graph
    builder and sets the device flag that the epoch check turns into an error."""
    from hydragnn_amd.ops import devcheck
    from hydragnn_amd.ops.radius import interaction_graph_static

    sizes = [5, 9]
    pos = torch.rand(sum(sizes) + 2, 3) * 0.5
    ptr = torch.tensor([0, 5, 14, 16])
    batch = torch.cat([torch.zeros(5), torch.ones(9), torch.full((2,), 2)]).long()
    mask = torch.cat([torch.ones(14, dtype=torch.bool), torch.zeros(2, dtype=torch.bool)])

    class D(dict):
        def get(self, k, d=None):
            return dict.get(self, k, d)

    d = D(node_mask=mask.cuda(), max_graph_nodes=6)
    d.batch, d.ptr = batch.cuda(), ptr.cuda()
    dst, src = interaction_graph_static(pos.cuda(), d, 2.0, 4)
    torch.cuda.synchronize()
    assert int(dst.limit) == 5 * 4  # graph 0 only (all its pairs within r, cap 4)
    assert int(devcheck.flag(pos.cuda().device, "radius_graph_size")) == 9
    with pytest.raises(RuntimeError, match="largest graph"):
        devcheck.check_all()
