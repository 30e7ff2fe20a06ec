"""DimeNet++ triplet angle + spherical basis kernel (csrc/dimenet.hip) against the fp64
torch composite of models/dimenet.py (reference DIMEStack.py:170-190, PyG
SphericalBasisLayer): values and the gradient with respect to the positions."""
import pytest
import torch

from hydragnn_amd.models.dimenet import SphericalBasisLayer, triplets_csr
from hydragnn_amd.ops import segment as seg
from hydragnn_amd.ops.geometry import edge_vectors_and_lengths

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _graph(n=60, seed=0):
    g = torch.Generator().manual_seed(seed)
    pos = torch.rand(n, 3, generator=g) * 4.0
    d = torch.cdist(pos, pos)
    src, dst = torch.nonzero(d < 2.5, as_tuple=True)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    order = torch.argsort(dst * n + src)
    src, dst = src[order], dst[order]
    return pos, src, dst


def _torch_sbf(layer, pos, dst_si, src_si, kj_si, ji_si):
    vec, dist = edge_vectors_and_lengths(pos, dst_si, src_si)
    pos_ji = seg.gather(vec, ji_si)
    pos_ki = seg.gather(vec, kj_si) + pos_ji
    a = (pos_ji * pos_ki).sum(-1)
    b = torch.linalg.cross(pos_ji, pos_ki).norm(dim=-1)
    return layer(dist.view(-1), torch.atan2(b, a), kj_si)


@pytest.mark.parametrize("n_sph,n_rad", [(7, 6), (3, 4)])
def test_sbf_matches_composite(n_sph, n_rad):
    pos, src, dst = _graph()
    N, E = pos.shape[0], src.numel()
    dst_si = seg.SegIndex.from_index(dst.to(dev), N, sorted_=True)
    src_si = seg.SegIndex.from_index(src.to(dev), N, sorted_=False)
    kj, ji = triplets_csr(dst_si, src_si, N)
    kj_si = seg.SegIndex.from_index(kj, E, sorted_=False)
    ji_si = seg.SegIndex.from_index(ji, E, sorted_=True)
    layer = SphericalBasisLayer(n_sph, n_rad, cutoff=3.0, envelope_exponent=5).to(dev)
    p1 = pos.to(dev).requires_grad_()
    vec, _ = edge_vectors_and_lengths(p1, dst_si, src_si)
    assert layer.native_ok(vec)
    out = layer.from_vectors(vec, kj_si, ji_si)
    G = torch.randn_like(out)
    (out * G).sum().backward()
    # fp64 composite on the CPU
    cpu = lambda si: seg.SegIndex(si.index.cpu(), si.rowptr.cpu(), None if si.perm is None else si.perm.cpu(),  # noqa
                                  si.num_segments)
    lay64 = SphericalBasisLayer(n_sph, n_rad, cutoff=3.0, envelope_exponent=5).double()
    p2 = pos.double().requires_grad_()
    ref = _torch_sbf(lay64, p2, cpu(dst_si), cpu(src_si), cpu(kj_si), cpu(ji_si))
    (ref * G.double().cpu()).sum().backward()
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(p1.grad.double().cpu(), p2.grad, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("F", [64, 16])
def test_lowrank_triplet_filter_matches_materialised(F):
    """DimeNet++ interaction: gather_mul_sum with the low-rank triplet filter s8 W2^T
    recomputed per column (models/dimenet.py _LowRankGMS, csrc/dimenet.hip lr_*) == the
    materialised filter in fp64: output and the gradients of x_kj, s8 and W2."""
    from hydragnn_amd.models.dimenet import _LowRankGMS

    pos, src, dst = _graph(seed=3)
    N, E = pos.shape[0], src.numel()
    dst_si = seg.SegIndex.from_index(dst.to(dev), N, sorted_=True)
    src_si = seg.SegIndex.from_index(src.to(dev), N, sorted_=False)
    kj, ji = triplets_csr(dst_si, src_si, N)
    kj_si = seg.SegIndex.from_index(kj, E, sorted_=False)
    ji_si = seg.SegIndex.from_index(ji, E, sorted_=True)
    T = kj.numel()
    g = torch.Generator().manual_seed(F)
    x = torch.randn(E, F, generator=g)
    s8 = torch.randn(T, 8, generator=g)
    W2 = torch.randn(F, 8, generator=g)
    go = torch.randn(E, F, generator=g)
    xs = [t.to(dev).requires_grad_() for t in (x, s8, W2)]
    out = _LowRankGMS.apply(xs[0], xs[1], xs[2], kj_si, ji_si)
    out.backward(go.to(dev))
    xr = [t.double().requires_grad_() for t in (x, s8, W2)]
    filt = xr[1] @ xr[2].t()
    ref = torch.zeros(E, F, dtype=torch.float64).index_add_(0, ji.long().cpu(), xr[0][kj.long().cpu()] * filt)
    ref.backward(go.double())
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    for a, b in zip(xs, xr):
        torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=1e-4, atol=1e-3)
