"""MACE radial embedding (Bessel basis x polynomial cutoff, ``csrc/radial.hip``
mace_radial_fwd/bwd, reference mace_utils/modules/radial.py:23-130) == the fp64 torch
composite, values and edge-length gradient, including lengths past the cutoff."""
import pytest
import torch

from hydragnn_amd.models.mace import RadialEmbeddingBlock, _MaceRadial
from hydragnn_amd.ops.pna import composite_mode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,p,rc", [(8, 5, 5.0), (6, 6, 4.0), (3, 3, 6.0)])
def test_mace_radial_matches_composite(K, p, rc):
    g = torch.Generator().manual_seed(K + p)
    r = (torch.rand(1000, 1, generator=g, dtype=torch.float64) * (rc * 1.2 - 0.3) + 0.3)
    blk = RadialEmbeddingBlock(rc, K, p)
    rr = r.clone().requires_grad_(True)
    ref = blk.double()(rr)
    go = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(go)

    dev = torch.device("cuda")
    blk = blk.float().to(dev)
    rd = r.float().to(dev).requires_grad_(True)
    out = blk(rd)
    assert "MaceRadial" in type(out.grad_fn).__name__
    out.backward(go.float().to(dev))
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(rd.grad.double().cpu(), rr.grad, rtol=1e-4, atol=1e-5)
    with composite_mode(True):
        comp = blk(rd.detach())
    assert not isinstance(comp.grad_fn, _MaceRadial)
    torch.testing.assert_close(comp, out.detach(), rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("shape,s", [((2048, 64), 0.125), ((37, 12), 1.7)])
def test_scaled_silu_matches_torch(shape, s):
    """FullyConnectedNet hidden activation silu(s x) (csrc/conv_misc.hip scaled_silu_*)."""
    from hydragnn_amd.ops.o3 import _ScaledSilu, scaled_silu

    g = torch.Generator().manual_seed(shape[0])
    x = torch.randn(shape, generator=g, dtype=torch.float64) * 4
    go = torch.randn(shape, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.silu(xr * s).backward(go)
    xd = x.float().cuda().requires_grad_(True)
    y = scaled_silu(xd, s)
    assert isinstance(y.grad_fn, _ScaledSilu._backward_cls)
    y.backward(go.float().cuda())
    torch.testing.assert_close(y.double().cpu(), torch.nn.functional.silu(x * s), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("linact", [False, True])
@pytest.mark.parametrize("N,E,nef,nd", [(60, 700, 8, 64), (9, 40, 5, 16)])
def test_fcn_first_layer_split_matches_concat(N, E, nef, nd, linact, monkeypatch):
    """MACE radial FCN with the first layer's cat[edge_feats, down[src], down[dst]] split at
    node level (ops/o3.py _FCNFirstSplit, csrc/conv_misc.hip edge_gather_silu) == the
    concatenated fp64 FullyConnectedNet: values and the gradients of edge_feats, down and
    every weight (``linact``: the hidden layer runs csrc/resmlp.hip lin_act, _LinSilu)."""
    from hydragnn_amd.ops import o3
    from hydragnn_amd.ops import segment as seg
    from hydragnn_amd.ops.o3 import FullyConnectedNet, _FCNFirstSplit

    monkeypatch.setattr(o3, "_FCN_LINACT", linact)
    g = torch.Generator().manual_seed(N + E)
    dst = torch.sort(torch.randint(0, N, (E,), generator=g)).values
    src = torch.randint(0, N, (E,), generator=g)
    ef = torch.randn(E, nef, generator=g, dtype=torch.float64)
    down = torch.randn(N, nd, generator=g, dtype=torch.float64)
    fcn = FullyConnectedNet([nef + 2 * nd, nd, nd, 3 * nd]).double()
    go = torch.randn(E, 3 * nd, generator=g, dtype=torch.float64)
    efr, downr = ef.clone().requires_grad_(True), down.clone().requires_grad_(True)
    ref = fcn(torch.cat([efr, downr[src], downr[dst]], -1))
    ref.backward(go)
    gref = [efr.grad, downr.grad] + [w.grad.clone() for w in fcn.weights]

    dev = torch.device("cuda")
    fcn = fcn.float().to(dev)
    for w in fcn.weights:
        w.grad = None
    dst_si = seg.SegIndex.from_index(dst.int().to(dev), N, sorted_=True)
    src_si = seg.SegIndex.from_index(src.int().to(dev), N, sorted_=False)
    efd = ef.float().to(dev).requires_grad_(True)
    downd = down.float().to(dev).requires_grad_(True)
    out = fcn.forward_split(efd, downd, src_si, dst_si)
    names = []
    fn = out.grad_fn
    while fn is not None and len(names) < 20:
        names.append(type(fn).__name__)
        fn = fn.next_functions[0][0] if fn.next_functions else None
    assert any("FCNFirstSplit" in n for n in names), names
    assert any("LinSilu" in n for n in names) == linact, names  # hidden layer: GEMM + silu in one launch
    out.backward(go.float().to(dev))
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-5)
    got = [efd.grad, downd.grad] + [w.grad for w in fcn.weights]
    for a, b in zip(got, gref):
        torch.testing.assert_close(a.double().cpu(), b, rtol=1e-4, atol=1e-4)
