"""SchNet continuous-filter network in one HIP launch each way (csrc/schnet.hip,
reference SCFStack.py:214-293): W = (ssp(rbf W1^T + b1) W2^T + b2) * C against the
plain-torch module chain in fp64 — values and every weight/bias gradient, with and
without the deferred grouped weight-gradient launch."""
import pytest
import torch
from torch import nn

from hydragnn_amd.models.layers import Linear
from hydragnn_amd.models.schnet import ShiftedSoftplus, _CFFilter, _filter_fusable
from hydragnn_amd.ops import linear as lin

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("E,K,F", [(1, 50, 64), (333, 50, 64), (5000, 10, 8), (2049, 64, 64), (100, 7, 33)])
@pytest.mark.parametrize("defer", [False, True])
def test_cf_filter_matches_module(E, K, F, defer):
    torch.manual_seed(E + K + F)
    net = nn.Sequential(Linear(K, F), ShiftedSoftplus(), Linear(F, F)).cuda()
    rbf = torch.rand(E, K, device="cuda")
    C = torch.rand(E, device="cuda")
    assert _filter_fusable(net, rbf, C)
    G = torch.randn(E, F, device="cuda")
    with lin.deferred_wgrad(defer):
        out = _CFFilter.apply(rbf, C, net[0].weight, net[0].bias, net[2].weight, net[2].bias)
        (out * G).sum().backward()
    got = [p.grad.clone() for p in net.parameters()]
    ref_net = nn.Sequential(nn.Linear(K, F), ShiftedSoftplus(), nn.Linear(F, F)).double()
    with torch.no_grad():
        for a, b in zip(ref_net.parameters(), net.parameters()):
            a.copy_(b.double().cpu())
    ref = ref_net(rbf.double().cpu()) * C.double().cpu().view(-1, 1)
    (ref * G.double().cpu()).sum().backward()
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-5, atol=1e-5)
    for a, b in zip(got, ref_net.parameters()):
        torch.testing.assert_close(a.double().cpu(), b.grad, rtol=1e-4, atol=1e-4 * max(1.0, E ** 0.5 / 10))


@pytest.mark.parametrize("M,F", [(1030, 64), (5000, 32), (2049, 17)])
@pytest.mark.parametrize("defer", [False, True])
def test_residual_silu_block_matches_module(M, F, defer):
    """DimeNet++ ResidualLayer in one launch each way (csrc/resmlp.hip):
    y = x + silu(lin2(silu(lin1(x)))) against the fp64 module chain — values, dx and every
    weight/bias gradient."""
    from hydragnn_amd.models.dimenet import ResidualLayer

    torch.manual_seed(M + F)
    layer = ResidualLayer(F, nn.SiLU()).cuda()
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.1 * torch.randn_like(p))
    x = torch.randn(M, F, device="cuda", requires_grad=True)
    G = torch.randn(M, F, device="cuda")
    with lin.deferred_wgrad(defer):
        y = layer(x)
        (y * G).sum().backward()
    assert y.grad_fn is not None and "ResMLP" in type(y.grad_fn).__name__
    x64 = x.detach().double().cpu().requires_grad_()
    l1 = nn.Linear(F, F).double()
    l2 = nn.Linear(F, F).double()
    with torch.no_grad():
        l1.weight.copy_(layer.lin1.weight.double().cpu())
        l1.bias.copy_(layer.lin1.bias.double().cpu())
        l2.weight.copy_(layer.lin2.weight.double().cpu())
        l2.bias.copy_(layer.lin2.bias.double().cpu())
    act = nn.SiLU()
    ref = x64 + act(l2(act(l1(x64))))
    (ref * G.double().cpu()).sum().backward()
    torch.testing.assert_close(y.double().cpu(), ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.double().cpu(), x64.grad, rtol=1e-4, atol=1e-4)
    tol = 1e-4 * max(1.0, M ** 0.5 / 10)
    for got, want in ((layer.lin1.weight.grad, l1.weight.grad), (layer.lin1.bias.grad, l1.bias.grad),
                      (layer.lin2.weight.grad, l2.weight.grad), (layer.lin2.bias.grad, l2.bias.grad)):
        torch.testing.assert_close(got.double().cpu(), want, rtol=1e-4, atol=tol)


@pytest.mark.parametrize("N,S", [(1, 1), (77, 5), (550, 10), (4000, 118), (130, 1024)])
def test_element_index_one_wave_matches_cpu(N, S):
    """ops.o3.element_index on the GPU (csrc/segment.hip elem_csr: stable counting sort in
    one wave) == the CPU twin (bincount + stable sort): index, CSR and permutation."""
    from hydragnn_amd.ops.o3 import element_index

    g = torch.Generator().manual_seed(N + S)
    elem = torch.randint(0, S, (N,), generator=g)
    if N > 10:
        elem[::7] = 0  # long runs of one element
    a = element_index(elem, S)
    b = element_index(elem.cuda(), S)
    assert torch.equal(a.index, b.index.cpu()) and torch.equal(a.rowptr, b.rowptr.cpu())
    assert torch.equal(a.perm, b.perm.cpu())


@pytest.mark.parametrize("I,O,bias,mul,add", [(64, 64, True, False, False), (64, 64, True, True, False),
                                              (64, 48, False, False, True), (40, 64, True, True, True)])
def test_dimenet_silu_linear_matches_fp64(I, O, bias, mul, add):
    """DimeNet++ act(lin(x)) * m + a step in one launch each way (models/dimenet.py silu_lin,
    csrc/resmlp.hip lin_act) == the fp64 module chain: values, dx, dW, db, dmul, dadd."""
    from torch import nn

    from hydragnn_amd.models.dimenet import _SiluLinear, silu_lin

    g = torch.Generator().manual_seed(I + O + 2 * mul + add)
    M = 3000
    lin = nn.Linear(I, O, bias=bias).double()
    x = torch.randn(M, I, generator=g, dtype=torch.float64)
    m = torch.randn(M, O, generator=g, dtype=torch.float64) if mul else None
    a = torch.randn(M, O, generator=g, dtype=torch.float64) if add else None
    go = torch.randn(M, O, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    mr = m.clone().requires_grad_(True) if mul else None
    ar = a.clone().requires_grad_(True) if add else None
    ref = torch.nn.functional.silu(lin(xr))
    if mul:
        ref = ref * mr
    if add:
        ref = ref + ar
    ref.backward(go)
    dev = torch.device("cuda")
    lind = nn.Linear(I, O, bias=bias).to(dev)
    with torch.no_grad():
        lind.weight.copy_(lin.weight.float())
        if bias:
            lind.bias.copy_(lin.bias.float())
    xd = x.float().to(dev).requires_grad_(True)
    md = m.float().to(dev).requires_grad_(True) if mul else None
    ad = a.float().to(dev).requires_grad_(True) if add else None
    out = silu_lin(lind, nn.SiLU(), xd, mul=md, add=ad)
    assert isinstance(out.grad_fn.__class__, type) and "SiluLinear" in type(out.grad_fn).__name__
    out.backward(go.float().to(dev))
    tol = dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), **tol)
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, **tol)
    torch.testing.assert_close(lind.weight.grad.double().cpu(), lin.weight.grad, rtol=1e-4, atol=1e-3)
    if bias:
        torch.testing.assert_close(lind.bias.grad.double().cpu(), lin.bias.grad, rtol=1e-4, atol=1e-3)
    if mul:
        torch.testing.assert_close(md.grad.double().cpu(), mr.grad, **tol)
    if add:
        torch.testing.assert_close(ad.grad.double().cpu(), ar.grad, **tol)
