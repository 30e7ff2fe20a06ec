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
