"""Split-K weight-gradient kernels (csrc/linear.hip ``linear_wgrad`` and the grouped
variant) over a sweep of narrow / odd shapes (I, O not multiples of the 64-wide tile,
unaligned row strides) against torch fp32 matmuls."""
import pytest
import torch

from hydragnn_amd import _native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 37, 1000])
@pytest.mark.parametrize("O,I", [(32, 1), (32, 8), (32, 4), (32, 64), (96, 32), (1, 32), (17, 5), (64, 17)])
def test_linear_wgrad_shapes(M, O, I):
    g = torch.Generator(device="cpu").manual_seed(M * 1000 + O * 10 + I)
    dy = torch.randn(M, O, generator=g).cuda()
    x = torch.randn(M, I, generator=g).cuda()
    dW, db = _native.ops().linear_wgrad(dy, x, True)
    torch.testing.assert_close(dW, dy.t() @ x, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, dy.sum(0), rtol=1e-4, atol=1e-4)
    dWs = [torch.empty(O, I, device="cuda")]
    dbs = [torch.empty(O, device="cuda")]
    _native.ops().linear_wgrad_grouped([dy], [x], dWs, dbs, [0])
    torch.testing.assert_close(dWs[0], dy.t() @ x, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dbs[0], dy.sum(0), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M", [37, 5000, 200000])
@pytest.mark.parametrize("O,I", [(8, 42), (16, 64), (3, 17)])
@pytest.mark.parametrize("block", [False, True])
def test_grouped_wgrad_swapped_narrow(M, O, I, block):
    """Bias-free wide-input / narrow-output maps (DimeNet's sbf projection, [T, 42] -> 8)
    run as the transposed narrow problem; dW written transposed, also into a column block
    of a wider gradient, plain and accumulating."""
    g = torch.Generator(device="cpu").manual_seed(M + O * 7 + I)
    dy = torch.randn(M, O, generator=g).cuda()
    x = torch.randn(M, I, generator=g).cuda()
    ref = (dy.double().t() @ x.double()).float()
    full = torch.randn(O, I + 5, generator=g).cuda()
    dW = full[:, 2:2 + I] if block else torch.zeros(O, I, device="cuda")
    before = full.clone()
    _native.ops().linear_wgrad_grouped([dy], [x], [dW], [torch.empty(0, device="cuda")], [0])
    torch.testing.assert_close(dW, ref, rtol=1e-4, atol=1e-3 * max(1.0, M ** 0.5 / 10))
    _native.ops().linear_wgrad_grouped([dy], [x], [dW], [torch.empty(0, device="cuda")], [1])
    torch.testing.assert_close(dW, 2 * ref, rtol=1e-4, atol=2e-3 * max(1.0, M ** 0.5 / 10))
    if block:  # the columns outside the block are untouched
        assert torch.equal(full[:, :2], before[:, :2]) and torch.equal(full[:, 2 + I:], before[:, 2 + I:])


@pytest.mark.parametrize("defer", [False, True])
def test_linear_cols_matches_slices(defer):
    """ops.linear.linear_cols: column blocks of one concat-linear weight (DimeNet's embedding
    block) with the blocks' weight gradients in the deferred grouped launch == autograd
    through weight slices."""
    from hydragnn_amd.ops import linear as lin

    g = torch.Generator(device="cpu").manual_seed(5)
    W0 = torch.randn(64, 200, generator=g)
    xs = [torch.randn(3000, k, generator=g).cuda() for k in (64, 64, 64, 8)]
    offs = [0, 64, 128, 192]
    G = torch.randn(3000, 64, generator=g).cuda()
    Wa = torch.nn.Parameter(W0.clone().cuda())
    with lin.deferred_wgrad(defer):
        y = sum(lin.linear_cols(x, Wa, k0) for x, k0 in zip(xs, offs))
        (y * G).sum().backward()
    Wb = W0.clone().cuda().requires_grad_()
    yb = sum(torch.nn.functional.linear(x, Wb[:, k0:k0 + x.shape[1]]) for x, k0 in zip(xs, offs))
    (yb * G).sum().backward()
    torch.testing.assert_close(y, yb, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(Wa.grad, Wb.grad, rtol=1e-4, atol=1e-2)
