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
