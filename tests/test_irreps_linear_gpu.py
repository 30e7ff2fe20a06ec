"""Native o3.Linear (csrc/irreps_linear.hip) against the plain-torch fp32 path of the same
module (``composite_mode``): outputs, input gradients and weight gradients, for the MACE
irreps shapes (scalar-only, l <= 1, l <= 2 mixed multiplicities, several input blocks of one
l feeding one output, an input block with no path)."""
import pytest
import torch

from hydragnn_amd.ops import o3
from hydragnn_amd.ops.pna import composite_mode

I = o3.Irreps

CASES = [
    (I([(64, 0, 1)]), I([(64, 0, 1)]), 544),
    (I([(64, 0, 1), (64, 1, -1)]), I([(64, 0, 1), (64, 1, -1)]), 544),
    (I([(64, 0, 1), (64, 1, -1), (64, 2, 1)]), I([(64, 0, 1), (64, 1, -1)]), 300),
    (I([(16, 0, 1), (24, 1, -1), (8, 0, 1), (5, 2, 1)]), I([(70, 0, 1), (3, 1, -1), (130, 2, 1)]), 37),
    (I([(64, 0, 1), (64, 1, -1), (64, 2, 1)]), I([(64, 0, 1)]), 1000),
    (I([(118, 0, 1)]), I([(64, 0, 1)]), 17),
    # a MACE message row after the uvu product (> 1024 columns: several blocks per l)
    (I([(64, 0, 1), (64, 1, -1), (64, 2, 1), (64, 1, -1), (64, 0, 1), (64, 2, 1), (64, 1, -1), (64, 3, -1),
        (64, 2, 1)]), I([(64, 0, 1), (64, 1, -1), (64, 2, 1)]), 300),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)))
def test_irreps_linear_native_vs_torch(case):
    ir_in, ir_out, N = CASES[case]
    torch.manual_seed(case)
    lin = o3.O3Linear(ir_in, ir_out).cuda()
    x = torch.randn(N, ir_in.dim, device="cuda", requires_grad=True)
    g = torch.randn(N, ir_out.dim, device="cuda")
    assert lin.native_ok(x)
    y = lin(x)
    dx, dw = torch.autograd.grad(y, (x, lin.weight), g)
    with composite_mode(True):
        assert not lin.native_ok(x)
        x64 = x.detach().double().requires_grad_(True)
        lin64 = o3.O3Linear(ir_in, ir_out).double().cuda()
        lin64.weight.data.copy_(lin.weight.data.double())
        y_ref = lin64(x64)
        dx_ref, dw_ref = torch.autograd.grad(y_ref, (x64, lin64.weight), g.double())
    torch.testing.assert_close(y.double(), y_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dx.double(), dx_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dw.double(), dw_ref, rtol=1e-4, atol=2e-3)
