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


@pytest.mark.gpu
@pytest.mark.parametrize("drop", [None, 2])
def test_irreps_linear_residual_and_multi(drop):
    """Residual epilogue (``O3Linear(x, residual=r)``) and the shared-input chain
    (``o3.linear_multi``: skip / up / down of a MACE interaction), with one output unused
    (its gradient is None), against the fp64 torch composite."""
    torch.manual_seed(7)
    ir_in = I([(64, 0, 1), (64, 1, -1)])
    outs = [I([(64, 0, 1), (64, 1, -1), (64, 2, 1)]), ir_in, I([(64, 0, 1)])]
    lins = [o3.O3Linear(ir_in, o).cuda() for o in outs]
    N = 301
    x = torch.randn(N, ir_in.dim, device="cuda", requires_grad=True)
    r = torch.randn(N, outs[1].dim, device="cuda", requires_grad=True)
    gs = [torch.randn(N, o.dim, device="cuda") for o in outs]

    def run(ls, xx, rr, gg):
        ys = o3.linear_multi(ls, xx)
        z = ls[1](ys[1], residual=rr)  # the product block's linear(.) + sc
        loss = sum((y * g).sum() for k, (y, g) in enumerate(zip(ys, gg)) if k != drop) + (z * gg[1]).sum()
        return torch.autograd.grad(loss, [xx, rr] + [lin.weight for lin in ls], allow_unused=True)

    got = run(lins, x, r, gs)
    with composite_mode(True):
        lins64 = [o3.O3Linear(ir_in, o).double().cuda() for o in outs]
        for a, b in zip(lins64, lins):
            a.weight.data.copy_(b.weight.data.double())
        ref = run(lins64, x.detach().double().requires_grad_(True), r.detach().double().requires_grad_(True),
                  [g.double() for g in gs])
    for a, b in zip(got, ref):
        if b is None:  # the unused output's weight
            assert a is None or not a.any()
            continue
        torch.testing.assert_close(a.double(), b, rtol=1e-4, atol=2e-3)
