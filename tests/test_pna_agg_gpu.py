"""Fused PNA degree-scaler aggregation (``ops.pna.pna_aggregate`` over ``csrc/segment.hip``
seg_pna_agg / seg_pna_agg_bwd: [mean, min, max, std] x scalers incl. inverse_linear, the
PNAEq message aggregation of reference PNAEqStack.py:59-66) == the fp64 torch composite on
CPU, forward and gradient, for sorted and permuted CSR indices with empty segments and
constant (std-masked) segments."""
import pytest
import torch

from hydragnn_amd.ops import segment as seg
from hydragnn_amd.ops.pna import pna_aggregate, pna_aggregate_composite, pna_avg_deg

pytestmark = pytest.mark.gpu

SC5 = ("identity", "amplification", "attenuation", "linear", "inverse_linear")


def _index(E, N, sorted_, g):
    idx = torch.randint(0, N - 3, (E,), generator=g)  # last 3 segments empty
    if sorted_:
        idx = idx.sort().values
    return idx


@pytest.mark.parametrize("sorted_", [True, False])
@pytest.mark.parametrize("F,E,N,scalers", [(64, 3000, 400, SC5), (32, 517, 61, SC5[:4]), (3, 40, 9, ("linear",))])
def test_pna_aggregate_matches_composite(sorted_, F, E, N, scalers):
    g = torch.Generator().manual_seed(F * 7 + E)
    idx = _index(E, N, sorted_, g)
    m = torch.randn(E, F, generator=g, dtype=torch.float64)
    # one constant segment: its std is clamped and masked to 0 (zero std gradient)
    m[idx == 0] = 0.5
    avg = pna_avg_deg(torch.tensor([0.0, 3.0, 10.0, 5.0, 2.0, 1.0]))
    si_c = seg.SegIndex.from_index(idx, N, sorted_=sorted_)
    mc = m.clone().requires_grad_(True)
    ref = pna_aggregate_composite(mc, si_c, avg, scalers=scalers)
    go = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(go)

    dev = torch.device("cuda")
    si = si_c.to(dev)
    md = m.float().to(dev).requires_grad_(True)
    out = pna_aggregate(md, si, avg, scalers=scalers)
    assert out.grad_fn is not None and "PNAAggFused" in type(out.grad_fn).__name__
    out.backward(go.float().to(dev))
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=2e-5, atol=2e-5)
    # fp32 E[x^2]-E[x]^2 cancellation feeds the std gradient 1/(d std): fp32-level error
    torch.testing.assert_close(md.grad.double().cpu(), mc.grad, rtol=1e-3, atol=1e-3)
