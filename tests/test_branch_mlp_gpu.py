"""Branch-stacked MLP read-out (ops/branch_mlp.py, csrc/branch_mlp.hip) == a plain fp64
per-row loop over each row's branch chain: outputs, the input gradient and every weight /
bias gradient (rows of padding branch -1 produce zeros and contribute nothing)."""
import pytest
import torch
from torch import nn

from hydragnn_amd.ops import branch_mlp as bm

pytestmark = pytest.mark.gpu


def _chain(dims, acts, trans, scales, bias, g):
    steps = []
    for l in range(len(dims) - 1):
        I, O = dims[l], dims[l + 1]
        W = nn.Parameter(torch.randn((I, O) if trans[l] else (O, I), generator=g) / I ** 0.5)
        b = nn.Parameter(torch.randn(O, generator=g) * 0.1) if (bias[l] and not trans[l]) else None
        steps.append((W, trans[l], b, acts[l], scales[l]))
    return steps


def _ref_row(x, steps):
    h = x
    for (W, tr, b, act, sc) in steps:
        h = h * sc
        z = h @ W if tr else h @ W.t()
        if b is not None:
            z = z + b
        h = act(z) if act is not None else z
    return h


@pytest.mark.parametrize("R,dims,acts,trans,nb", [
    (77, [64, 50, 50, 3], [nn.ReLU(), nn.ReLU(), None], [0, 0, 0], 5),
    (33, [118, 1], [None], [1], 5),
    (40, [64, 64, 64, 3], [nn.SiLU(), nn.SiLU(), None], [1, 0, 0], 3),
    (12, [128, 96, 1], [nn.Tanh(), None], [0, 0], 2),
])
def test_branch_mlp_matches_per_row_loop(R, dims, acts, trans, nb):
    g = torch.Generator().manual_seed(R + nb)
    scales = [0.7 if t else 1.0 for t in trans]
    chains = [_chain(dims, acts, trans, scales, [1] * len(trans), g) for _ in range(nb)]
    x = torch.randn(R, dims[0], generator=g, dtype=torch.float64)
    rid = torch.randint(-1, nb, (R,), generator=g)
    go = torch.randn(R, dims[-1], generator=g, dtype=torch.float64)
    # fp64 reference
    ref_chains = [[(nn.Parameter(W.detach().double()), tr, None if b is None else nn.Parameter(b.detach().double()),
                    a, s) for (W, tr, b, a, s) in c] for c in chains]
    xr = x.clone().requires_grad_(True)
    outs = []
    for r in range(R):
        q = int(rid[r])
        outs.append(_ref_row(xr[r:r + 1], ref_chains[q]) if q >= 0 else torch.zeros(1, dims[-1], dtype=torch.float64))
    ref = torch.cat(outs, 0)
    ref.backward(go)
    dev = torch.device("cuda")
    dchains = [[(nn.Parameter(W.detach().to(dev)), tr, None if b is None else nn.Parameter(b.detach().to(dev)), a, s)
                for (W, tr, b, a, s) in c] for c in chains]
    # the input as a column slice of wider rows (the MACE scalar block): read with its stride
    wide = torch.cat([x.float(), torch.randn(R, 5, generator=g)], 1).to(dev).requires_grad_(True)
    xd = wide[:, :dims[0]]
    assert bm.eligible(xd, dchains) and not xd.is_contiguous()
    out = bm.branch_mlp(xd, rid.int().to(dev), dchains, dims[-1])
    out.backward(go.float().to(dev))
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(wide.grad[:, :dims[0]].double().cpu(), xr.grad, rtol=1e-4, atol=1e-5)
    assert not wide.grad[:, dims[0]:].abs().sum()
    for c, rc in zip(dchains, ref_chains):
        for (W, _, b, _, _), (rW, _, rb, _, _) in zip(c, rc):
            gw = W.grad if W.grad is not None else torch.zeros_like(W)
            rgw = rW.grad if rW.grad is not None else torch.zeros_like(rW)
            torch.testing.assert_close(gw.double().cpu(), rgw, rtol=1e-4, atol=1e-5)
            if b is not None:
                gb = b.grad if b.grad is not None else torch.zeros_like(b)
                rgb = rb.grad if rb.grad is not None else torch.zeros_like(rb)
                torch.testing.assert_close(gb.double().cpu(), rgb, rtol=1e-4, atol=1e-5)


def test_branch_mlp_accumulates_into_previous_readouts():
    """``acc``: out = acc + chain(x) (padding rows keep acc), d acc = the upstream gradient."""
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    chains = [[(nn.Parameter(torch.randn(3, 16, generator=g).to(dev)), 0,
                nn.Parameter(torch.randn(3, generator=g).to(dev)), None, 1.0)] for _ in range(2)]
    x = torch.randn(9, 16, generator=g).to(dev).requires_grad_(True)
    rid = torch.tensor([0, 1, -1, 1, 0, 0, -1, 1, 1], dtype=torch.int32, device=dev)
    acc = torch.randn(9, 3, generator=g).to(dev).requires_grad_(True)
    out = bm.branch_mlp(x, rid, chains, 3, acc=acc)
    base = bm.branch_mlp(x.detach(), rid, chains, 3)
    torch.testing.assert_close(out, acc.detach() + base, rtol=1e-6, atol=1e-6)
    go = torch.randn(9, 3, generator=g).to(dev)
    out.backward(go)
    torch.testing.assert_close(acc.grad, go)
