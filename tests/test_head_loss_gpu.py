"""Fused graph head + masked loss (``ops/mlp.py`` _HeadLoss over ``csrc/mlp.hip``
head_loss_fwd/bwd, one workgroup each way) == plain fp32 PyTorch: Linear/ReLU chain, masked
mean loss over kept rows, autograd gradients of the input and of every weight."""
import pytest
import torch

from hydragnn_amd.ops import mlp as _mlp

pytestmark = pytest.mark.gpu


def _ref_loss(kind, pred, target, mask):
    keep = mask.view(-1, 1) if mask is not None else torch.ones_like(pred, dtype=torch.bool)
    d = (pred - target)[keep.expand_as(pred)]
    if kind == "mae":
        return d.abs().mean()
    if kind == "smooth_l1":
        a = d.abs()
        return torch.where(a < 1.0, 0.5 * d * d, a - 0.5).mean()
    l = (d * d).mean()
    return l.sqrt() if kind == "rmse" else l


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("kind", ["mae", "mse", "rmse", "smooth_l1"])
@pytest.mark.parametrize("G,dims,masked", [(33, [64, 50, 50, 50, 25, 1], True), (1, [32, 16, 1], False),
                                           (100, [64, 64, 3], True)])
def test_head_loss_matches_torch(kind, G, dims, masked, fused):
    dev = torch.device("cuda")
    torch.manual_seed(G + len(dims))
    lins = [torch.nn.Linear(dims[i], dims[i + 1]).to(dev) for i in range(len(dims) - 1)]
    seq = []
    for i, l in enumerate(lins):
        seq.append(l)
        if i < len(lins) - 1:
            seq.append(torch.nn.ReLU())
    seq = torch.nn.Sequential(*seq)
    x = torch.randn(G, dims[0], device=dev, requires_grad=True)
    target = torch.randn(G, dims[-1], device=dev)
    mask = (torch.arange(G, device=dev) < max(1, G - 2)) if masked else None
    layers = _mlp.head_loss_layers([seq], G, dims[0], kind)
    assert layers is not None
    loss, pred = _mlp.head_loss(x, layers, target, mask, kind, fused=fused)
    gx, *gw = torch.autograd.grad(loss * 1.7, [x] + [p for l in lins for p in (l.weight, l.bias)])

    xr = x.detach().clone().requires_grad_(True)
    pr = seq(xr)
    lr = _ref_loss(kind, pr, target, mask)
    gxr, *gwr = torch.autograd.grad(lr * 1.7, [xr] + [p for l in lins for p in (l.weight, l.bias)])
    torch.testing.assert_close(pred, pr.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss, lr.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gx, gxr, rtol=1e-4, atol=1e-6)
    for a, b in zip(gw, gwr):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def test_head_loss_fused_unit_seed():
    """The fused path returns its in-forward gradients unscaled for a marked unit seed (the
    training step's), and scales them for any other upstream gradient."""
    dev = torch.device("cuda")
    torch.manual_seed(3)
    dims = [64, 50, 25, 1]
    seq = torch.nn.Sequential(torch.nn.Linear(64, 50), torch.nn.ReLU(), torch.nn.Linear(50, 25), torch.nn.ReLU(),
                              torch.nn.Linear(25, 1)).to(dev)
    params = list(seq.parameters())
    x = torch.randn(33, dims[0], device=dev, requires_grad=True)
    target = torch.randn(33, 1, device=dev)
    layers = _mlp.head_loss_layers([seq], 33, 64, "mae")
    ref = None
    for seed in (_mlp.mark_unit_seed(torch.ones((), device=dev)), torch.ones((), device=dev),
                 torch.full((), 2.0, device=dev)):
        for p in params + [x]:
            p.grad = None
        loss, _ = _mlp.head_loss(x, layers, target, None, "mae", fused=True)
        torch.autograd.backward(loss, seed)
        got = [x.grad.clone()] + [p.grad.clone() for p in params]
        if ref is None:
            ref = got
        for a, b in zip(got, ref):
            torch.testing.assert_close(a, b * float(seed), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("kind", ["mae", "mse", "smooth_l1"])
@pytest.mark.parametrize("G,dims,masked", [(33, [64, 50, 50, 50, 25, 1], True), (1, [32, 16, 1], False),
                                           (100, [128, 64, 3], True), (7, [128, 50, 50, 50, 50, 25, 2], True),
                                           (5, [64, 96, 1], False)])
def test_head_loss_dx_matches_torch(kind, G, dims, masked):
    """head_loss_dx (the dx-only launch of the training step's critical path; the
    one-workgroup-per-row kernel for widths <= 64, the row-split kernel otherwise) == the
    autograd input gradient of the fp32 Linear/ReLU chain and masked mean loss."""
    dev = torch.device("cuda")
    torch.manual_seed(7 * G + len(dims))
    lins = [torch.nn.Linear(dims[i], dims[i + 1]).to(dev) for i in range(len(dims) - 1)]
    seq = []
    for i, l in enumerate(lins):
        seq.append(l)
        if i < len(lins) - 1:
            seq.append(torch.nn.ReLU())
    seq = torch.nn.Sequential(*seq)
    x = torch.randn(G, dims[0], device=dev)
    target = torch.randn(G, dims[-1], device=dev)
    mask = (torch.arange(G, device=dev) < max(1, G - 2)) if masked else None
    relu = [1] * (len(lins) - 1) + [0]
    from hydragnn_amd import _native

    dx = _native.ops().head_loss_dx(x, [l.weight.detach() for l in lins], [l.bias.detach() for l in lins], relu,
                                    target, mask, {"mse": 0, "mae": 1, "smooth_l1": 3}[kind])
    xr = x.clone().requires_grad_(True)
    (gxr,) = torch.autograd.grad(_ref_loss(kind, seq(xr), target, mask), [xr])
    torch.testing.assert_close(dx, gxr, rtol=1e-4, atol=1e-6)
