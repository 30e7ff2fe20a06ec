"""MFMA GEMM engine (``csrc/gemm.hip``) vs plain PyTorch fp32 references.

Forward ``act(sum_p X_p W_p^T + b) (+ residual)`` and the one-launch backward
(dX_p, dW_p via in-launch split-K reduction, db via the ones column, ReLU
derivative from the saved output) over node-/edge-sized row counts, odd widths,
strided (column-sliced) operands and both precisions.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref(pairs, b, act, res):
    y = sum(x.double() @ w.double().t() for x, w in pairs)
    if b is not None:
        y = y + b.double()
    if act:
        y = torch.relu(y)
    if res is not None:
        y = y + res.double()
    return y


@pytest.mark.parametrize("M,K,N", [(1, 3, 1), (37, 5, 7), (2311, 64, 64), (2311, 1088, 64), (23105, 64, 64),
                                   (23105, 7, 65), (130, 129, 200), (4096, 866, 866)])
@pytest.mark.parametrize("act", [0, 1])
def test_mm_forward_backward_fp32(M, K, N, act):
    from hydragnn_amd.ops.linear import linear

    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=DEV, requires_grad=True)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).requires_grad_()
    b = torch.randn(N, device=DEV, requires_grad=True)
    y = linear(x, W, b, act=act)
    yr = _ref([(x, W)], b, act, None)
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    xd, Wd, bd = x.detach().double().requires_grad_(), W.detach().double().requires_grad_(), \
        b.detach().double().requires_grad_()
    _ref([(xd, Wd)], bd, act, None).backward(g.double())
    tol = dict(rtol=1e-4, atol=1e-3 * max(1.0, (M / 1000) ** 0.5))
    torch.testing.assert_close(x.grad.double(), xd.grad, **tol)
    torch.testing.assert_close(W.grad.double(), Wd.grad, **tol)
    torch.testing.assert_close(b.grad.double(), bd.grad, **tol)


def test_mm_segments_residual_strided():
    """3 column blocks of one concat-linear (sliced, strided weight views) + residual."""
    from hydragnn_amd.ops.linear import linear_act

    torch.manual_seed(3)
    M, N = 3001, 48
    xs = [torch.randn(M, k, device=DEV, requires_grad=True) for k in (16, 16, 5)]
    Wfull = torch.randn(N, 37, device=DEV, requires_grad=True)
    ws = [Wfull[:, :16], Wfull[:, 16:32], Wfull[:, 32:]]
    b = torch.randn(N, device=DEV, requires_grad=True)
    res = torch.randn(M, N, device=DEV, requires_grad=True)
    y = linear_act(list(zip(xs, ws)), b, 0, residual=res)
    yr = _ref(list(zip(xs, ws)), b, 0, res)
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    xds = [x.detach().double().requires_grad_() for x in xs]
    Wd = Wfull.detach().double().requires_grad_()
    bd = b.detach().double().requires_grad_()
    rd = res.detach().double().requires_grad_()
    _ref(list(zip(xds, [Wd[:, :16], Wd[:, 16:32], Wd[:, 32:]])), bd, 0, rd).backward(g.double())
    for x, xd in zip(xs, xds):
        torch.testing.assert_close(x.grad.double(), xd.grad, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(Wfull.grad.double(), Wd.grad, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(b.grad.double(), bd.grad, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(res.grad.double(), rd.grad)


def test_mm_bf16_close_to_fp32():
    from hydragnn_amd.ops.linear import linear, precision

    torch.manual_seed(4)
    x = torch.randn(5000, 256, device=DEV)
    W = torch.randn(192, 256, device=DEV) / 16
    b = torch.randn(192, device=DEV)
    with precision("bf16"):
        y = linear(x, W, b, act=1)
    yr = _ref([(x, W)], b, 1, None)
    rel = (y.double() - yr).norm() / yr.norm()
    assert rel < 1e-2, float(rel)


def test_mm_deterministic_split_k():
    from hydragnn_amd.ops.linear import linear

    torch.manual_seed(5)
    x = torch.randn(50000, 64, device=DEV, requires_grad=True)
    W = torch.randn(64, 64, device=DEV, requires_grad=True)
    outs = []
    for _ in range(3):
        x.grad = W.grad = None
        linear(x, W).sum().backward()
        outs.append(W.grad.clone())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def test_wgrad_grouped_matches_torch():
    """Grouped deferred weight gradients (csrc/linear.hip ``linear_wgrad_grouped``): several
    problems of different shapes / strides in one launch pair, write and accumulate modes."""
    import hydragnn_amd._native as nat

    torch.manual_seed(11)
    # (I <= 16 problems take the narrow path: one lane per output row, all I columns)
    shapes = [(2311, 64, 64, True), (23105, 64, 7, True), (37, 5, 130, False), (2311, 192, 64, True),
              (4000, 33, 66, False), (1, 3, 3, True), (24571, 130, 16, True), (9001, 6, 6, False),
              (24576, 64, 1, False)]
    dys, xs, dws, dbs, acc, ref_w, ref_b = [], [], [], [], [], [], []
    for k, (M, O, I, hb) in enumerate(shapes):
        dy = torch.randn(M, O + 3, device=DEV)[:, 1:O + 1]  # strided (column-sliced) operand
        x = torch.randn(M, I, device=DEV)
        a = k % 2
        dw = torch.randn(O, I, device=DEV) if a else torch.empty(O, I, device=DEV)
        db = (torch.randn(O, device=DEV) if a else torch.empty(O, device=DEV)) if hb else torch.empty(0, device=DEV)
        ref_w.append(dy.double().t() @ x.double() + (dw.double() if a else 0))
        ref_b.append(dy.double().sum(0) + (db.double() if a else 0) if hb else None)
        dys.append(dy), xs.append(x), dws.append(dw), dbs.append(db), acc.append(a)
    nat.ops().linear_wgrad_grouped(dys, xs, dws, dbs, acc)
    for k, (M, O, I, hb) in enumerate(shapes):
        tol = dict(rtol=1e-4, atol=1e-3 * max(1.0, (M / 1000) ** 0.5))
        torch.testing.assert_close(dws[k].double(), ref_w[k], **tol)
        if hb:
            torch.testing.assert_close(dbs[k].double(), ref_b[k], **tol)

