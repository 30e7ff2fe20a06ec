"""bf16 MFMA GEMM engine (csrc/bgemm.hip) against plain-torch fp32 references computed on
the same bf16-rounded operands."""
import pytest
import torch

from hydragnn_amd.ops import bgemm as bg

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _rb(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def _close(a, b, tol=2e-2):
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"max err {err} vs ref scale {ref}"


@pytest.mark.parametrize("M", [1, 200, 1000, 4097, 20000])
@pytest.mark.parametrize("bm", [64, 128, 256, 1064, 1128, 1256])
def test_nt_plain(M, bm):
    torch.manual_seed(0)
    K, Np, N = 192, 256, 250
    A, B = _rb(M, K), _rb(Np, K, scale=0.1)
    bias = torch.randn(N, device=dev)
    outf = torch.empty(M, N, device=dev)
    outb = torch.empty(M, Np, device=dev, dtype=torch.bfloat16)
    bg.nt(A, B, K, N, bias=bias, act=1, outf=outf, outb=outb, ones_col=N, bm=bm)
    ref = torch.relu(A.float() @ B.float()[:N].T + bias)
    _close(outf, ref, 1e-3)
    _close(outb[:, :N].float(), ref)
    assert (outb[:, N].float() == 1).all() and (outb[:, N + 1:].float() == 0).all()


def test_nt_epilogues():
    torch.manual_seed(1)
    M, K1, K2, Np, N, R = 3000, 128, 192, 384, 300, 700
    A, A2, B = _rb(M, K1), _rb(M, K2), _rb(Np, K1 + K2, scale=0.1)
    gate = _rb(M, Np)
    addg = torch.randn(R, N + 4, device=dev)
    idx = torch.randint(0, R, (M,), device=dev, dtype=torch.int32)
    rowvec = torch.randn(N, device=dev)
    rowdot = torch.zeros(M, device=dev)
    outf = torch.randn(M, N, device=dev)
    prev = outf.clone()
    bg.nt(A, B, K1 + K2, N, A2=A2, k1=K1, gate=gate, addg=addg, addg_idx=idx, outf=outf, beta=1.0, rowvec=rowvec,
          rowdot=rowdot)
    z = torch.cat([A, A2], 1).float() @ B.float()[:N].T + addg[idx.long(), :N]
    z = z * (gate[:, :N].float() > 0)
    _close(outf - prev, z, 1e-3)
    _close(rowdot, z @ rowvec, 1e-3)


@pytest.mark.parametrize("M", [64, 1000, 35000])
def test_tn_reduce(M):
    torch.manual_seed(2)
    Np, K1, K2 = 256, 128, 256
    G, X, X2 = _rb(M, Np), _rb(M, K1), _rb(M, K2)
    N, K = 250, K1 + 200
    out = torch.randn(N, K, device=dev)
    prev = out.clone()
    bias = torch.randn(N, device=dev)
    bprev = bias.clone()
    bg.wgrad(G, X, Np, K1 + K2, [(out, 0, bias, 5)], X2=X2, kc1=K1, beta=1.0)
    full = G.float().T @ torch.cat([X, X2], 1).float()
    _close(out - prev, full[:N, :K], 1e-3)
    _close(bias - bprev, full[:N, 5], 1e-3)


def test_tn_fused_reduce_multi_out_deterministic():
    """two destination rectangles + transposed (strided) output; the per-tile arrival
    counters are left at zero and repeated products are bitwise identical (fixed split order)"""
    torch.manual_seed(5)
    M, Np, Kp = 20000, 384, 256
    G, X = _rb(M, Np), _rb(M, Kp)
    full = G.float().T @ X.float()
    a = torch.empty(100, 200, device=dev)
    bt = torch.empty(120, 130, device=dev).T  # [130, 120] view with ldk != 1
    ba = torch.empty(100, device=dev)
    bg.wgrad(G, X, Np, Kp, [(a, 0, ba, 200), (bt, 250, None, -1, 100)])
    _close(a, full[:100, :200], 1e-3)
    _close(ba, full[:100, 200], 1e-3)
    _close(bt, full[250:380, 100:220], 1e-3)
    first = a.clone()
    for _ in range(3):
        bg.wgrad(G, X, Np, Kp, [(a, 0, ba, 200), (bt, 250, None, -1, 100)])
        assert torch.equal(a, first)
    torch.cuda.synchronize()
    for c in bg._counters.values():
        assert int(c.abs().sum()) == 0


def test_cast_weights_and_pad():
    torch.manual_seed(3)
    W = torch.randn(866, 889, device=dev)
    (wb, wt), = bg.weight_images([W])
    assert wb.shape == (896, 896) and wt.shape == (896, 896)
    assert torch.equal(wb[:866, :889], W.to(torch.bfloat16))
    assert torch.equal(wt[:889, :866], W.T.to(torch.bfloat16))
    assert (wb[866:].float() == 0).all() and (wb[:, 889:].float() == 0).all()
    x = torch.randn(100, 866, device=dev)
    g = _rb(100, 896)
    xb = bg.cast_pad(x, 896, gate=g)
    ref = x * (g[:, :866].float() > 0)
    assert torch.equal(xb[:, :866], ref.to(torch.bfloat16))
    assert (xb[:, 866].float() == 1).all() and (xb[:, 867:].float() == 0).all()


@pytest.mark.parametrize("act", [0, 1])
def test_bf16_linear_grad(act):
    torch.manual_seed(4)
    M, K, N = 5000, 866, 889
    x = torch.randn(M, K, device=dev, requires_grad=True)
    W = (torch.randn(N, K, device=dev) * 0.03).requires_grad_()
    b = torch.randn(N, device=dev, requires_grad=True)
    y = bg.bf16_linear(x, W, b, act)
    gy = torch.randn(M, N, device=dev)
    y.backward(gy)
    xr = x.detach().to(torch.bfloat16).float().requires_grad_()
    Wr = W.detach().to(torch.bfloat16).float().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = xr @ Wr.T + br
    if act == 1:
        yr = torch.relu(yr)
    yr.backward(gy)
    _close(y, yr, 1e-3)
    _close(x.grad, xr.grad, 2e-2)
    _close(W.grad, Wr.grad, 2e-2)
    _close(b.grad, br.grad, 2e-2)


def test_branch_mlp_matches_per_branch():
    """Branch-grouped head GEMMs (rows sorted by branch, tiles straddling branch boundaries,
    an empty branch) against per-branch evaluation with the same bf16 rounding points
    (BF16Linear layer by layer), and loosely against fp32."""
    torch.manual_seed(5)
    nb, dims = 4, [200, 150, 150, 3]
    seqs = []
    for _ in range(nb):
        seqs.append(torch.nn.Sequential(torch.nn.Linear(dims[0], dims[1]), torch.nn.ReLU(),
                                        torch.nn.Linear(dims[1], dims[2]), torch.nn.ReLU(),
                                        torch.nn.Linear(dims[2], dims[3])).to(dev))
    sizes = [300, 0, 77, 1000]
    bid = torch.cat([torch.full((n,), b, dtype=torch.int32) for b, n in enumerate(sizes)]).to(dev)
    x = torch.randn(bid.numel(), dims[0], device=dev, requires_grad=True)
    boff = bg.branch_offsets(bid, nb)
    assert boff.tolist() == [0, 300, 300, 377, 1377]
    y = bg.branch_mlp(x, seqs, bid, boff)
    G = torch.randn_like(y)
    (y * G).sum().backward()
    gx = x.grad.clone()
    gw = [[p.grad.clone() for p in s.parameters()] for s in seqs]

    def run_ref(bf16):
        for s in seqs:
            s.zero_grad()
        x.grad = None
        outs = []
        for b in range(nb):
            h = x[boff[b]:boff[b + 1]]
            mods = list(seqs[b])
            for i in range(0, len(mods), 2):
                lin = mods[i]
                act = 1 if i + 1 < len(mods) else 0
                if bf16:
                    h = bg.bf16_linear(h, lin.weight, lin.bias, act)
                else:
                    h = lin(h)
                    h = torch.relu(h) if act else h
            outs.append(h)
        ref = torch.cat(outs)
        (ref * G).sum().backward()
        return ref.detach(), x.grad.clone(), [[p.grad.clone() for p in s.parameters()] for s in seqs]

    def rel(a, b):
        return ((a - b).norm() / (b.norm() + 1e-12)).item()

    rb, gxb, gwb = run_ref(True)
    rf, gxf, gwf = run_ref(False)
    assert rel(y, rb) < 2e-3 and rel(y, rf) < 1e-2
    assert rel(gx, gxb) < 5e-3, rel(gx, gxb)
    assert rel(gx, gxf) < 1e-1
    for b in range(nb):
        for g, r in zip(gw[b], gwb[b]):
            if sizes[b] == 0:
                assert g.abs().max().item() == 0.0
            else:
                assert rel(g, r) < 5e-3, (b, g.shape, rel(g, r))
