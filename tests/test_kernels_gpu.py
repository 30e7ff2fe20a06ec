"""HIP kernel numerics vs plain-PyTorch fp32 references (run on MI355X: -m gpu).

Every op is checked forward AND backward against the CPU composite path of the
same op (ops/*.py), which is built only from standard torch ops.
"""
import math

import pytest
import torch

from hydragnn_amd import _native
from hydragnn_amd.ops import segment as seg
from hydragnn_amd.ops.attention import attention_reference, make_segments, segment_attention
from hydragnn_amd.ops.pna import composite_mode, pna_avg_deg, pna_message_aggregate, pna_weight_prep

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(N=300, E=2400, seed=0):
    g = torch.Generator().manual_seed(seed)
    dst = torch.randint(0, N, (E,), generator=g)
    dst[:5] = N - 1  # a heavier node
    src = torch.randint(0, N, (E,), generator=g)
    order = torch.argsort(dst, stable=True)
    dst, src = dst[order], src[order]
    # leave some isolated nodes
    keep = (dst % 17) != 3
    dst, src = dst[keep], src[keep]
    dst_si = seg.SegIndex.from_index(dst, N, sorted_=True)
    src_si = seg.SegIndex.from_index(src, N, sorted_=False)
    return dst_si, src_si, dst.numel()


def test_native_loaded():
    assert _native.load(), _native._error


@pytest.mark.parametrize("F", [1, 3, 8, 64, 130, 866])
def test_segment_sum_gather(F):
    dst_si, src_si, E = _graph()
    x = torch.randn(E, F, dtype=torch.float32)
    for si in (dst_si, src_si):
        ref = seg.segment_sum(x.clone().requires_grad_(), si)
        xg = x.to(DEV).requires_grad_()
        out = seg.segment_sum(xg, si.to(DEV))
        torch.testing.assert_close(out.cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
        g = torch.randn_like(ref)
        out.backward(g.to(DEV))
        torch.testing.assert_close(xg.grad.cpu(), g[si.index64], rtol=0, atol=0)
        # gather + its backward (= segment sum over the same SegIndex)
        xn = torch.randn(si.num_segments, F)
        xng = xn.to(DEV).requires_grad_()
        go = seg.gather(xng, si.to(DEV))
        torch.testing.assert_close(go.cpu(), xn[si.index64])
        gg = torch.randn(E, F)
        go.backward(gg.to(DEV))
        ref_g = torch.zeros_like(xn).index_add_(0, si.index64, gg)
        torch.testing.assert_close(xng.grad.cpu(), ref_g, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("view", ["dst", "src"])
def test_segment_minmax(view):
    """Native segment min / max == the CPU composite, sorted (dst) and permuted (src) CSR;
    ties (rounded values) go to the smallest row id in both."""
    dst_si, src_si, E = _graph()
    si = dst_si if view == "dst" else src_si
    x = torch.randn(E, 16).mul(4).round()  # many ties
    for is_max in (True, False):
        f = seg.segment_max if is_max else seg.segment_min
        xc = x.clone().requires_grad_()
        ref = f(xc, si)
        xg = x.to(DEV).requires_grad_()
        out = f(xg, si.to(DEV))
        torch.testing.assert_close(out.cpu(), ref.detach())
        g = torch.randn_like(ref)
        ref.backward(g)
        out.backward(g.to(DEV))
        torch.testing.assert_close(xg.grad.cpu(), xc.grad)


@pytest.mark.parametrize("F", [8, 64, 6])
@pytest.mark.parametrize("with_edges", [True, False])
def test_pna_fused_vs_composite(F, with_edges):
    dst_si, src_si, E = _graph(N=257, E=3000, seed=F)
    N = dst_si.num_segments
    deg = torch.bincount(dst_si.degree().long(), minlength=12).double()
    avg = pna_avg_deg(deg)
    x = torch.randn(N, F)
    AB = torch.randn(N, 2 * F)
    C = torch.randn(E, F) if with_edges else None
    G = torch.randn(E, F) if with_edges else None
    ins = [t for t in (x, AB, C, G) if t is not None]
    cpu = [t.clone().requires_grad_() for t in ins]
    gpu = [t.to(DEV).requires_grad_() for t in ins]
    if with_edges:
        zc = pna_message_aggregate(cpu[0], cpu[1], cpu[2], cpu[3], dst_si, src_si, avg)
        zg = pna_message_aggregate(gpu[0], gpu[1], gpu[2], gpu[3], dst_si.to(DEV), src_si.to(DEV), avg)
    else:
        zc = pna_message_aggregate(cpu[0], cpu[1], None, None, dst_si, src_si, avg)
        zg = pna_message_aggregate(gpu[0], gpu[1], None, None, dst_si.to(DEV), src_si.to(DEV), avg)
    assert zg.shape == (N, 17 * F)
    torch.testing.assert_close(zg.cpu(), zc.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(zc)
    zc.backward(g)
    zg.backward(g.to(DEV))
    for a, b in zip(gpu, cpu):
        torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=2e-4, atol=2e-4)


@pytest.mark.parametrize("F,d", [(64, 1), (32, 3), (5, 2)])
def test_pna_weight_prep(F, d):
    g = torch.Generator().manual_seed(F + d)
    ps = [torch.randn(*sh, generator=g) for sh in ((F, 3 * F), (F,), (F, d + F), (F,))]
    outs_g = [torch.randn(*sh, generator=g) for sh in ((2 * F, F), (F, F), (F, d), (F,))]

    def run(dev, composite):
        xs = [p.detach().clone().to(dev).requires_grad_(True) for p in ps]
        with composite_mode(composite):
            outs = pna_weight_prep(*xs)
        sum((o * go.to(dev)).sum() for o, go in zip(outs, outs_g)).backward()
        return [o.detach().cpu() for o in outs], [x.grad.cpu() for x in xs]

    (o_ref, g_ref), (o_hip, g_hip) = run("cpu", True), run(DEV, False)
    for a, b in zip(o_hip + g_hip, o_ref + g_ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("D", [4, 8, 16, 32, 64])
@pytest.mark.parametrize("scope", ["batch", "graph"])
def test_attention(D, scope):
    H = 4
    F = H * D
    torch.manual_seed(D)
    ptr = torch.tensor([0, 37, 100, 101, 180, 300])
    N = 303  # 3 padding rows
    seg_id, seg_ptr = make_segments(N, scope, ptr=ptr, num_valid=300)
    qkv = torch.randn(N, 3 * F)
    qc = qkv.clone().requires_grad_()
    ref = attention_reference(qc, H, seg_id)
    qg = qkv.to(DEV).requires_grad_()
    out = segment_attention(qg, H, seg_id.to(DEV), seg_ptr.to(DEV))
    # 8-wide heads: the MFMA kernels of csrc/attention8.hip; the rest: packed-fp32 VALU
    assert ("Attn8" in type(out.grad_fn).__name__) == (D == 8), type(out.grad_fn).__name__
    torch.testing.assert_close(out.cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.to(DEV))
    torch.testing.assert_close(qg.grad.cpu(), qc.grad, rtol=2e-4, atol=2e-4)


def test_attention_long_sequence():
    """Batch scope over a few thousand tokens (the OC20 GPS regime), D=8."""
    H, D, N = 8, 8, 2500
    seg_id, seg_ptr = make_segments(N, "batch")
    qkv = torch.randn(N, 3 * H * D)
    ref = attention_reference(qkv, H, seg_id)
    out = segment_attention(qkv.to(DEV), H, seg_id.to(DEV), seg_ptr.to(DEV))
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("splits", [1, 2, 3, 7, 16])
@pytest.mark.parametrize("scope", ["batch", "graph"])
def test_attention_key_splits(splits, scope):
    """Every split count (explicit, bypassing the heuristic) gives the same fwd/bwd."""
    from hydragnn_amd import _native

    H, D = 8, 8
    F = H * D
    torch.manual_seed(splits)
    ptr = torch.tensor([0, 300, 301, 700, 1333])
    N = 1400
    seg_id, seg_ptr = make_segments(N, scope, ptr=ptr, num_valid=1333)
    qkv = torch.randn(N, 3 * F)
    qc = qkv.clone().requires_grad_()
    ref = attention_reference(qc, H, seg_id)
    g = torch.randn_like(ref)
    ref.backward(g)
    scale = 1.0 / D ** 0.5
    ops = _native.ops()
    qd, sid, sptr = qkv.to(DEV), seg_id.to(DEV), seg_ptr.to(DEV)
    O, LSE = ops.attn_fwd(qd, sid, sptr, H, scale, N, splits)
    torch.testing.assert_close(O.cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    dqkv = ops.attn_bwd(g.to(DEV), qd, O, LSE, sid, sptr, H, scale, N, splits)
    torch.testing.assert_close(dqkv.cpu(), qc.grad, rtol=2e-4, atol=2e-4)


def test_fused_adamw_matches_cpu():
    from hydragnn_amd.optim.adamw import FusedAdamW

    torch.manual_seed(0)
    ps = [torch.randn(3000), torch.randn(17, 5), torch.randn(1)]
    cpu = [p.clone().requires_grad_() for p in ps]
    gpu = [p.to(DEV).requires_grad_() for p in ps]
    oc = FusedAdamW(cpu, lr=1e-2, weight_decay=0.05)
    og = FusedAdamW(gpu, lr=1e-2, weight_decay=0.05)
    ref = torch.optim.AdamW([p.clone().requires_grad_() for p in ps], lr=1e-2, weight_decay=0.05)
    for it in range(4):
        grads = [torch.randn_like(p) for p in ps]
        for p, g in zip(cpu, grads):
            p.grad = g.clone()
        for p, g in zip(gpu, grads):
            p.grad = g.to(DEV)
        for p, g in zip(ref.param_groups[0]["params"], grads):
            p.grad = g.clone()
        oc.step()
        og.step()
        ref.step()
    for a, b, c in zip(gpu, cpu, ref.param_groups[0]["params"]):
        torch.testing.assert_close(a.detach().cpu(), b.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(b.detach(), c.detach(), rtol=1e-5, atol=1e-6)


def test_fused_adamw_guard_and_step_counts():
    """A NaN guard skips the whole update (parameters, moments, step counts) and is counted;
    the launch's last block advances every used parameter's step count exactly once (one
    launch, no separate counter kernel)."""
    from hydragnn_amd.optim.adamw import FusedAdamW

    torch.manual_seed(1)
    ps = [torch.randn(5000, device=DEV).requires_grad_(), torch.randn(3, 3, device=DEV).requires_grad_()]
    opt = FusedAdamW(ps, lr=1e-2)
    for p in ps:
        p.grad = torch.randn_like(p)
    opt.step()
    before = [p.detach().clone() for p in ps]
    assert [float(opt.state[p]["step"]) for p in ps] == [1.0, 1.0]
    opt.guard = torch.tensor(float("nan"), device=DEV)
    opt.step()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(ps, before))
    assert [float(opt.state[p]["step"]) for p in ps] == [1.0, 1.0]
    assert opt.skipped_steps() == 1
    opt.guard = torch.tensor(0.5, device=DEV)
    for _ in range(3):
        opt.step()
    assert [float(opt.state[p]["step"]) for p in ps] == [4.0, 4.0]
    assert not any(torch.equal(a, b) for a, b in zip(ps, before))


@pytest.mark.parametrize("F", [64, 7, 300])
@pytest.mark.parametrize("masked", [False, True])
def test_batchnorm_fused(F, masked):
    from hydragnn_amd.ops.norm import _masked_batch_norm, batch_norm

    torch.manual_seed(F)
    N = 1000
    x = torch.randn(N, F) * 3 + 1
    nv = 777 if masked else None
    bn_c = torch.nn.BatchNorm1d(F)
    with torch.no_grad():
        bn_c.weight.uniform_(0.5, 1.5)
        bn_c.bias.uniform_(-0.5, 0.5)
    bn_g = torch.nn.BatchNorm1d(F).to(DEV)
    bn_g.load_state_dict(bn_c.state_dict())
    xc = x.clone().requires_grad_()
    yc = _masked_batch_norm(xc, bn_c, nv) if masked else bn_c(xc)
    xg = x.to(DEV).requires_grad_()
    nvg = torch.tensor(nv, dtype=torch.int32, device=DEV) if masked else None
    yg = batch_norm(xg, bn_g, nvg)
    torch.testing.assert_close(yg.cpu(), yc.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn(N, F)
    yc.backward(g)
    yg.backward(g.to(DEV))
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn_g.weight.grad.cpu(), bn_c.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bn_g.bias.grad.cpu(), bn_c.bias.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bn_g.running_mean.cpu(), bn_c.running_mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn_g.running_var.cpu(), bn_c.running_var, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("fused", [False, True])
def test_batchnorm_huge_activations(fused):
    """|x| ~ 1e21 (an fp32 sum of squares overflows; torch's own fp32 BatchNorm returns all
    zeros here): the fp64-accumulated statistics give the exact normalisation, no inf/NaN
    (both the standalone and the fused BN kernels)."""
    from hydragnn_amd.ops.norm import batch_norm, norm_add

    torch.manual_seed(0)
    N, F = 700, 20
    x = (torch.randn(N, F) + 0.5) * 1e21
    bn_c = torch.nn.BatchNorm1d(F)
    bn_g = torch.nn.BatchNorm1d(F).to(DEV)
    xd = x.double()
    yc = ((xd - xd.mean(0)) / torch.sqrt(xd.var(0, unbiased=False) + bn_c.eps)).float()
    xg = x.to(DEV)
    if fused:
        from hydragnn_amd.models.layers import BatchNorm

        m = BatchNorm(F).to(DEV)
        yg = norm_add(xg, m, None, relu=False)
    else:
        yg = batch_norm(xg, bn_g, None)
    assert torch.isfinite(yg).all()
    torch.testing.assert_close(yg.cpu(), yc.detach(), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("M,O,I", [(23000, 64, 64), (5000, 64, 1088), (3000, 7, 130), (1500, 192, 64)])
def test_linear_wgrad(M, O, I):
    from hydragnn_amd.ops.linear import linear, linear_sum

    torch.manual_seed(M)
    x = torch.randn(M, I)
    W = torch.randn(O, I) / I ** 0.5
    b = torch.randn(O)
    xc, Wc, bc = (t.clone().requires_grad_() for t in (x, W, b))
    xg, Wg, bg = (t.to(DEV).requires_grad_() for t in (x, W, b))
    yc = torch.nn.functional.linear(xc, Wc, bc)
    yg = linear(xg, Wg, bg)
    g = torch.randn(M, O)
    yc.backward(g)
    yg.backward(g.to(DEV))
    torch.testing.assert_close(yg.detach().cpu(), yc.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(Wg.grad.cpu(), Wc.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bg.grad.cpu(), bc.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(xg.grad.cpu(), xc.grad, rtol=1e-4, atol=1e-4)
    # two-input sum form
    x2 = torch.randn(M, 5)
    W2 = torch.randn(O, 5)
    W2c, W2g = W2.clone().requires_grad_(), W2.to(DEV).requires_grad_()
    Wc.grad = None
    Wg.grad = None
    yc = torch.nn.functional.linear(xc, Wc, bc) + x2 @ W2c.t()
    yg = linear_sum([(xg, Wg), (x2.to(DEV), W2g)], bg)
    yc.backward(g)
    yg.backward(g.to(DEV))
    torch.testing.assert_close(W2g.grad.cpu(), W2c.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(Wg.grad.cpu(), Wc.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("lmax_node,lmax_sh", [(1, 2), (2, 3), (0, 1)])
def test_tp_uvu_native_matches_reference(lmax_node, lmax_sh):
    """HIP uvu tensor product (MACE message) fwd/bwd == the einsum reference."""
    from hydragnn_amd.ops import o3

    torch.manual_seed(lmax_node * 10 + lmax_sh)
    ir1 = o3.Irreps.natural(24, lmax_node)
    ir2 = o3.Irreps.sh(lmax_sh)
    out_ir, ins = o3.tp_uvu_instructions(ir1, ir2, o3.Irreps.natural(1, 3))
    tp = o3.TensorProductUVU(ir1, ir2, out_ir, ins)
    assert tp.native_ok
    E = 300
    x1 = torch.randn(E, ir1.dim, dtype=torch.float32)
    x2 = torch.randn(E, ir2.dim, dtype=torch.float32)
    w = torch.randn(E, tp.weight_numel, dtype=torch.float32)
    ref_in = [t.clone().requires_grad_() for t in (x1, x2, w)]
    ref = tp.forward_reference(*ref_in)
    tpg = tp.to(DEV)
    gin = [t.to(DEV).requires_grad_() for t in (x1, x2, w)]
    out = tpg(*gin)
    torch.testing.assert_close(out.cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.to(DEV))
    for a, b in zip(gin, ref_in):
        torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("y_grad", [True, False])
@pytest.mark.parametrize("lmax_node,lmax_sh", [(1, 2), (2, 3)])
def test_tp_conv_fused_matches_composite(lmax_node, lmax_sh, y_grad):
    """Fused MACE convolution (gather x1[src] -> uvu TP -> segment sum by dst, one launch
    each way) == segment_sum(TP(gather)) reference, values and all three gradients (and,
    for edge attributes without a gradient, the backward variant that skips gY)."""
    from hydragnn_amd.ops import o3
    from hydragnn_amd.ops import segment as seg

    torch.manual_seed(7 + lmax_node)
    ir1 = o3.Irreps.natural(32, lmax_node)
    ir2 = o3.Irreps.sh(lmax_sh)
    out_ir, ins = o3.tp_uvu_instructions(ir1, ir2, o3.Irreps.natural(1, 3))
    tp = o3.TensorProductUVU(ir1, ir2, out_ir, ins).to(DEV)
    N, E = 90, 700
    src = torch.randint(0, N, (E,))
    dst = torch.sort(torch.randint(0, N, (E,))).values
    src_si = seg.SegIndex.from_index(src.to(DEV), N, sorted_=False)
    dst_si = seg.SegIndex.from_index(dst.to(DEV), N, sorted_=True)
    x1 = torch.randn(N, ir1.dim, device=DEV, requires_grad=True)
    y = torch.randn(E, ir2.dim, device=DEV, requires_grad=y_grad)
    w = torch.randn(E, tp.weight_numel, device=DEV, requires_grad=True)
    out = tp.conv(x1, y, w, src_si, dst_si)
    xr, yr, wr = [t.detach().double().cpu().requires_grad_() for t in (x1, y, w)]
    tp64 = o3.TensorProductUVU(ir1, ir2, out_ir, ins).double()
    ref = torch.zeros(N, out.shape[1], dtype=torch.float64).index_add_(
        0, dst, tp64.forward_reference(xr[src], yr, wr))
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(ref)
    out.backward(g.float().to(DEV))
    ref.backward(g)
    for a, b in zip((x1, y, w), (xr, yr, wr)):
        if a is y and not y_grad:
            assert y.grad is None
            continue
        torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("correlation,lmax_out", [(2, 1), (3, 1), (3, 2)])
def test_symmetric_contraction_native(correlation, lmax_out):
    """MACE product basis kernel (csrc/symcon.hip) == the torch Horner path (fp64 CPU),
    outputs, d x and the per-element weight gradients."""
    from hydragnn_amd.ops import o3

    torch.manual_seed(correlation * 10 + lmax_out)
    H, ne, N = 32, 5, 300
    irreps_out = o3.Irreps.natural(H, lmax_out)
    sc = o3.SymmetricContraction(2, irreps_out, correlation, H, ne)
    elem = torch.randint(0, ne, (N,))
    x = torch.randn(N, H, 9)
    sc64 = o3.SymmetricContraction(2, irreps_out, correlation, H, ne).double()
    sc64.load_state_dict(sc.state_dict())
    scg = sc.to(DEV)
    xg = x.to(DEV).requires_grad_()
    esi = o3.element_index(elem.to(DEV), ne)
    assert scg.native_ok(xg, esi)
    out = scg(xg, esi)
    xr = x.double().requires_grad_()
    ref = sc64(xr, elem)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(ref)
    out.backward(g.float().to(DEV))
    ref.backward(g)
    torch.testing.assert_close(xg.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-3)
    for a, b in zip(scg.parameters(), sc64.parameters()):
        torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("G,dims,relus", [(33, [64, 50, 50, 50, 25, 1], [1, 1, 1, 1, 0]),
                                          (203, [7, 128, 3], [1, 0]), (1, [16, 8], [1])])
def test_fused_mlp_chain(G, dims, relus):
    from torch import nn

    from hydragnn_amd.ops.mlp import sequential_chain

    torch.manual_seed(G)
    mods = []
    for i, r in enumerate(relus):
        mods.append(nn.Linear(dims[i], dims[i + 1]))
        if r:
            mods.append(nn.ReLU())
    seq = nn.Sequential(*mods[:2]), nn.Sequential(*mods[2:])
    x = torch.randn(G, dims[0])
    go = torch.randn(G, dims[-1])

    def run(dev):
        for s in seq:
            s.to(dev).zero_grad()
        xx = x.clone().to(dev).requires_grad_(True)
        out = sequential_chain(xx, *seq) if dev == DEV else seq[1](seq[0](xx))
        (out * go.to(dev)).sum().backward()
        grads = [p.grad.cpu().clone() for s in seq for p in s.parameters()]
        return out.detach().cpu(), xx.grad.cpu(), grads

    o_r, dx_r, g_r = run("cpu")
    o_h, dx_h, g_h = run(DEV)
    torch.testing.assert_close(o_h, o_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dx_h, dx_r, rtol=1e-5, atol=1e-5)
    for a, b in zip(g_h, g_r):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("E,F,K,L", [(3000, 64, 6, 3), (257, 70, 8, 1)])
def test_radial_features(E, F, K, L):
    from torch import nn

    from hydragnn_amd.ops.geometry import BesselBasis
    from hydragnn_amd.ops.radial import radial_features

    torch.manual_seed(E)

    class _C(nn.Module):
        def __init__(self):
            super().__init__()
            self.rbf_emb = nn.Sequential(nn.Linear(K, F), nn.ReLU())
            self.rbf_lin = nn.Linear(K, F, bias=False)

    basis = BesselBasis(K, cutoff=5.0, envelope_exponent=5)
    convs = nn.ModuleList([_C() for _ in range(L)])
    dist = 0.3 + torch.rand(E) * 5.7  # some edges beyond the cutoff
    gos = [(torch.randn(E, F), torch.randn(E, F)) for _ in range(L)]

    def run(dev):
        basis.to(dev).zero_grad()
        convs.to(dev).zero_grad()
        d = dist.clone().to(dev).requires_grad_(True)
        outs = radial_features(d, basis, list(convs))
        loss = sum((r * a.to(dev)).sum() + (g * b.to(dev)).sum() for (r, g), (a, b) in zip(outs, gos))
        loss.backward()
        grads = [d.grad, basis.freq.grad] + [p.grad for p in convs.parameters()]
        return [t.detach().cpu() for rg in outs for t in rg], [g.detach().cpu().clone() for g in grads]

    o_r, g_r = run("cpu")
    o_h, g_h = run(DEV)
    for a, b in zip(o_h, o_r):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)
    for a, b in zip(g_h, g_r):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3 * max(1.0, float(b.abs().max())))


@pytest.mark.parametrize("shapes,F,rows", [([64, 1], 64, 23117), ([6], 64, 1000), ([3, 5, 7], 100, 130),
                                           ([124, 64], 96, 777), ([1], 1, 65)])
def test_edge_linear_fwd(shapes, F, rows):
    """One-pass small-K concat-linear (csrc/linear.hip) vs fp32 torch, incl. a strided input."""
    from hydragnn_amd import _native

    torch.manual_seed(rows)
    big = torch.randn(rows, sum(shapes) + 3, device=DEV)
    xs, off = [], 0
    for k in shapes:
        xs.append(big[:, off:off + k])  # row stride > width (column slices of one buffer)
        off += k
    ws = [torch.randn(F, k, device=DEV) for k in shapes]
    b = torch.randn(F, device=DEV)
    y = _native.ops().edge_linear_fwd(xs, ws, b)
    ref = sum(x.double() @ w.double().t() for x, w in zip(xs, ws)) + b.double()
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-4)
    y0 = _native.ops().edge_linear_fwd(xs, ws, None)
    torch.testing.assert_close(y0.double(), ref - b.double(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("F", [8, 64, 3])
def test_gather_mul_sum_native(F):
    """Native gather-multiply-segment-sum (+ its gradient ops, incl. a double backward) vs the
    fp32 CPU composite."""
    from hydragnn_amd.ops import segment as seg

    torch.manual_seed(F)
    N, E = 300, 2500
    src = torch.randint(0, N, (E,))
    dst = torch.sort(torch.randint(0, N, (E,))).values
    x = torch.randn(N, F)
    w = torch.randn(E, F)

    def run(dev):
        gsi = seg.SegIndex.from_index(src.to(dev), N)
        ssi = seg.SegIndex.from_index(dst.to(dev), N, sorted_=True)
        xx = x.to(dev).requires_grad_()
        ww = w.to(dev).requires_grad_()
        out = seg.gather_mul_sum(xx, ww, gsi, ssi)
        gx, gw = torch.autograd.grad(out.pow(2).sum(), (xx, ww), create_graph=True)
        (ggx,) = torch.autograd.grad(gw.pow(2).sum() + gx.sum(), xx)
        return [t.detach().cpu() for t in (out, gx, gw, ggx)]

    for a, b in zip(run(DEV), run("cpu")):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("lmax", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("normalize", [True, False])
def test_spherical_harmonics_native(lmax, normalize):
    """One-launch SH kernel (+ dual-number backward) vs the fp64 composite recurrences."""
    from hydragnn_amd.ops import o3

    torch.manual_seed(lmax)
    v = torch.randn(3000, 3, dtype=torch.float64)
    v[0] = 0.0  # zero vector: finite output and gradient with eps
    eps = 1e-9
    vd = v.clone().requires_grad_()
    ref = o3.spherical_harmonics(lmax, vd, normalize=normalize, eps=eps)
    g = torch.randn_like(ref)
    vg = v.float().to(DEV).requires_grad_()
    out = o3.spherical_harmonics(lmax, vg, normalize=normalize, eps=eps)
    scale = 1.0 if normalize else float(v.norm(dim=1).max()) ** lmax
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-5 * scale)
    if lmax == 0:  # Y_00 is a constant: no gradient path in the composite
        return
    ref.backward(g)
    out.backward(g.float().to(DEV))
    sel = slice(1, None)  # the zero vector's gradient is eps-dominated
    torch.testing.assert_close(vg.grad.double().cpu()[sel], vd.grad[sel], rtol=1e-3, atol=1e-3 * max(1.0, scale))


def test_edge_basis_native():
    """Gaussian smearing, sinc expansion and cosine cutoff kernels (fwd + d/dd) vs fp64 torch."""
    import math

    from hydragnn_amd.ops import geometry as geo

    torch.manual_seed(7)
    d = torch.rand(5000, dtype=torch.float64) * 6.0 + 0.05
    gs = geo.GaussianSmearing(0.0, 5.0, 50).to(DEV)
    cases = [
        (lambda t: gs(t), lambda t: torch.exp(gs.coeff * (t.view(-1, 1) - gs.offset.double().cpu().view(1, -1)) ** 2)),
        (lambda t: geo.sinc_expansion(t, 8, 5.0),
         lambda t: torch.sin(t.unsqueeze(-1) * (torch.arange(8, dtype=t.dtype) + 1) * math.pi / 5.0) / t.unsqueeze(-1)),
        (lambda t: geo.cosine_cutoff(t, 5.0, masked=True),
         lambda t: torch.where(t < 5.0, 0.5 * (torch.cos(math.pi * t / 5.0) + 1), torch.zeros_like(t))),
        (lambda t: geo.cosine_cutoff(t, 5.0, masked=False), lambda t: 0.5 * (torch.cos(math.pi * t / 5.0) + 1)),
    ]
    for f_gpu, f_ref in cases:
        dr = d.clone().requires_grad_()
        ref = f_ref(dr)
        g = torch.randn_like(ref)
        ref.backward(g)
        dg = d.float().to(DEV).requires_grad_()
        out = f_gpu(dg)
        out.backward(g.float().to(DEV))
        torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(dg.grad.double().cpu(), dr.grad, rtol=1e-3, atol=1e-3)


def test_gather_mul_sum_slack_limit():
    """Static-capacity radius graph (ops/radius.interaction_graph_static): the slack slots
    past the real edges all belong to the last (padding) receiver.  With the CSR limit the
    native gather-multiply-sum skips them: rows before it match the reference exactly, and
    the launch time does not grow with the slack (it summed the slack serially before)."""
    import time

    torch.manual_seed(5)
    N, F, deg = 2048, 64, 8
    E = N * deg
    src = torch.randint(0, N - 1, (E,), dtype=torch.int32)
    dst = torch.arange(N - 1, dtype=torch.int32).repeat_interleave(deg)[:E]
    dst = torch.cat([dst, torch.full((E - dst.numel(),), N - 1, dtype=torch.int32)])
    x = torch.randn(N, F, device=DEV)

    def build(slack):
        s_src = torch.cat([src, torch.full((slack,), N - 1, dtype=torch.int32)]).to(DEV)
        s_dst = torch.cat([dst, torch.full((slack,), N - 1, dtype=torch.int32)]).to(DEV)
        cnt = torch.bincount(dst.long(), minlength=N).to(torch.int32)
        rp = torch.cat([cnt.new_zeros(1), torch.cumsum(cnt, 0, dtype=torch.int32)]).to(DEV)
        lim = rp[N:N + 1].clone()
        rp[N] = E + slack
        w = torch.randn(E + slack, F, device=DEV)
        w[E:] = 1.0
        return seg.SegIndex(s_src, rp.clone(), None, N), seg.SegIndex(s_dst, rp, None, N, lim), w

    gsi0, ssi0, w0 = build(0)
    ref = seg.gather_mul_sum(x, w0, gsi0, ssi0)
    times = {}
    for slack in (0, 400_000):
        gsi, ssi, w = build(slack)
        w[:E] = w0[:E]
        out = seg.gather_mul_sum(x, w, gsi, ssi)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(50):
            seg.gather_mul_sum(x, w, gsi, ssi)
        torch.cuda.synchronize()
        times[slack] = (time.perf_counter() - t) / 50
    assert times[400_000] < 2.0 * times[0] + 20e-6, times


def test_relu_rowmask_matches_torch():
    """Between-layer ReLU + padding-row zeroing in one launch each way (models/base.py
    _act_zero_rows, csrc/conv_misc.hip relu_rowmask) == relu then torch.where."""
    from hydragnn_amd.models.base import _act_zero_rows, _zero_rows

    g = torch.Generator().manual_seed(3)
    x = torch.randn(301, 64, generator=g).cuda().requires_grad_(True)
    keep = (torch.rand(301, generator=g) > 0.2).cuda()
    y = _act_zero_rows(torch.nn.ReLU(), x, keep)
    assert "ReluRowMask" in type(y.grad_fn).__name__
    xr = x.detach().clone().requires_grad_(True)
    yr = _zero_rows(torch.relu(xr), keep)
    torch.testing.assert_close(y, yr, rtol=0, atol=0)
    go = torch.randn(301, 64, generator=g).cuda()
    y.backward(go)
    yr.backward(go)
    torch.testing.assert_close(x.grad, xr.grad, rtol=0, atol=0)


def test_segment_mean_native_matches_cpu_with_limit_and_grad():
    """segment_mean on the GPU (division fused into the segment-sum kernel, ops/segment.py
    _SegMean) == the CPU composite, with a padded tail skipped by the limit, values and the
    input gradient (also to second order, as force training differentiates it twice)."""
    from hydragnn_amd.ops import segment as seg

    g = torch.Generator().manual_seed(11)
    N, S = 500, 37
    idx = torch.sort(torch.randint(0, S - 1, (N,), generator=g)).values
    idx[-40:] = S - 1  # the padding segment
    x = torch.randn(N, 24, generator=g, dtype=torch.float64)
    x[-40:] = 0.0
    lim = torch.tensor([N - 40], dtype=torch.int32)
    si_c = seg.SegIndex.from_index(idx.int(), S, sorted_=True)
    xc = x.clone().requires_grad_(True)
    ref = seg.segment_mean(xc, si_c)
    go = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (gr,) = torch.autograd.grad((ref * go).sum(), xc, create_graph=True)
    dev = torch.device("cuda")
    si_d = seg.SegIndex.from_index(idx.int().to(dev), S, sorted_=True)
    xd = x.float().to(dev).requires_grad_(True)
    out = seg.segment_mean(xd, si_d, limit=lim.to(dev))
    assert "SegMean" in type(out.grad_fn).__name__
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    (gd,) = torch.autograd.grad((out * go.float().to(dev)).sum(), xd, create_graph=True)
    torch.testing.assert_close(gd.double().cpu()[:-40], gr.detach()[:-40], rtol=1e-5, atol=1e-6)
    # the mean is linear: its gradient does not depend on x (no second-order term), and the
    # create_graph backward must not fail (force training differentiates through it twice)
    if gd.requires_grad:
        h = torch.randn(gd.shape, generator=g)
        (ggd,) = torch.autograd.grad((gd * h.to(dev)).sum(), xd, allow_unused=True)
        assert ggd is None or torch.all(ggd == 0)
