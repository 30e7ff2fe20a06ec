"""CPU reference checks of the op layer (composite paths) against naive loops."""
import math

import torch

from hydragnn_amd.ops import segment as seg
from hydragnn_amd.ops.attention import attention_reference, make_segments
from hydragnn_amd.ops.pna import pna_avg_deg, pna_message_aggregate


def _naive_seg(x, idx, N, fn):
    out = []
    for n in range(N):
        rows = x[idx == n]
        out.append(fn(rows) if rows.shape[0] else torch.zeros(x.shape[1]))
    return torch.stack(out)


def test_segment_reductions_match_naive():
    torch.manual_seed(0)
    N, E, F = 20, 90, 5
    idx = torch.randint(0, N, (E,))
    idx[idx == 3] = 4  # node 3 isolated
    x = torch.randn(E, F)
    si = seg.SegIndex.from_index(idx, N)
    torch.testing.assert_close(seg.segment_sum(x, si), _naive_seg(x, idx, N, lambda r: r.sum(0)))
    torch.testing.assert_close(seg.segment_mean(x, si), _naive_seg(x, idx, N, lambda r: r.mean(0)))
    torch.testing.assert_close(seg.segment_max(x, si), _naive_seg(x, idx, N, lambda r: r.max(0).values))
    torch.testing.assert_close(seg.segment_min(x, si), _naive_seg(x, idx, N, lambda r: r.min(0).values))


def test_gather_segment_double_backward():
    torch.manual_seed(1)
    N, E = 7, 30
    idx = torch.sort(torch.randint(0, N, (E,))).values
    si = seg.SegIndex.from_index(idx, N, sorted_=True)
    x = torch.randn(N, 3, dtype=torch.float64, requires_grad=True)
    f = lambda t: seg.segment_sum(seg.gather(t, si) ** 2, si)
    assert torch.autograd.gradcheck(f, (x,))
    assert torch.autograd.gradgradcheck(f, (x,))


def test_pna_composite_semantics():
    torch.manual_seed(2)
    N, F = 9, 4
    dst = torch.tensor([0, 0, 1, 2, 2, 2, 4, 5, 5, 8])
    src = torch.tensor([1, 2, 0, 3, 4, 5, 3, 7, 8, 0])
    dsi = seg.SegIndex.from_index(dst, N, sorted_=True)
    ssi = seg.SegIndex.from_index(src, N)
    x = torch.randn(N, F)
    AB = torch.randn(N, 2 * F)
    deg_hist = torch.bincount(torch.bincount(dst, minlength=N), minlength=5).double()
    avg = pna_avg_deg(deg_hist)
    Z = pna_message_aggregate(x, AB, None, None, dsi, ssi, avg)
    m = AB[dst, :F] + AB[src, F:]
    for n in range(N):
        rows = m[dst == n]
        d = max(rows.shape[0], 1)
        if rows.shape[0]:
            mean, mn, mx = rows.mean(0), rows.min(0).values, rows.max(0).values
            var = (rows * rows).mean(0) - mean * mean
            sd = var.clamp(min=1e-5).sqrt()
            sd = torch.where(sd <= 1e-5 ** 0.5, torch.zeros_like(sd), sd)
        else:
            mean = mn = mx = sd = torch.zeros(F)
        agg = torch.cat([mean, mn, mx, sd])
        lg = math.log(d + 1)
        exp = torch.cat([x[n], agg, agg * lg / avg["log"], agg * avg["log"] / lg, agg * d / avg["lin"]])
        torch.testing.assert_close(Z[n], exp, rtol=1e-5, atol=1e-6)


def test_attention_reference_segments():
    torch.manual_seed(3)
    N, H, D = 10, 2, 4
    ptr = torch.tensor([0, 4, 10])
    sid, sptr = make_segments(N, "graph", ptr=ptr)
    qkv = torch.randn(N, 3 * H * D)
    out = attention_reference(qkv, H, sid)
    mha = torch.nn.MultiheadAttention(H * D, H, batch_first=True, bias=False)
    # graph 0 alone through a standard attention must match
    q, k, v = qkv[:4, :8], qkv[:4, 8:16], qkv[:4, 16:]
    qh, kh, vh = (t.view(4, H, D).transpose(0, 1) for t in (q, k, v))
    ref = torch.softmax(qh @ kh.transpose(1, 2) / math.sqrt(D), -1) @ vh
    torch.testing.assert_close(out[:4], ref.transpose(0, 1).reshape(4, H * D))


def test_fused_adamw_cpu_matches_torch():
    from hydragnn_amd.optim.adamw import FusedAdamW

    torch.manual_seed(4)
    ps = [torch.randn(50), torch.randn(3, 4)]
    a = [p.clone().requires_grad_() for p in ps]
    b = [p.clone().requires_grad_() for p in ps]
    oa = FusedAdamW(a, lr=0.01, weight_decay=0.1)
    ob = torch.optim.AdamW(b, lr=0.01, weight_decay=0.1)
    for _ in range(3):
        g = [torch.randn_like(p) for p in ps]
        for p, gg in zip(a, g):
            p.grad = gg.clone()
        for p, gg in zip(b, g):
            p.grad = gg.clone()
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y)


def test_mace_element_lookup_equals_one_hot():
    """Element-indexed tables gathered through an element SegIndex == the one-hot GEMMs
    (node embedding and symmetric contraction), forward and backward."""
    from hydragnn_amd.ops import o3

    torch.manual_seed(0)
    elem = torch.randint(0, 118, (57,))
    oh = torch.nn.functional.one_hot(elem, 118).float()
    si = o3.element_index(elem, 118)
    lin = o3.O3Linear(o3.Irreps([(118, 0, 1)]), o3.Irreps([(16, 0, 1)]))
    a, b = lin.lookup(si), lin(oh)
    torch.testing.assert_close(a, b)
    g = torch.randn_like(a)
    ga = torch.autograd.grad(a, lin.weight, g)[0]
    gb = torch.autograd.grad(lin(oh), lin.weight, g)[0]
    torch.testing.assert_close(ga, gb)
    sc = o3.SymmetricContraction(1, o3.Irreps([(8, 0, 1), (8, 1, -1)]), 3, 8, 118)
    x = torch.randn(57, 8, 4, requires_grad=True)
    ya, yb = sc(x, si), sc(x, oh)
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    w = sc.contractions[0].weights[0]
    gy = torch.randn_like(ya)
    torch.testing.assert_close(torch.autograd.grad(ya, w, gy)[0], torch.autograd.grad(sc(x, oh), w, gy)[0],
                               rtol=1e-5, atol=1e-6)


def test_mace_per_layer_correlation():
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.models.create import create_model

    heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 8,
                                                             "num_headlayers": 1, "dim_headlayers": [8]}}]}
    m = create_model("MACE", 1, 8, [1], 0, "", "", 0, ["graph"], heads, "relu", "mse", [1.0], 3, use_gpu=False,
                     radius=5.0, num_radial=4, max_ell=1, node_max_ell=1, avg_num_neighbors=4.0,
                     correlation=[3, 2, 1], envelope_exponent=5)
    corrs = [c.prod.symmetric_contractions.contractions[0].correlation for c in m.graph_convs]
    assert corrs == [3, 2, 1]


def test_gather_mul_sum_matches_composite_and_twice_differentiable():
    """gather_mul_sum == segment_sum(gather(x) * w) and its closed derivative family passes
    gradcheck and gradgradcheck in fp64 (the force-training double backward)."""
    from hydragnn_amd.ops import segment as seg

    torch.manual_seed(0)
    N, E, F = 7, 23, 3
    src = torch.randint(0, N, (E,))
    dst = torch.sort(torch.randint(0, N, (E,))).values
    gsi = seg.SegIndex.from_index(src, N)
    ssi = seg.SegIndex.from_index(dst, N, sorted_=True)
    x = torch.randn(N, F, dtype=torch.float64, requires_grad=True)
    w = torch.randn(E, F, dtype=torch.float64, requires_grad=True)
    ref = torch.zeros(N, F, dtype=torch.float64).index_add_(0, dst, x[src] * w)
    torch.testing.assert_close(seg.gather_mul_sum(x, w, gsi, ssi), ref)
    torch.autograd.gradcheck(lambda a, b: seg.gather_mul_sum(a, b, gsi, ssi), (x, w))
    torch.autograd.gradgradcheck(lambda a, b: seg.gather_mul_sum(a, b, gsi, ssi), (x, w))


def test_fcn_folded_scales_match_definition():
    """e3nn FullyConnectedNet: x W_i / sqrt(fan_i), silu * C between layers.  The folded
    forward (C and the next 1/sqrt(fan) as one multiply; optionally the last scale left to
    the consumer) gives the same values."""
    import math

    from hydragnn_amd.ops import o3

    torch.manual_seed(0)
    f = o3.FullyConnectedNet([10, 8, 8, 8, 6])
    x = torch.randn(5, 10)
    h = x
    for i, W in enumerate(f.weights):
        h = h @ W / math.sqrt(W.shape[0])
        if i < 3:
            h = torch.nn.functional.silu(h) * o3._SILU_C
    torch.testing.assert_close(f(x), h)
    f.defer_last_scale = True
    torch.testing.assert_close(f(x) * f.last_scale(), h)


def test_composite_attention_dense_batch_matches_masked_to_second_order():
    """Force training's composite attention on many short segments runs as a dense
    per-segment batch [S, H, L, L] (memory O(sum L^2), not O(N^2)); values, first and second
    derivatives equal the masked [H, N, N] form."""
    from hydragnn_amd.ops import attention as A

    g = torch.Generator().manual_seed(0)
    lens = [int(x) for x in torch.randint(2, 10, (20,), generator=g)]
    N, H, D = sum(lens), 4, 4
    F = H * D
    ptr = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    sid = torch.repeat_interleave(torch.arange(len(lens)), torch.tensor(lens)).int()
    qkv = torch.randn(N, 3 * F, generator=g, dtype=torch.float64, requires_grad=True)
    assert A._attention_dense_batch(qkv, H, sid, ptr, None) is not None
    from hydragnn_amd.ops.pna import composite_mode

    a = A.attention_reference(qkv, H, sid)
    with composite_mode(True):
        b = A.attention_reference(qkv, H, sid, seg_ptr=ptr)
    torch.testing.assert_close(a, b)
    w = torch.randn(a.shape, generator=g, dtype=torch.float64)
    ga, = torch.autograd.grad((a * w).sum(), qkv, create_graph=True)
    gb, = torch.autograd.grad((b * w).sum(), qkv, create_graph=True)
    torch.testing.assert_close(ga, gb)
    h = torch.randn(ga.shape, generator=g, dtype=torch.float64)
    gga, = torch.autograd.grad((ga * h).sum(), qkv)
    ggb, = torch.autograd.grad((gb * h).sum(), qkv)
    torch.testing.assert_close(gga, ggb)
