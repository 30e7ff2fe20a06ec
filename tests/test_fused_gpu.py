"""Numerics of the fused dropout+residual+BatchNorm(+ReLU, +padding mask) kernel
(``csrc/norm_fused.hip``) against a plain fp32 PyTorch composite of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, mask_scale, bn, nv, relu, zero_pad):
    z = a * mask_scale if mask_scale is not None else a
    if b is not None:
        z = z + b
    zz = z[:nv]
    mean = zz.mean(0)
    var = zz.var(0, unbiased=False)
    y = (z - mean) * torch.rsqrt(var + bn.eps) * bn.weight + bn.bias
    if relu:
        y = torch.relu(y)
    if zero_pad:
        m = (torch.arange(z.shape[0], device=z.device) < nv).float().view(-1, 1)
        y = y * m
    return y, mean, var


@pytest.mark.parametrize("N,C", [(2816, 64), (1000, 50), (17, 8), (9000, 128)])
@pytest.mark.parametrize("resid", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.25])
@pytest.mark.parametrize("relu,zero_pad", [(False, False), (True, True)])
def test_norm_add(N, C, resid, p, relu, zero_pad):
    from hydragnn_amd import _native
    from hydragnn_amd.models.layers import BatchNorm
    from hydragnn_amd.ops import rng
    from hydragnn_amd.ops.norm import norm_add

    torch.manual_seed(N + C)
    dev = "cuda"
    nv = N - N // 7
    a = torch.randn(N, C, device=dev, requires_grad=True)
    b = torch.randn(N, C, device=dev, requires_grad=True) if resid else None
    bn = BatchNorm(C).to(dev)
    with torch.no_grad():
        bn.module.weight.uniform_(0.5, 1.5)
        bn.module.bias.uniform_(-0.5, 0.5)
    bn.train()
    rng.advance(dev)
    salt = 12345
    y = norm_add(a, bn, torch.tensor([nv], dtype=torch.int32, device=dev), residual=b, p=p, relu=relu,
                 zero_pad=zero_pad, salt=salt, training=True)
    ms = None
    if p > 0:
        ms = _native.ops().dropout_hash(torch.ones(N, C, device=dev), rng.counter(dev), salt, p)
        frac = float((ms == 0).float().mean())
        assert abs(frac - p) < 4 * (p * (1 - p) / (N * C)) ** 0.5 + 0.01, frac
    a2 = a.detach().clone().requires_grad_()
    b2 = b.detach().clone().requires_grad_() if resid else None
    w2 = bn.module.weight.detach().clone().requires_grad_()
    bb2 = bn.module.bias.detach().clone().requires_grad_()

    class _BN:
        eps = bn.module.eps
        weight = w2
        bias = bb2

    yr, mean, var = _ref(a2, b2, ms, _BN, nv, relu, zero_pad)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    # running stats (momentum 0.1, unbiased var)
    torch.testing.assert_close(bn.module.running_mean, 0.1 * mean.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.module.running_var, 0.9 + 0.1 * var.detach() * nv / (nv - 1), rtol=1e-4,
                               atol=1e-5)
    assert int(bn.module.num_batches_tracked) == 1
    g = torch.randn_like(y)
    (y * g).sum().backward()
    (yr * g).sum().backward()
    torch.testing.assert_close(a.grad, a2.grad, rtol=1e-3, atol=1e-4)
    if resid:
        torch.testing.assert_close(b.grad, b2.grad, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.module.weight.grad, w2.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.module.bias.grad, bb2.grad, rtol=1e-3, atol=1e-3)


def test_hash_dropout_graph_replay_changes_mask():
    """The counter advance is captured: every replay draws a new mask."""
    from hydragnn_amd.ops import rng

    dev = "cuda"
    x = torch.ones(4096, device=dev)
    rng.advance(dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            rng.advance(dev)
            y = rng.dropout(x, 0.5, True, 7)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rng.advance(dev)
        y = rng.dropout(x, 0.5, True, 7)
    g.replay()
    m1 = y.clone()
    g.replay()
    m2 = y.clone()
    assert not torch.equal(m1, m2)
    assert abs(float((m1 == 0).float().mean()) - 0.5) < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("padded", [False, True])
def test_native_store_assemble_matches_torch(padded):
    """csrc/assemble.hip (one launch) == the plain-torch batch assembly, field by field."""
    import numpy as np

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.data.synthetic import oc20_like

    samples = oc20_like(12, seed=3, radius=6.0, max_neighbours=8, pe_dim=4, min_atoms=5, max_atoms=20)
    for s in samples:
        s["y"] = torch.cat([s["energy"].reshape(-1), s["x"][:, 0]])
        s["y_loc"] = torch.tensor([[0, 1, 1 + s.num_nodes]])
    store = DeviceGraphStore(samples, "cuda", head_types=["graph", "node"], head_dims=[1, 1])
    idx = [3, 0, 7, 5, 11]
    N, E = store.sizes_of(idx)
    lay = store.layout(idx, Np=N + 37, Ep=E + 100, Gp=len(idx) + 1) if padded else store.layout(idx)
    dev = store.upload(idx, lay)
    a = store.assemble(dev, lay)
    b = store._assemble_torch(dev, lay)
    for k in list(store.node_keys) + list(store.edge_keys) + list(store.graph_keys) + ["edge_index", "batch", "ptr"]:
        torch.testing.assert_close(a[k], b[k], msg=k)
    for ta, tb in zip(a.targets, b.targets):
        torch.testing.assert_close(ta, tb)
    if padded:
        assert torch.equal(a.node_mask, b.node_mask) and torch.equal(a.graph_mask, b.graph_mask)
    assert np.isfinite(a.pos.cpu().numpy()).all()


@pytest.mark.parametrize("kind", ["mse", "mae", "rmse", "smooth_l1"])
@pytest.mark.parametrize("masked", [False, True])
def test_fused_masked_loss_matches_composite(kind, masked):
    """csrc/loss.hip (one launch each way) vs the torch composite of train/step.masked_loss."""
    from hydragnn_amd.ops.pna import composite_mode
    from hydragnn_amd.train.step import masked_loss

    torch.manual_seed(7)
    pred = torch.randn(333, 3, device="cuda", requires_grad=True)
    target = torch.randn(333, 3, device="cuda")
    mask = (torch.rand(333, device="cuda") > 0.3) if masked else None
    l1 = masked_loss(kind, pred, target, mask)
    (g1,) = torch.autograd.grad(l1 * 1.7, pred)
    with composite_mode(True):
        l2 = masked_loss(kind, pred, target, mask)
        (g2,) = torch.autograd.grad(l2 * 1.7, pred)
    torch.testing.assert_close(l1, l2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(g1, g2, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("C,edge,drop", [(8, False, 0.0), (20, True, 0.0), (32, True, 0.3), (5, False, 0.25)])
def test_fused_gatv2_matches_composite(C, edge, drop):
    """csrc/gat.hip (one launch forward, one backward + by-source segment sum) vs the torch
    composite GATv2 of models/gat.py: output and every gradient, incl. identical dropout
    masks (same counter hash, same element indices)."""
    import copy

    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.models.gat import GATv2Conv
    from hydragnn_amd.models.layers import Ctx
    from hydragnn_amd.ops.pna import composite_mode

    torch.manual_seed(C)
    samples = oc20_like(6, seed=C, radius=5.0, max_neighbours=10, pe_dim=2, min_atoms=20, max_atoms=40)
    store = DeviceGraphStore(samples, "cuda")
    b = store.batch(list(range(6)))
    H, F = 6, 16
    conv = GATv2Conv(F, C, heads=H, negative_slope=0.05, dropout=drop, edge_dim=1 if edge else None).cuda()
    conv.train(drop > 0)
    x = torch.randn(b.num_nodes, F, device="cuda", requires_grad=True)
    ea = torch.rand(b.edge_index.shape[1], 1, device="cuda") if edge else None
    ctx = Ctx(dst_si=b.dst_si, src_si=b.src_si, edge_attr=ea)
    out1, _ = conv(x, None, ctx)
    g = torch.randn_like(out1)
    params = [x] + [p for p in conv.parameters()]
    gr1 = torch.autograd.grad(out1, params, g, allow_unused=True)
    with composite_mode(True):
        out2, _ = conv(x, None, ctx)
        gr2 = torch.autograd.grad(out2, params, g, allow_unused=True)
    torch.testing.assert_close(out1, out2, rtol=1e-4, atol=1e-5)
    for a, c in zip(gr1, gr2):
        if a is None or c is None:
            assert a is None and c is None
            continue
        torch.testing.assert_close(a, c, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("edge", [False, True])
def test_fused_cgconv_gate_matches_composite(edge):
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.models.cgcnn import CGConv
    from hydragnn_amd.models.layers import Ctx
    from hydragnn_amd.ops.pna import composite_mode

    torch.manual_seed(1)
    samples = oc20_like(6, seed=2, radius=5.0, max_neighbours=10, pe_dim=2, min_atoms=20, max_atoms=40)
    b = DeviceGraphStore(samples, "cuda").batch(list(range(6)))
    C = 24
    conv = CGConv(C, dim=3 if edge else 0).cuda()
    x = torch.randn(b.num_nodes, C, device="cuda", requires_grad=True)
    ctx = Ctx(dst_si=b.dst_si, src_si=b.src_si,
              edge_attr=torch.rand(b.edge_index.shape[1], 3, device="cuda") if edge else None)
    params = [x] + list(conv.parameters())
    o1, _ = conv(x, None, ctx)
    g = torch.randn_like(o1)
    g1 = torch.autograd.grad(o1, params, g)
    with composite_mode(True):
        o2, _ = conv(x, None, ctx)
        g2 = torch.autograd.grad(o2, params, g)
    torch.testing.assert_close(o1, o2, rtol=1e-4, atol=1e-4)
    for a, c in zip(g1, g2):
        torch.testing.assert_close(a, c, rtol=1e-3, atol=1e-4)


def test_fused_mfconv_banks_match_composite():
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.models.basic import MFConv
    from hydragnn_amd.models.layers import Ctx
    from hydragnn_amd.ops.pna import composite_mode

    torch.manual_seed(2)
    samples = oc20_like(6, seed=3, radius=5.0, max_neighbours=12, pe_dim=2, min_atoms=20, max_atoms=40)
    b = DeviceGraphStore(samples, "cuda").batch(list(range(6)))
    conv = MFConv(16, 24, max_degree=10).cuda()
    x = torch.randn(b.num_nodes, 16, device="cuda", requires_grad=True)
    ctx = Ctx(dst_si=b.dst_si, src_si=b.src_si)
    params = [x] + list(conv.parameters())
    o1, _ = conv(x, None, ctx)
    g = torch.randn_like(o1)
    g1 = torch.autograd.grad(o1, params, g, allow_unused=True)
    with composite_mode(True):
        o2, _ = conv(x, None, ctx)
        g2 = torch.autograd.grad(o2, params, g, allow_unused=True)
    torch.testing.assert_close(o1, o2, rtol=1e-4, atol=1e-4)
    for a, c in zip(g1, g2):
        if a is None or c is None:
            assert (a is None or not a.abs().sum()) and (c is None or not c.abs().sum())
            continue
        torch.testing.assert_close(a, c, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("edge,act", [(0, "relu"), (2, "silu"), (1, "relu"), (5, "silu")])
def test_fused_egnn_edge_stage_matches_composite(edge, act):
    """EGNN edge_mlp first stage act(A[src] + B[dst] + r w + b (+ e-term)) fused (one pass
    each way, csrc/conv_misc.hip) vs the composite; full E_GCL layer outputs and grads, the
    edge attributes' included.  Edge attributes of <= 3 columns join the radial column in
    the pass (r [E, K], w [K, H]); wider ones are a separate [E, H] term."""
    from torch import nn

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.data.synthetic import oc20_like
    from hydragnn_amd.models.egnn import E_GCL
    from hydragnn_amd.models.layers import Ctx
    from hydragnn_amd.ops.pna import composite_mode

    torch.manual_seed(3)
    samples = oc20_like(6, seed=4, radius=5.0, max_neighbours=10, pe_dim=2, min_atoms=20, max_atoms=40)
    b = DeviceGraphStore(samples, "cuda").batch(list(range(6)))
    H = 40
    layer = E_GCL(H, H, H, edge_attr_dim=edge, act_fn=nn.ReLU() if act == "relu" else nn.SiLU(),
                  equivariant=True).cuda()
    x = torch.randn(b.num_nodes, H, device="cuda", requires_grad=True)
    pos = b.pos.clone().requires_grad_(True)
    ea = torch.rand(b.edge_index.shape[1], edge, device="cuda", requires_grad=True) if edge else None
    ctx = Ctx(dst_si=b.dst_si, src_si=b.src_si, edge_attr=ea)
    params = [x, pos] + ([ea] if edge else []) + list(layer.parameters())
    o1 = layer(x, pos, ctx)
    gx, gp = torch.randn_like(o1[0]), torch.randn_like(o1[1])
    g1 = torch.autograd.grad(o1, params, (gx, gp), allow_unused=True)
    with composite_mode(True):
        o2 = layer(x, pos, ctx)
        g2 = torch.autograd.grad(o2, params, (gx, gp), allow_unused=True)
    for a, c in zip(o1, o2):
        torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-4)
    for a, c in zip(g1, g2):
        if a is None or c is None:
            assert a is None and c is None
            continue
        torch.testing.assert_close(a, c, rtol=1e-3, atol=2e-4)
