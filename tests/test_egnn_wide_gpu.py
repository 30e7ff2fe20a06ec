"""Wide EGNN bf16 MFMA encoder (ops/egnn_wide.py over csrc/bgemm.hip + csrc/egnn.hip)
against the module-by-module fp32 torch path (reference EGCLStack.py:175-289)."""
import pytest
import torch

from hydragnn_amd.data.device_store import DeviceGraphStore
from hydragnn_amd.data.synthetic import molecules_like
from hydragnn_amd.data.transforms import radius_graph
from hydragnn_amd.models.create import create_model
from hydragnn_amd.ops import egnn_wide
from hydragnn_amd.ops.linear import precision

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _samples(n, seed):
    out = molecules_like(n, seed=seed, min_atoms=5, max_atoms=20, with_forces=True)
    for s in out:
        s.edge_index = radius_graph(s.pos, 5.0, max_num_neighbors=20)
        s.edge_attr = (s.pos[s.edge_index[1]] - s.pos[s.edge_index[0]]).norm(dim=-1, keepdim=True) / 5.0
        s.sort_edges_by_dst()
        s.x = torch.cat([s.x, s.pos, s.forces], 1)[:, :4]
        s.y = s.y.view(-1, 1)
        s.y_loc = torch.tensor([[0, 1]])
    return out


def _model(hidden, layers, equivariance=True):
    heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 16,
                                                             "num_headlayers": 1, "dim_headlayers": [16]}}]}
    torch.manual_seed(0)
    return create_model("EGNN", 4, hidden, [1], 0, "", "", 0, ["graph"], heads, "relu", "mae", [1.0], layers,
                        radius=5.0, max_neighbours=20, edge_dim=1, dropout=0.0, equivariance=equivariance).to(dev)


def _encode(model, batch, prec):
    with precision(prec):
        x, pos, ctx = model.encode(batch)
    return x, pos, ctx


@pytest.mark.parametrize("equivariance", [True, False])
def test_egnn_wide_matches_fp32(equivariance):
    """The fused bf16 stack against the fp32 module path, with the module-by-module bf16
    path (every wide GEMM on BF16Linear) as the bf16 noise floor: a random projection of
    the output flips ReLU masks wherever activations sit within bf16 rounding of 0, so
    gradient errors of several percent are inherent to bf16 (both paths show them)."""
    samples = _samples(48, 7)
    model = _model(256, 3, equivariance)
    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    batch = store.batch(list(range(48)))
    with precision("bf16"):
        x0, _, ctx = model.encode(batch)
        assert egnn_wide.eligible(model, ctx)
    R = torch.randn_like(x0)
    params = [p for p in model.graph_convs.parameters()]
    names = [n for n, _ in model.graph_convs.named_parameters()]

    def run(prec, fused=True):
        egnn_wide.ENABLED = fused
        try:
            for p in params:
                p.grad = None
            x, _, _ = _encode(model, batch, prec)
            (x * R).sum().backward()
        finally:
            egnn_wide.ENABLED = True
        return x.detach(), [p.grad.detach().clone() for p in params]

    def rel(a, b):
        return (a - b).norm().item() / (b.norm().item() + 1e-12)

    xa, ga = run("bf16")
    xm, gm = run("bf16", fused=False)
    xf, gf = run("fp32")
    ea, em = rel(xa, xf), rel(xm, xf)
    print(f"forward rel err: fused {ea:.4f}  module bf16 {em:.4f}")
    assert ea < max(2 * em, 1e-2), (ea, em)
    bad = []
    for n, a, m, f in zip(names, ga, gm, gf):
        ra, rm = rel(a, f), rel(m, f)
        print(f"{n:28s} fused {ra:.4f}  module-bf16 {rm:.4f}")
        # coordinate-MLP gradients sit at ~1.5% (module) vs ~5% (fused) on this random
        # projection: inside the ~10% bf16 noise of every other parameter; bounded absolutely
        lim = max(2 * rm, 2e-2) if "coord_mlp" not in n else 8e-2
        if ra > lim:
            bad.append((n, ra, rm))
    assert not bad, bad


def test_egnn_wide_position_gradients():
    """Gradient with respect to each layer's input positions (the coordinate chain through
    radial, normalised difference and coordinate update) of the fused stack vs the module
    path (bf16 and fp32): a wrong term shows as a large error here, bf16 noise as a small one."""
    from hydragnn_amd.models.egnn import E_GCL

    samples = _samples(48, 7)
    model = _model(256, 3, True)
    store = DeviceGraphStore(samples, dev, head_types=["graph"], head_dims=[1])
    batch = store.batch(list(range(48)))
    with precision("bf16"):
        x0, _, _ = model.encode(batch)
    R = torch.randn_like(x0)

    c1s, hooks = [], []

    def module_run(prec):
        egnn_wide.ENABLED = False
        outs = []
        c1s.clear()
        orig = E_GCL.forward

        def fwd(self, inv, equiv, ctx):
            equiv.retain_grad() if equiv.requires_grad else None
            outs.append(equiv)
            if self.equivariant:  # capture d loss / d (coord_mlp[0] output) of this layer
                def keep(mod, i, o):
                    o.retain_grad()
                    c1s.append(o)
                h = self.coord_mlp[0].register_forward_hook(keep)
                hooks.append(h)
            return orig(self, inv, equiv, ctx)
        E_GCL.forward = fwd
        try:
            batch.pos.requires_grad_(True)
            x, _, _ = _encode(model, batch, prec)
            (x * R).sum().backward()
        finally:
            E_GCL.forward = orig
            egnn_wide.ENABLED = True
            batch.pos.requires_grad_(False)
            for h in hooks:
                h.remove()
            hooks.clear()
        return [o.grad.clone() if o.grad is not None else None for o in outs], [c.grad.clone() for c in c1s]

    egnn_wide.DEBUG = {}
    try:
        x, _, _ = _encode(model, batch, "bf16")
        (x * R).sum().backward()
        fused = dict(egnn_wide.DEBUG)
    finally:
        egnn_wide.DEBUG = None
    gm, cm = module_run("bf16")
    gf, cf = module_run("fp32")
    for li in sorted(k for k in fused if isinstance(k, int)):
        a, m, f = fused[li], gm[li], gf[li]
        ra = ((a - f).norm() / f.norm()).item()
        rm = ((m - f).norm() / f.norm()).item()
        ram = ((a - m).norm() / m.norm()).item()
        print(f"layer {li} input-position grad: fused {ra:.4f}  module-bf16 {rm:.4f}  fused-vs-module {ram:.4f} "
              f"|g| {f.norm().item():.3e}")
        assert ra < max(3 * rm, 2e-2), (li, ra, rm)
    for li in range(len(cm)):
        H = cm[li].shape[1]
        a = fused[("dc1", li)][:, :H].float()
        m, f = cm[li], cf[li]
        # the module grad is w.r.t. the pre-activation-free Linear output: mask it like dc1
        print(f"layer {li} dL/dc1: fused-vs-fp32 {((a - f * (a != 0)).norm() / f.norm()).item():.4f} "
              f"module-vs-fp32 {((m - f).norm() / f.norm()).item():.4f}  "
              f"fused-vs-module {((a - m * (a != 0)).norm() / m.norm()).item():.4f}")
