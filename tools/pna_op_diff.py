"""Fused PNA kernel vs composite path on the GPU, on the real inputs of the CI-sized model
(captured from its first training batch).  Prints max |diff| per Z block and per gradient."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.data.synthetic import degree_histogram, oc20_like  # noqa: E402
from hydragnn_amd.models.create import create_model  # noqa: E402
from hydragnn_amd.ops import pna as P  # noqa: E402

samples = oc20_like(96, seed=8, min_atoms=4, max_atoms=12, radius=4.0, max_neighbours=6, pe_dim=1)
for s in samples:
    s["x"] = s["x"][:, :1]
deg = degree_histogram(samples, 6)
heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": 4,
                                                         "num_headlayers": 2, "dim_headlayers": [10, 10]}}]}
m = create_model("PNA", 1, 8, [1], 1, None, None, 0, ["graph"], heads, "relu", "mse", [1.0], 2, pna_deg=deg,
                 edge_dim=1, use_gpu=False, init_seed=3).cuda()
st = DeviceGraphStore(samples, "cuda", head_types=["graph"], head_dims=[1])
b = st.batch(list(range(32)))
caught = []
orig = P.pna_message_aggregate


def spy(x, AB, C, G, dst_si, src_si, avg_deg):
    caught.append((x.detach().clone(), AB.detach().clone(), None if C is None else C.detach().clone(),
                   None if G is None else G.detach().clone(), dst_si, src_si, avg_deg))
    return orig(x, AB, C, G, dst_si, src_si, avg_deg)


import hydragnn_amd.models.pnaplus as pp  # noqa: E402

pp.pna_message_aggregate = spy
m(b)
pp.pna_message_aggregate = orig
torch.manual_seed(0)
for li, (x, AB, C, G, dsi, ssi, avg) in enumerate(caught):
    outs = {}
    for name, comp in (("fused", False), ("composite", True)):
        xs = x.clone().requires_grad_()
        ABs = AB.clone().requires_grad_()
        Cs = None if C is None else C.clone().requires_grad_()
        with P.composite_mode(comp):
            Z = P.pna_message_aggregate(xs, ABs, Cs, G, dsi, ssi, avg)
        g = torch.randn(Z.shape, generator=torch.Generator().manual_seed(1)).cuda()
        Z.backward(g)
        outs[name] = (Z.detach(), xs.grad, ABs.grad, None if Cs is None else Cs.grad)
    F = x.shape[1]
    Zf, Zc = outs["fused"][0], outs["composite"][0]
    names = ["x"] + [f"{s}:{a}" for s in ("id", "amp", "att", "lin") for a in ("mean", "min", "max", "std")]
    print(f"layer {li}: F={F}  N={x.shape[0]}  E={dsi.index.numel()}  |Z|max={Zc.abs().max().item():.3e}")
    for k, nm in enumerate(names):
        d = (Zf[:, k * F:(k + 1) * F] - Zc[:, k * F:(k + 1) * F]).abs()
        if d.max() > 0:
            i = int(d.max(1).values.argmax())
            print(f"   Z[{nm:9s}] max|d| {d.max().item():.3e} at node {i} (deg {int(dsi.degree()[i])}): "
                  f"fused {Zf[i, k * F:(k + 1) * F].tolist()} comp {Zc[i, k * F:(k + 1) * F].tolist()}")
    for gi, gn in ((1, "dx"), (2, "dAB"), (3, "dC")):
        a, c = outs["fused"][gi], outs["composite"][gi]
        if a is not None and c is not None:
            d = (a - c).abs()
            print(f"   {gn:4s} max|d| {d.max().item():.3e}  (|ref|max {c.abs().max().item():.3e})  "
                  f"row {int(d.max(1).values.argmax())}")
