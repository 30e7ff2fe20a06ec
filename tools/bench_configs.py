"""Training throughput of the other BASELINE.json configurations on one MI355X
(``bench.py`` is the driver's headline: config 4, OC20 PNAPlus + GPS).

  2  qm9_schnet        QM9-shaped molecules, SchNet 4 layers, graph energy head, batch 64
                       (in-forward radius graph, static capacity: captured step)
  3  md17_painn_forces MD17-shaped frames, PAINN (equivariant), node energy head, energy +
                       forces = -dE/dpos (compute_grad_energy, double backward), batch 32
  5a multibranch_egnn  SC25 multibranch shape: EGNN hidden 866 x 4, 5 branches, graph energy +
                       node force heads (3 x 889), batch 128, branch routing by dataset_name
                       (captured step: dense per-row branch select)
  5b multibranch_mace  the BASELINE.json variant of config 5 with MACE (hidden 64, l_max 2,
                       correlation 2, 3 layers), 5 branches, batch 32
  qm9_schnet_gps       the reference QM9 example architecture: SchNet x 2 + GPS (8 heads)
  oc20_gps_h128        config 4 at hidden 128 (16 heads)
  qm9_dimenet          DimeNet++ (reference example hyper-parameters), hidden 64 x 3, batch 64

All synthetic data / random-init weights, fp32.  Prints one JSON line per config.
Usage: python tools/bench_configs.py [names...] [--steps 20] [--warmup 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydragnn_amd.data.device_store import DeviceGraphStore  # noqa: E402
from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.synthetic import degree_histogram, md_trajectory, molecules_like  # noqa: E402
from hydragnn_amd.data.transforms import radius_graph  # noqa: E402
from hydragnn_amd.models.create import create_model  # noqa: E402
from hydragnn_amd.ops.linear import get_precision  # noqa: E402
from hydragnn_amd.ops.pna import composite_mode  # noqa: E402
from hydragnn_amd.train.step import TrainStep  # noqa: E402


def _with_edges(samples, r, k):
    for s in samples:
        s.edge_index = radius_graph(s.pos, r, max_num_neighbors=k)
        s.edge_attr = (s.pos[s.edge_index[1]] - s.pos[s.edge_index[0]]).norm(dim=-1, keepdim=True) / r
        s.sort_edges_by_dst()
    return samples


def _gheads(nb, dims, shared=50):
    return [{"type": f"branch-{b}", "architecture": {"num_sharedlayers": 2, "dim_sharedlayers": shared,
                                                     "num_headlayers": len(dims), "dim_headlayers": dims}}
            for b in range(nb)]


def _nheads(nb, dims):
    return [{"type": f"branch-{b}", "architecture": {"num_headlayers": len(dims), "dim_headlayers": dims,
                                                     "type": "mlp"}} for b in range(nb)]


def qm9_schnet(dev):
    s = _with_edges(molecules_like(1024, seed=1), 7.0, 5)
    heads = {"graph": _gheads(1, [50, 25], 5)}
    m = create_model("SchNet", 1, 64, [1], 0, "", "", 0, ["graph"], heads, "relu", "mse", [1.0], 4,
                     num_gaussians=50, num_filters=64, radius=7.0, max_neighbours=5, dropout=0.0)
    return m, s, 64, ["graph"], [1], False


def qm9_schnet_gps(dev):
    """The reference QM9 example's architecture (examples/qm9/qm9.json): SchNet hidden 64 x 2
    layers + GPS multihead attention (8 heads, pe_dim 2), 10 gaussians, 8 filters, batch 64."""
    from hydragnn_amd.data.transforms import laplacian_pe, relative_pe

    s = _with_edges(molecules_like(1024, seed=1), 7.0, 5)
    for k, g in enumerate(s):
        g.pe = laplacian_pe(g.edge_index, g.num_nodes, 2, seed=k)
        g.rel_pe = relative_pe(g.pe, g.edge_index)
    heads = {"graph": _gheads(1, [50, 25], 5)}
    m = create_model("SchNet", 1, 64, [1], 2, "GPS", "multihead", 8, ["graph"], heads, "relu", "mse", [1.0], 2,
                     num_gaussians=10, num_filters=8, radius=7.0, max_neighbours=5, dropout=0.0)
    return m, s, 64, ["graph"], [1], False


def oc20_gps(dev):
    """BASELINE config 4 exactly as bench.py runs it (hidden 64, 8 heads, 3 layers)."""
    from hydragnn_amd.data.synthetic import oc20_like

    s = oc20_like(512, seed=1000, radius=10.0, max_neighbours=10, pe_dim=16)
    deg = degree_histogram(s, max_degree=10).to(torch.float64)
    heads = {"graph": _gheads(1, [50, 25], 50)}
    m = create_model("PNAPlus", 4, 64, [1], 16, "GPS", "multihead", 8, ["graph"], heads, "relu", "mae", [1.0], 3,
                     pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=10.0, max_neighbours=10)
    return m, s, 32, ["graph"], [1], False


def oc20_gps_h128(dev, nheads=16):
    """BASELINE config 4 (OC20 PNAPlus + GPS, bench.py) at hidden 128 (16 heads of 8)."""
    from hydragnn_amd.data.synthetic import oc20_like

    s = oc20_like(512, seed=1000, radius=10.0, max_neighbours=10, pe_dim=16)
    deg = degree_histogram(s, max_degree=10).to(torch.float64)
    heads = {"graph": _gheads(1, [50, 25], 50)}
    m = create_model("PNAPlus", 4, 128, [1], 16, "GPS", "multihead", nheads, ["graph"], heads, "relu", "mae", [1.0],
                     3, pna_deg=deg, edge_dim=1, envelope_exponent=5, num_radial=6, radius=10.0, max_neighbours=10,
                     dropout=0.0)
    return m, s, 32, ["graph"], [1], False


def oc20_gps_h128_8h(dev):
    """Config 4 at hidden 128 with the BASELINE's 8 heads (head width 16)."""
    return oc20_gps_h128(dev, nheads=8)


def qm9_dimenet(dev):
    """DimeNet++ with the reference's example hyper-parameters (examples/mptrj/*.json:
    int_emb 64, basis_emb 8, out_emb 128, 1 + 2 residual layers, 6 radial x 7 spherical),
    hidden 64 x 3 layers on QM9-shaped molecules, radius 5, batch 64 (captured step: the
    triplets come from the static-capacity device builder)."""
    s = _with_edges(molecules_like(1024, seed=1), 5.0, 20)
    heads = {"graph": _gheads(1, [50, 25], 50)}
    m = create_model("DimeNet", 1, 64, [1], 0, "", "", 0, ["graph"], heads, "relu", "mae", [1.0], 3,
                     radius=5.0, max_neighbours=20, num_radial=6, num_spherical=7, envelope_exponent=5,
                     basis_emb_size=8, int_emb_size=64, out_emb_size=128, num_after_skip=2, num_before_skip=1,
                     dropout=0.0)
    return m, s, 64, ["graph"], [1], False


def md17_painn_forces(dev):
    s = _with_edges(md_trajectory(1024, seed=2, num_atoms=21), 5.0, 20)
    heads = {"node": _nheads(1, [64, 32])}
    m = create_model("PAINN", 1, 64, [1], 0, "", "", 0, ["node"], heads, "relu", "mse", [1.0], 3,
                     num_radial=6, radius=5.0, max_neighbours=20, edge_dim=None, equivariance=True, dropout=0.0)
    return m, s, 32, ["node"], [1], True


def _md17_forces(mpnn, **kw):
    """MD17-shaped energy + force training (config 3's data and head) for another stack: the
    force path of these stacks runs the composite (twice-differentiable torch) ops."""
    s = _with_edges(md_trajectory(1024, seed=2, num_atoms=21), 5.0, 20)
    heads = {"node": _nheads(1, [64, 32])}
    m = create_model(mpnn, 1, 64, [1], 0, "", "", 0, ["node"], heads, "relu", "mse", [1.0], 3,
                     num_radial=6, radius=5.0, max_neighbours=20, equivariance=True, dropout=0.0, **kw)
    return m, s, 32, ["node"], [1], True


def md17_egnn_forces(dev):
    """EGNN energy + forces (the atomistic examples' --compute_grad_energy, e.g. mptrj)."""
    return _md17_forces("EGNN", edge_dim=None)


def md17_pnaeq_forces(dev):
    """PNAEq energy + forces (the physics-informed multibranch GFM example's stack)."""
    s = _with_edges(md_trajectory(1024, seed=2, num_atoms=21), 5.0, 20)
    deg = degree_histogram(s, max_degree=20).to(torch.float64)
    heads = {"node": _nheads(1, [64, 32])}
    m = create_model("PNAEq", 1, 64, [1], 0, "", "", 0, ["node"], heads, "relu", "mse", [1.0], 3,
                     num_radial=6, radius=5.0, max_neighbours=20, equivariance=True, dropout=0.0, edge_dim=None,
                     pna_deg=deg, envelope_exponent=5)
    return m, s, 32, ["node"], [1], True


def _multibranch(mpnn, dev, hidden, layers, hd, batch, in_dim=4, **kw):
    out = []
    for k in range(5):
        for t in molecules_like(384, seed=10 + k, min_atoms=4 + 3 * k, max_atoms=12 + 6 * k, with_forces=True):
            x = torch.cat([t.x, t.pos, t.forces], 1)
            out.append(Graph(x=x, pos=t.pos, y=t.y, forces=t.forces, dataset_name=torch.tensor([[k]])))
    out = _with_edges(out, 5.0, 20)
    for g in out:  # node target = forces (3); graph target = energy per atom
        g.x = g.x[:, :in_dim]
    heads = {"graph": _gheads(5, hd), "node": _nheads(5, hd)}
    m = create_model(mpnn, in_dim, hidden, [1, 3], 0, "", "", 0, ["graph", "node"], heads, "relu", "mae", [1.0, 100.0],
                     layers, radius=5.0, max_neighbours=20, edge_dim=1, dropout=0.0, **kw)
    return m, out, batch, ["graph", "node"], [1, 3], False


def multibranch_egnn(dev):
    return _multibranch("EGNN", dev, 866, 4, [889, 889, 889], 128, equivariance=True)


def multibranch_mace(dev):
    return _multibranch("MACE", dev, 64, 3, [64, 64], 32, max_ell=2, node_max_ell=1, correlation=2, num_radial=8,
                        envelope_exponent=5, radial_type="bessel", avg_num_neighbors=12.0,
                        in_dim=1)  # MACE embeds raw atomic numbers


CONFIGS = {"qm9_schnet": qm9_schnet, "md17_painn_forces": md17_painn_forces, "multibranch_egnn": multibranch_egnn,
           "multibranch_mace": multibranch_mace, "qm9_schnet_gps": qm9_schnet_gps, "oc20_gps_h128": oc20_gps_h128,
           "oc20_gps_h128_8h": oc20_gps_h128_8h, "md17_egnn_forces": md17_egnn_forces,
           "md17_pnaeq_forces": md17_pnaeq_forces,
           "oc20_gps": oc20_gps,
           "qm9_dimenet": qm9_dimenet}


def _targets_for_store(samples, head_types):
    """Attach per-head targets the store packs: graph -> y, node -> forces."""
    for s in samples:
        ys = []
        for t in head_types:
            ys.append(s.y.view(-1, 1) if t == "graph" else s.forces.reshape(-1, 1))
        s.y = torch.cat(ys, 0)
        s.y_loc = torch.tensor([[0] + list(np.cumsum([y.numel() for y in ys]))])
    return samples


def run(name, steps, warmup, dev):
    from hydragnn_amd.ops import bgemm as _bg

    _bg.stats["nt"] = 0  # bf16 GEMM launches of THIS configuration (dtype label)
    model, samples, B, ht, hd, forces = CONFIGS[name](dev)
    model = model.to(dev)
    if not forces:
        samples = _targets_for_store(samples, ht)
    store = DeviceGraphStore(samples, dev, head_types=None if forces else ht, head_dims=None if forces else hd)
    rng = np.random.default_rng(0)
    sampler = None
    single = os.environ.get("BENCH_SINGLE_BRANCH") == "1" and store.dataset_name is not None
    if single:
        # the reference SC25 layout: each rank loads ONE dataset, so every batch holds one
        # branch; on one GPU the steps rotate over the branches (the per-rank mean)
        dn = store.dataset_name.reshape(-1)
        pools = [np.flatnonzero(dn == b) for b in np.unique(dn)]
        turn = [0]

        def sampler(r):
            p = pools[turn[0] % len(pools)]
            turn[0] += 1
            return list(r.choice(p, size=min(B, len(p)), replace=False))
    if forces:
        ts = TrainStep(model, lr=1e-3, mode=os.environ.get("BENCH_FORCES_MODE", "graph"), compute_grad_energy=True,
                       node_bucket=int(os.environ.get("BENCH_NODE_BUCKET", "512")),
                       edge_bucket=int(os.environ.get("BENCH_EDGE_BUCKET", "4096")))
        ts.prepare(store, B, draw=sampler)
        ts.precapture(store, B, draw=sampler)

        def step(idx):
            return ts(store, idx)[0]
    else:
        # captured step (multi-branch models decode densely; SchNet's in-forward radius
        # graph has a data-dependent edge count and steps eagerly)
        mode = os.environ.get("BENCH_MODE", "eager" if not getattr(model, "capturable", True) else "graph")
        nbk = 512 if name.startswith("multibranch") else 256
        ts = TrainStep(model, lr=1e-3, mode=mode, node_bucket=nbk, edge_bucket=8 * nbk)
        ts.prepare(store, B, draw=sampler)
        if ts.mode == "graph":
            ts.precapture(store, B, draw=sampler)

        def step(idx):
            return ts(store, idx)[0]
    draw = (lambda: sampler(rng)) if single else (lambda: list(rng.choice(len(store), size=B, replace=False)))
    for _ in range(warmup):
        step(draw())
    torch.cuda.synchronize()
    if os.environ.get("BENCH_OP_PROFILE") == "1":  # op-level attribution of 3 steps
        from torch.profiler import ProfilerActivity, profile

        shapes = os.environ.get("BENCH_OP_SHAPES") == "1"  # group by input shapes too
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=shapes) as prof:
            for _ in range(3):
                step(draw())
            torch.cuda.synchronize()
        # BENCH_OP_SORT=count: the most frequently launched ops first (launch-bound steps)
        key = "count" if os.environ.get("BENCH_OP_SORT") == "count" else "self_device_time_total"
        print(prof.key_averages(group_by_input_shape=shapes).table(sort_by=key, row_limit=70, max_name_column_width=60,
                                                                   max_shapes_column_width=70), flush=True)
    mark = os.environ.get("HYDRA_PROFILE_MARK") == "1"
    if mark:  # spin kernels bracket the timed steps: rocpd_summary.py --between spin_kernel
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step(draw())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if mark:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    nodes = float(np.mean([s.num_nodes for s in samples]))
    dtype = get_precision()
    if dtype == "bf16":
        # label honestly: "bf16" only if bf16 MFMA GEMMs (csrc/bgemm.hip) were issued for the
        # step (counted at the launcher, so launches recorded into a captured graph count too;
        # maps below the bf16 size threshold stay fp32, e.g. every QM9 SchNet map)
        from hydragnn_amd.ops import bgemm as _bg

        dtype = "bf16" if _bg.stats["nt"] else "fp32 (bf16 requested; every map below the bf16 size threshold)"
    if single:
        name += "/single-branch-batches"
    return {"metric": "training graphs/sec (1 GPU)", "config": name, "value": round(B * steps / el, 2),
            "unit": "graphs/s", "ms_per_step": round(1000 * el / steps, 3), "batch": B, "avg_nodes": round(nodes, 1),
            "params": sum(p.numel() for p in model.parameters()), "dtype": dtype, "final_loss": float(loss),
            "data": "synthetic", "mode": ts.mode}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*", default=list(CONFIGS))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    from hydragnn_amd.ops.linear import set_precision

    set_precision(a.precision)
    dev = torch.device("cuda:0")
    for n in a.names:
        print(json.dumps(run(n, a.steps, a.warmup, dev)), flush=True)


if __name__ == "__main__":
    main()
