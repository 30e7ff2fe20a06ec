"""Multi-process (gloo, CPU) tests of the data- and task-parallel runtime.

The reference runs its whole suite a second time under ``mpirun -n 2`` with gloo
(``.github/workflows/CI.yml:55-56``); here each test spawns 2 ranks with
``torch.multiprocessing`` and rendezvous on 127.0.0.1.  Covered: bucketed
backward-overlapped all-reduce (``parallel/ddp.py``) == full-batch gradients;
the padded/captured train-step sync structure keeps ranks bit-identical; ZeRO-1
== AdamW; SyncBatchNorm == BatchNorm over the concatenated batch; metric
reductions; task-parallel MultiTaskModelMP over 4 ranks / 2 branches; and an
end-to-end 2-rank ``run_training`` on the CI data.
"""
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn_name, args, errq):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                          LOCAL_RANK=str(rank), HYDRAGNN_BACKEND="gloo", HYDRAGNN_MASTER_PORT=str(port))
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fn = globals().get(fn_name)
        if fn is None:  # bodies defined in other test modules: "module:function"
            import importlib

            mod, _, name = fn_name.partition(":")
            fn = getattr(importlib.import_module(mod), name)
        fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")
        raise


def run_ranks(fn_name, world=2, args=()):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn_name, args, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
            errs.append("timeout")
    assert not errs and all(p.exitcode == 0 for p in procs), "\n".join(errs) or [p.exitcode for p in procs]


# ---------------------------------------------------------------------------- rank bodies

def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(6, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32), torch.nn.Tanh(),
                               torch.nn.Linear(32, 3))


def _ddp_body(rank, world):
    from hydragnn_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(123)
    X, Y = torch.randn(8 * world, 6), torch.randn(8 * world, 3)
    ref = _mlp()
    torch.nn.functional.mse_loss(ref(X), Y).backward()
    model = DistributedDataParallel(_mlp(), bucket_cap_mb=0.002)  # ~500 floats per bucket: several buckets
    assert len(model.buckets) > 1
    for step in range(2):
        model.zero_grad()
        sl = slice(rank * 8, (rank + 1) * 8)
        torch.nn.functional.mse_loss(model(X[sl]), Y[sl]).backward()
    for (n, a), b in zip(model.module.named_parameters(), ref.parameters()):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6, msg=n)


def _bucketed_sync_body(rank, world):
    """BucketedGradSync (captured-step gradient sync, several buckets launched in index
    order from backward hooks) == the average of the ranks' local gradients."""
    import copy

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.train.step import TrainStep, batch_loss

    samples, model = _store_model()
    ref = copy.deepcopy(model)
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1])
    step = TrainStep(model, lr=0.0, mode="graph", world=world, node_bucket=64, edge_bucket=512,
                     bucket_cap_mb=0.004)
    assert len(step.sync.buckets) > 2
    idx = [4 * rank + k for k in range(4)]
    step(store, idx)
    # local gradient of the same padded batch, no sync
    N, E = store.sizes_of(idx)
    Np, Ep = step.bucket_of(N, E)
    batch = store.assemble(store.upload(idx, store.layout(idx, Np=Np, Ep=Ep, Gp=5)),
                           store.layout(idx, Np=Np, Ep=Ep, Gp=5))
    loss, _ = batch_loss(ref, ref(batch), batch)
    loss.backward()
    local = torch.cat([p.grad.reshape(-1) for p in ref.parameters() if p.requires_grad])
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    want = sum(allg) / world
    got = torch.cat([p.grad.reshape(-1) for p in step.module.parameters() if p.requires_grad])
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6)


def _store_model():
    from hydragnn_amd.data.synthetic import degree_histogram, oc20_like
    from hydragnn_amd.models.create import create_model

    samples = oc20_like(24, seed=11, radius=6.0, max_neighbours=8, pe_dim=4, min_atoms=6, max_atoms=14)
    heads = {"graph": [{"type": "branch-0", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 8,
                                                             "num_headlayers": 1, "dim_headlayers": [8]}}]}
    torch.manual_seed(0)
    m = create_model("PNAPlus", 4, 16, [1], 4, "GPS", "multihead", 2, ["graph"], heads, "relu", "mae", [1.0], 2,
                     pna_deg=degree_histogram(samples, 8), edge_dim=1, envelope_exponent=5, num_radial=4,
                     radius=6.0, max_neighbours=8, use_gpu=False, dropout=0.0)
    return samples, m


def _trainstep_body(rank, world):
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.train.step import TrainStep

    samples, model = _store_model()
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1])
    step = TrainStep(model, lr=1e-3, mode="graph", world=world, node_bucket=64, edge_bucket=512)
    step.prepare(store, 4)
    for it in range(3):
        idx = [(4 * (rank + world * it) + k) % len(store) for k in range(4)]
        loss, _ = step(store, idx)
        assert torch.isfinite(loss)
    flat = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()])
    allp = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(allp, flat)
    for t in allp[1:]:
        assert torch.equal(t, allp[0]), "ranks diverged"
    g = torch.cat([p.grad.reshape(-1) for p in step.module.parameters()])
    allg = [torch.empty_like(g) for _ in range(world)]
    dist.all_gather(allg, g)
    assert torch.equal(allg[0], allg[1]), "averaged gradients differ across ranks"


def _nan_guard_body(rank, world):
    """One rank's NaN loss must make EVERY rank skip the update (the all-reduced gradient
    carries the NaN to all ranks): parameters stay bit-identical across ranks and
    unchanged; the next finite step updates all ranks together."""
    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.train.step import TrainStep

    samples, model = _store_model()
    store = DeviceGraphStore(samples, "cpu", head_types=["graph"], head_dims=[1])
    step = TrainStep(model, lr=1e-2, mode="graph", world=world, node_bucket=64, edge_bucket=512)
    step.prepare(store, 4)
    orig = step._loss
    poison = {"on": True}

    def _loss(batch):
        loss, tasks = orig(batch)
        if poison["on"] and rank == 1:
            loss = loss * float("nan")
        return loss, tasks

    step._loss = _loss
    p0 = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()]).clone()
    step(store, [4 * rank + k for k in range(4)])
    p1 = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()])
    assert torch.equal(p0, p1), "a rank applied the update of a step with a non-finite loss"
    poison["on"] = False
    step(store, [4 * rank + k for k in range(4)])
    p2 = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()])
    assert not torch.equal(p1, p2) and torch.isfinite(p2).all()
    allp = [torch.empty_like(p2) for _ in range(world)]
    dist.all_gather(allp, p2)
    assert torch.equal(allp[0], allp[1]), "ranks diverged after a guarded step"


def _zero_body(rank, world):
    from hydragnn_amd.parallel.zero import ZeroRedundancyOptimizer

    torch.manual_seed(5)
    ref, sh = _mlp(), _mlp()
    opt_ref = torch.optim.AdamW(ref.parameters(), lr=1e-2)
    opt = ZeroRedundancyOptimizer(list(sh.parameters()), lambda ps: torch.optim.AdamW(ps, lr=1e-2))
    for it in range(3):
        g = [torch.randn_like(p) for p in ref.parameters()]
        for p, gg in zip(ref.parameters(), g):
            p.grad = gg.clone()
        for p, gg in zip(sh.parameters(), g):
            p.grad = gg.clone()
        opt_ref.step()
        opt.step()
    for a, b in zip(sh.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    st = opt.consolidate_state_dict(to=0)
    if rank == 0:
        assert opt.state_dict() is not None
    # reduce_grads: per-rank gradients are reduce-scattered by the optimizer itself
    torch.manual_seed(6)
    ref, sh = _mlp(), _mlp()
    opt_ref = torch.optim.AdamW(ref.parameters(), lr=1e-2)
    opt = ZeroRedundancyOptimizer(list(sh.parameters()), lambda ps: torch.optim.AdamW(ps, lr=1e-2),
                                  reduce_grads=True)
    for it in range(3):
        g = [[torch.randn_like(p) for p in ref.parameters()] for _ in range(world)]
        for i, p in enumerate(ref.parameters()):
            p.grad = sum(g[r][i] for r in range(world)) / world
        for i, p in enumerate(sh.parameters()):
            p.grad = g[rank][i].clone()
        opt_ref.step()
        opt.step()
    for a, b in zip(sh.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _zero_unused_body(rank, world):
    """A head used only on alternating steps (multibranch batches missing a branch): its
    stale gradient must never be re-applied, and while it has no gradient on any rank it
    gets no update at all (no weight decay / moments), as with per-parameter optimizers.
    Per-parameter ownership matches torch AdamW exactly; the flat layout shares one step
    counter per shard (bias correction), so there the skipped parameter is checked to be
    frozen on its skipped steps and every other parameter to match exactly."""
    from hydragnn_amd.parallel.zero import ZeroRedundancyOptimizer

    for elementwise in (True, False):
        for reduce in (False, True):
            torch.manual_seed(11)
            ref, sh = _mlp(), _mlp()
            sh.load_state_dict(ref.state_dict())
            mk = lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.1)  # noqa: E731
            opt_ref = mk(ref.parameters())
            opt = ZeroRedundancyOptimizer(list(sh.parameters()), mk, reduce_grads=reduce, elementwise=elementwise)
            nparam = len(list(ref.parameters()))
            for it in range(6):
                g = [[torch.randn_like(p) for p in ref.parameters()] for _ in range(world)]
                skip = it % 2 == 1  # the last bias ("a branch head") has no gradient on odd steps
                for i, p in enumerate(ref.parameters()):
                    p.grad = None if (skip and i == nparam - 1) else (
                        sum(g[r][i] for r in range(world)) / world if reduce else g[0][i].clone())
                for i, p in enumerate(sh.parameters()):
                    p.grad = None if (skip and i == nparam - 1) else (g[rank][i].clone() if reduce else g[0][i].clone())
                before = list(sh.parameters())[-1].detach().clone()
                opt_ref.step()
                opt.step()
                if skip:
                    assert torch.equal(list(sh.parameters())[-1], before), "unused parameter was updated"
                opt_ref.zero_grad(set_to_none=True)
                opt.zero_grad(set_to_none=True)
            pairs = list(zip(sh.parameters(), ref.parameters()))
            if elementwise:
                pairs = pairs[:-1]
            for a, b in pairs:
                torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
            st = opt.state_dict()
            bad = dict(st, layout="param" if elementwise else "flat")
            with pytest.raises(ValueError):
                opt.load_state_dict(bad)


def _zero_one_rank_unused_body(rank, world):
    """Only rank 1 lacks a gradient for the last parameter (its batch has no sample of that
    branch): every rank must still join the usage-flag all-reduce (a rank-local early return
    would desynchronise the collectives), and the parameter is USED globally, so it is
    updated with the average of the gradients that exist (zeros from rank 1)."""
    from hydragnn_amd.parallel.zero import ZeroRedundancyOptimizer

    for elementwise in (True, False):
        torch.manual_seed(5)
        ref, sh = _mlp(), _mlp()
        sh.load_state_dict(ref.state_dict())
        mk = lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.1)  # noqa: E731
        opt_ref = mk(ref.parameters())
        opt = ZeroRedundancyOptimizer(list(sh.parameters()), mk, reduce_grads=True, elementwise=elementwise)
        nparam = len(list(ref.parameters()))
        for it in range(3):
            g = [[torch.randn_like(p) for p in ref.parameters()] for _ in range(world)]
            for i, p in enumerate(ref.parameters()):
                p.grad = sum(g[r][i] for r in range(world) if not (r == 1 and i == nparam - 1)) / world
            for i, p in enumerate(sh.parameters()):
                p.grad = None if (rank == 1 and i == nparam - 1) else g[rank][i].clone()
            opt_ref.step()
            opt.step()
            opt_ref.zero_grad(set_to_none=True)
            opt.zero_grad(set_to_none=True)
        for a, b in zip(sh.parameters(), ref.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _syncbn_body(rank, world):
    from hydragnn_amd.parallel.ddp import SyncBatchNorm

    torch.manual_seed(9)
    x = torch.randn(10 * world, 5) * 2 + 1
    bn_ref = torch.nn.BatchNorm1d(5)
    xr = x.clone().requires_grad_()
    g = torch.randn_like(x)
    bn_ref(xr).backward(g)
    bn = torch.nn.BatchNorm1d(5)
    sbn = SyncBatchNorm(bn)
    sl = slice(rank * 10, (rank + 1) * 10)
    xl = x[sl].clone().requires_grad_()
    y = sbn(xl)
    y.backward(g[sl])
    torch.testing.assert_close(xl.grad, xr.grad[sl], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_mean, bn_ref.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var, bn_ref.running_var, rtol=1e-5, atol=1e-6)
    # parameter grads are local partial sums; their all-reduce == the full-batch grads
    dw = bn.weight.grad.clone()
    dist.all_reduce(dw)
    torch.testing.assert_close(dw, bn_ref.weight.grad, rtol=1e-4, atol=1e-5)


def _reduce_body(rank, world):
    from hydragnn_amd.train.train_validate_test import gather_tensor_ranks, reduce_values_ranks

    v = reduce_values_ranks(torch.tensor([float(rank + 1)]))
    assert abs(float(v) - (1 + world) / 2) < 1e-6
    rows = torch.full((rank + 2, 3), float(rank))
    allrows = gather_tensor_ranks(rows)
    assert allrows.shape[0] == sum(r + 2 for r in range(world))


def _timers_body(rank, world):
    """Ranks time different regions (rank 1 has an extra timer, rank 0 one of its own):
    the reduction unions the names and never mismatches or hangs (ref Appendix D #13)."""
    from hydragnn_amd.utils.time_utils import Timer, gather_timers

    Timer.reset()
    names = ["common"] + (["only_rank1_a", "only_rank1_b"] if rank == 1 else ["zz_rank0"])
    for n in names:
        t = Timer(n)
        t.start()
        t.stop()
    Timer.timers_local["common"] = float(rank + 1)
    st = gather_timers()
    assert set(st) == {"common", "only_rank1_a", "only_rank1_b", "zz_rank0"}
    mn, mx, avg, calls = st["common"]
    assert (mn, mx, avg, calls) == (1.0, 2.0, 1.5, 2)
    assert st["only_rank1_a"][3] == 1 and st["zz_rank0"][3] == 1


def _filecount_body(rank, world):
    from hydragnn_amd.data.lsms import check_same_count_across_ranks

    assert check_same_count_across_ranks(7, "same") == 7
    try:
        check_same_count_across_ranks(7 + rank, "differs")
    except RuntimeError as e:
        assert "ranks disagree" in str(e)
    else:
        raise AssertionError("mismatched file counts not detected")


def _train_body(rank, world, workdir):
    from graph_train_util import unittest_train_model

    os.environ["HYDRAGNN_DEVICE_DATA"] = "0"
    unittest_train_model("PNA", "", "", "ci", False, workdir,
                         overwrite_config={"NeuralNetwork": {"Training": {"num_epoch": 30}}})


def _task_parallel_body(rank, world):
    from hydragnn_amd.data.graph import collate
    from hydragnn_amd.data.synthetic import degree_histogram, oc20_like
    from hydragnn_amd.models.create import create_model
    from hydragnn_amd.models.multitask import MultiTaskModelMP, branch_groups

    bid, group, lists = branch_groups([3, 1])
    assert lists == [[0, 1, 2], [3]]
    samples = oc20_like(8, seed=20 + rank, radius=5.0, max_neighbours=8, pe_dim=2, min_atoms=5, max_atoms=10)
    for g in samples:
        g.dataset_name = torch.tensor([[bid]])
    heads = {"graph": [{"type": f"branch-{b}", "architecture": {"num_sharedlayers": 1, "dim_sharedlayers": 8,
                                                                  "num_headlayers": 1, "dim_headlayers": [8]}}
                       for b in range(2)]}
    torch.manual_seed(0)
    base = create_model("EGNN", 4, 12, [1], 2, "", "multihead", 1, ["graph"], heads, "relu", "mse", [1.0], 2,
                        use_gpu=False, edge_dim=None, dropout=0.0)
    model = MultiTaskModelMP(base, bid, group)
    names = [n for n, _ in model.named_parameters()]
    assert not any(f"branch-{1 - bid}" in n for n in names), "other branch not pruned"
    b = collate(samples)
    pred = model(b)
    pred[0].pow(2).mean().backward()
    enc = torch.cat([p.grad.reshape(-1) for n, p in model.named_parameters()
                     if not n.startswith(("graph_shared", "heads_NN"))])
    dec = torch.cat([p.grad.reshape(-1) for n, p in model.named_parameters()
                     if n.startswith(("graph_shared", "heads_NN"))])
    allenc = [torch.empty_like(enc) for _ in range(world)]
    dist.all_gather(allenc, enc)
    for t in allenc[1:]:
        torch.testing.assert_close(t, allenc[0])
    alldec = [torch.empty_like(dec) for _ in range(world)]
    dist.all_gather(alldec, dec)  # branch 0's ranks agree with each other
    for r in lists[bid]:
        torch.testing.assert_close(alldec[r], dec)



def _task_parallel_captured_body(rank, world):
    """TrainStep drives MultiTaskModelMP in graph mode (statically padded step, the CPU twin
    of the captured one): encoder gradients all-reduced over WORLD, the branch decoder's over
    its branch group, both through the step's bucketed sync — equal to the eager wrapper
    (two DDP communicators) after several AdamW steps."""
    import copy
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_multibranch_capture import _data, _model

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.models.multitask import MultiTaskModelMP, branch_groups
    from hydragnn_amd.parallel.ddp import MultiGradSync
    from hydragnn_amd.train.step import TrainStep

    bid, group, lists = branch_groups([2, 2])
    samples = _data(16)
    for g in samples:
        g.dataset_name = torch.tensor([[bid]])
    base = _model("EGNN")
    m_e = MultiTaskModelMP(copy.deepcopy(base), bid, group)
    m_g = MultiTaskModelMP(base, bid, group)
    store = DeviceGraphStore(samples, "cpu", head_types=["graph", "node"], head_dims=[1, 1])
    eager = TrainStep(m_e, lr=1e-2, mode="eager", world=world)
    cap = TrainStep(m_g, lr=1e-2, mode="graph", world=world, node_bucket=64, edge_bucket=256,
                    bucket_cap_mb=0.004)
    assert cap.mode == "graph" and isinstance(cap.sync, MultiGradSync)
    assert len(cap.sync.syncs[0].buckets) > 1
    rng = np.random.default_rng(rank)
    for _ in range(3):
        idx = list(rng.choice(len(samples), 5, replace=False))
        le, lc = float(eager(store, idx)[0]), float(cap(store, idx)[0])
        assert abs(le - lc) <= 1e-4 * max(1.0, abs(le)), (le, lc)
    for (n, pe), (_, pg) in zip(m_e.named_parameters(), m_g.named_parameters()):
        torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-5, msg=n)
    enc = torch.cat([p.detach().reshape(-1) for n, p in m_g.named_parameters()
                     if not n.startswith(("graph_shared", "heads_NN"))])
    allenc = [torch.empty_like(enc) for _ in range(world)]
    dist.all_gather(allenc, enc)  # the encoder stays identical on every rank
    for t in allenc[1:]:
        torch.testing.assert_close(t, allenc[0])


def _bnsync_body(rank, world):
    """Rank-local BN running statistics are made identical (rank 0's) once per epoch."""
    from hydragnn_amd.models.layers import BatchNorm
    from hydragnn_amd.train.train_validate_test import _sync_running_stats

    m = torch.nn.Sequential(BatchNorm(4))
    m.train()
    m(torch.randn(16, 4) * (rank + 1) + rank)
    _sync_running_stats(m)
    rm = [b.clone() for b in m.buffers() if b.is_floating_point()]
    for t in rm:
        allv = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        for v in allv[1:]:
            torch.testing.assert_close(v, allv[0])



def _aggr_backend_body(rank, world):
    """HYDRAGNN_AGGR_BACKEND: torch / mpi reduce across ranks, anything else stays local."""
    import os

    from hydragnn_amd.train.train_validate_test import reduce_values_ranks
    from hydragnn_amd.utils.config_utils import _allreduce

    v = torch.tensor([float(rank + 1)])
    for backend, want in (("torch", 1.5), ("mpi", 1.5), ("local", float(rank + 1))):
        os.environ["HYDRAGNN_AGGR_BACKEND"] = backend
        assert float(reduce_values_ranks(v)) == want, backend
        s = _allreduce(torch.tensor([rank + 1]), dist.ReduceOp.SUM)
        assert int(s) == (3 if backend != "local" else rank + 1), backend
    os.environ.pop("HYDRAGNN_AGGR_BACKEND")


def _multibranch_capture_body(rank, world):
    """Captured-step (statically padded, dense / grouped multi-branch decode, bucketed
    gradient sync) on 4 ranks == the rank average of the eager per-branch-range gradients."""
    import copy
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_multibranch_capture import _data, _model

    from hydragnn_amd.data.device_store import DeviceGraphStore
    from hydragnn_amd.train.step import TrainStep, batch_loss

    samples = _data(24)
    model = _model("EGNN")
    ref = copy.deepcopy(model)
    store = DeviceGraphStore(samples, "cpu", head_types=["graph", "node"], head_dims=[1, 1])
    step = TrainStep(model, lr=0.0, mode="graph", world=world, node_bucket=64, edge_bucket=256,
                     bucket_cap_mb=0.004)
    assert step.mode == "graph" and len(step.sync.buckets) > 1
    idx = [6 * rank + k for k in range(6)]
    step(store, idx)
    batch = store.batch(idx)  # eager: branch-sorted ranges decode
    loss, _ = batch_loss(ref, ref(batch), batch)
    loss.backward()
    local = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros(p.numel())
                       for p in ref.parameters() if p.requires_grad])
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    want = sum(allg) / world
    got = torch.cat([p.grad.reshape(-1) for p in step.module.parameters() if p.requires_grad])
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------------------- tests

def test_ddp_bucketed_allreduce_matches_full_batch():
    run_ranks("_ddp_body")


def test_trainstep_ranks_stay_in_sync():
    run_ranks("_trainstep_body")


def test_bucketed_grad_sync_matches_rank_average():
    run_ranks("_bucketed_sync_body")


def test_zero1_matches_adamw():
    run_ranks("_zero_body")


def test_nan_guard_is_global():
    run_ranks("_nan_guard_body")


def test_zero1_unused_parameters():
    run_ranks("_zero_unused_body")


def test_zero1_unused_on_one_rank_only():
    run_ranks("_zero_one_rank_unused_body")


def test_syncbatchnorm_matches_full_batch():
    run_ranks("_syncbn_body")


def test_metric_reductions():
    run_ranks("_reduce_body")


def test_timer_reduction_with_rank_specific_timers():
    run_ranks("_timers_body")


def test_raw_file_count_check():
    run_ranks("_filecount_body")


def test_captured_multibranch_four_ranks_matches_eager():
    run_ranks("_multibranch_capture_body", world=4)


def test_task_parallel_multibranch_four_ranks():
    run_ranks("_task_parallel_body", world=4)


def test_task_parallel_captured_step_four_ranks():
    run_ranks("_task_parallel_captured_body", world=4)


@pytest.mark.slow
def test_run_training_two_ranks(tmp_path):
    run_ranks("_train_body", args=(str(tmp_path),))


def test_bn_running_stats_synced_per_epoch():
    run_ranks("_bnsync_body")


def test_aggr_backend_flag():
    run_ranks("_aggr_backend_body")


# ------------------------------------------------- early flush of deferred weight gradients

class _DeferLin(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is DEFERRED (recorded for the grouped flush, as
    the GPU tall linears do), so the CPU gloo ranks exercise the flush / bucket protocol."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x)
        ctx.params = (W, b)
        return x @ W.t() + b

    @staticmethod
    def backward(ctx, dy):
        from hydragnn_amd.ops import linear as _lin

        (x,) = ctx.saved_tensors
        W, b = ctx.params
        assert _lin._can_defer(W, b)
        _lin._record((dy, x, W, b))
        return dy @ W, None, None


def _early_flush_body(rank, world):
    from hydragnn_amd.ops import linear as _lin
    from hydragnn_amd.parallel import gradslots
    from hydragnn_amd.parallel.ddp import BucketedGradSync

    def run(early):
        os.environ["HYDRA_EARLY_WGRAD_FLUSH"] = "1" if early else "0"
        torch.manual_seed(0)
        lins = [torch.nn.Linear(48, 48) for _ in range(6)]
        params = [p for l in lins for p in (l.weight, l.bias)]
        sync = BucketedGradSync(params, bucket_cap_mb=0.02)  # ~2 layers per bucket
        assert len(sync.buckets) >= 3
        launches = []
        orig = sync._launch

        def launch(bi):
            launches.append((bi, len(_lin._defer["items"])))
            return orig(bi)
        sync._launch = launch
        outs = []
        for step in range(2):
            g = torch.Generator().manual_seed(100 * rank + step)
            x = torch.randn(64, 48, generator=g)
            sync.release()
            sync.set_loss(None)
            launches.clear()
            _lin._defer["early"] = 0
            with gradslots.use(sync):
                sync.begin()
                with _lin.deferred_wgrad(True):
                    h = x
                    for l in lins:
                        h = torch.relu(_DeferLin.apply(h, l.weight, l.bias))
                    h.pow(2).mean().backward()
                sync.finish()
            outs.append(sync.flat[:sync.total].clone())
        return outs, list(launches), _lin._defer["early"]

    base, _, n0 = run(False)
    got, launches, n1 = run(True)
    assert n0 == 0
    # step 2 (the first with the learned hold set) flushed early: buckets were reduced while
    # deferred problems of earlier layers were still unrecorded
    assert n1 >= 2, n1
    assert any(k > 0 or bi < len(launches) - 1 for bi, k in launches[:-1])
    for a, b in zip(base, got):
        assert torch.equal(a, b)  # bit-identical to the end-of-backward flush
    # and equal to the rank average of plain autograd gradients
    torch.manual_seed(0)
    lins = [torch.nn.Linear(48, 48) for _ in range(6)]
    g = torch.Generator().manual_seed(100 * rank + 1)
    x = torch.randn(64, 48, generator=g)
    h = x
    for l in lins:
        h = torch.relu(l(h))
    h.pow(2).mean().backward()
    local = torch.cat([p.grad.reshape(-1) for p in reversed([p for l in lins for p in (l.weight, l.bias)])])
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    torch.testing.assert_close(got[1], sum(allg) / world, rtol=1e-5, atol=1e-6)


def test_early_deferred_wgrad_flush_two_ranks():
    run_ranks("_early_flush_body")
