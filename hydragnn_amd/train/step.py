"""One training step on the GPU-resident data path, eager or hipGraph-captured.

MI355X design: the GNN workloads of the reference are small-tensor, launch-
bound problems (OC20 PNAPlus+GPS, hidden 64: a step issues several hundred
kernels of a few microseconds each).  PyTorch-eager dispatch costs more CPU
time per kernel than the GPU spends on it, so the production path captures the
whole step —

    batch assembly (gathers out of the HBM dataset pool) -> forward -> masked
    loss -> backward -> [gradient all-reduce] -> AdamW

— as hipGraphs (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replays
them.  Shapes are made static by padding every batch up to a (nodes, edges)
bucket (``DeviceGraphStore.layout``); one graph is captured per bucket (a
handful per dataset) with its own memory pool.  For world_size > 1 the bucketed
gradient all-reduces (RCCL over xGMI) are captured INTO the same graph on a
comm stream that forks off backward as each bucket completes
(``parallel.ddp.BucketedGradSync``): one graph launch per step, collectives
overlapped with the remaining backward kernels.

The per-step host work is only: draw indices, build the int32 plan (numpy),
one pinned H2D copy, one or two graph launches.
"""
import math
import os
import time

import numpy as np
import torch

from ..parallel.ddp import BucketedGradSync, DistributedDataParallel, MultiGradSync


_LOSS_KIND = {"mse": 0, "mae": 1, "rmse": 2, "smooth_l1": 3}


class _FusedMaskedLoss(torch.autograd.Function):
    """One HIP launch forward, one backward (csrc/loss.hip) for the masked losses of a
    padded batch; the composite below stays the CPU / double-backward path."""

    @staticmethod
    def forward(ctx, pred, target, mask, kind):
        from .. import _native

        out = _native.ops().masked_loss_fwd(pred, target, mask, kind)
        ctx.save_for_backward(pred, target, mask, out)
        ctx.kind = kind
        return out[0]

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        pred, target, mask, out = ctx.saved_tensors
        return _native.ops().masked_loss_bwd(g.reshape(1), pred, target, mask, out, ctx.kind), None, None, None


def _fused_loss_ok(kind, pred, target, mask):
    from ..ops.pna import fused

    return (kind in _LOSS_KIND and pred.is_cuda and pred.dtype == torch.float32 and target.dtype == torch.float32
            and fused("loss") and pred.dim() >= 1 and pred.shape == target.shape
            and (mask is None or mask.numel() == pred.shape[0]))


def masked_loss(kind, pred, target, mask=None, var=None):
    """Reference loss functions restricted to rows where ``mask`` is true."""
    if _fused_loss_ok(kind, pred, target, mask):
        return _FusedMaskedLoss.apply(pred.contiguous(), target.contiguous(),
                                      None if mask is None else mask.contiguous(), _LOSS_KIND[kind])
    if mask is None:
        if kind == "mse":
            return torch.nn.functional.mse_loss(pred, target)
        if kind == "mae":
            return torch.nn.functional.l1_loss(pred, target)
        if kind == "rmse":
            return torch.sqrt(torch.nn.functional.mse_loss(pred, target))
        if kind == "smooth_l1":
            return torch.nn.functional.smooth_l1_loss(pred, target)
        if kind == "GaussianNLLLoss":
            return torch.nn.functional.gaussian_nll_loss(pred, target, var)
        raise ValueError(kind)
    keep = mask.view(-1, *([1] * (pred.dim() - 1)))
    m = keep.to(pred.dtype)
    denom = m.sum() * (pred.numel() // pred.shape[0])
    # padded rows never reach the loss, whatever they hold (NaN-safe select, not a product)
    diff = torch.where(keep, pred - target, torch.zeros((), dtype=pred.dtype, device=pred.device))
    if kind in ("mse", "rmse"):
        l = (diff * diff * m).sum() / denom
        return torch.sqrt(l) if kind == "rmse" else l
    if kind == "mae":
        return (diff.abs() * m).sum() / denom
    if kind == "smooth_l1":
        a = diff.abs()
        return (torch.where(a < 1.0, 0.5 * a * a, a - 0.5) * m).sum() / denom
    if kind == "GaussianNLLLoss":
        v = torch.where(keep, var, torch.ones((), dtype=var.dtype, device=var.device)).clamp(min=1e-6)
        return (0.5 * (torch.log(v) + diff * diff / v) * m).sum() / denom
    raise ValueError(kind)


def batch_loss(module, pred, batch):
    """Task-weighted multi-head loss against the per-head targets of a store batch."""
    var = None
    if module.var_output:
        pred, var = pred
    tot = 0
    tasks = []
    for ih in range(module.num_heads):
        mask = batch.get("graph_mask") if module.head_type[ih] == "graph" else batch.get("node_mask")
        v = None if var is None else var[ih]
        l = masked_loss(module.loss_function_type, pred[ih], batch.targets[ih], mask, v)
        w = module.loss_weights[ih]
        lw = l if (not torch.is_tensor(w) and w == 1.0) else l * w
        tot = lw if ih == 0 else tot + lw
        tasks.append(l)
    return tot, tasks


class FlatGrads:
    """All parameter gradients as views of ONE flat buffer (the unit of the
    optimizer's pointer table and of the gradient all-reduce).

    Backward runs with ``p.grad = None`` so autograd *steals* each freshly
    computed gradient (no per-parameter accumulate-add kernel, which was ~130
    launches/step on the OC20 PNAPlus+GPS model), then ``gather`` packs them
    into the flat buffer with batched concatenation copies (a few launches)
    and re-attaches the views."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else "cpu"
        self.flat = torch.zeros(n, device=dev, dtype=self.params[0].dtype if self.params else torch.float32)
        self.attach()

    def attach(self):
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero(self):
        self.flat.zero_()

    def release(self):
        for p in self.params:
            p.grad = None

    def gather(self):
        gs, none = [], []
        for p in self.params:
            g = p.grad
            if g is None:
                none.append(p)
            gs.append(torch.zeros(p.numel(), device=self.flat.device, dtype=self.flat.dtype) if g is None
                      else g.reshape(-1))
        torch.cat(gs, out=self.flat)
        self.attach()
        # parameters the step did not reach keep grad None (torch / reference semantics: the
        # optimizer skips them — no weight or moment decay for absent branch heads)
        for p in none:
            p.grad = None


def _broadcast_state(module):
    import torch.distributed as dist

    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=0)


class _Captured:
    """One captured bucket: two step graphs that differ only in the pinned host buffer their
    first node (an H2D memcpy of the packed plan into ``dev_plan``) reads.  Steps alternate
    between them, so the host writes the next step's plan into the buffer the PREVIOUS
    graph read while the current one runs.  (A separate ``copy_`` call per step blocked the
    host until the queued graph finished on ROCm — 0.41 ms per OC20 step — and left the GPU
    idle while the next replay was being issued.)"""

    def __init__(self):
        self.graphs = [None, None]
        self.pinned = [None, None]
        self.done = [None, None]  # event after the last replay that read pinned[j]
        self.losses = [None, None]
        self.taskss = [None, None]
        self.next = 0
        self.g_opt = None
        self.dev_plan = None
        self.hparams = None  # optimizer hyper-parameters the captured update was built with
        self.dev_seed = None
        self.seeded = False
        self.lay = None
        self.branch = None  # branch-keyed capture: the batch's single branch id

    # the most recently replayed graph's outputs (and graph 0 for callers that want one)
    @property
    def g_fwd_bwd(self):
        return self.graphs[0]

    @property
    def loss(self):
        return self.losses[self.next ^ 1]

    @property
    def tasks(self):
        return self.taskss[self.next ^ 1]


class TrainStep:
    def __init__(self, model, lr=1e-3, mode="graph", world=1, optimizer=None, weight_decay=0.01,
                 node_bucket=256, edge_bucket=2048, max_graphs=16, bucket_cap_mb=None, compute_grad_energy=False):
        # compute_grad_energy: energy + force loss with forces = -dE/dpos (double backward,
        # reference Base.energy_force_loss); the whole step — including the create_graph
        # backward through the segment ops — is captured like any other step
        from ..models.multitask import MultiTaskModelMP

        self.forces = compute_grad_energy
        self.model = model
        # task parallel (SC25 "TP1"): encoder synced over WORLD, this rank's branch decoder
        # over its branch group (two communicators, both in the captured step)
        self.taskpar = model if isinstance(model, MultiTaskModelMP) else None
        self.module = model.module if isinstance(model, (DistributedDataParallel, MultiTaskModelMP)) else model
        self.world = world
        self.mode = mode
        dev = next(self.module.parameters()).device
        self.device = dev
        # multi-branch models: a batch of ONE branch (every batch of an SC25 rank, which loads
        # one dataset) is captured under a branch-keyed bucket and decodes that branch's heads
        # only; a mixed batch replays a dense-decode capture when that pays
        # (_capture_multibranch), else steps eagerly.  HYDRA_BRANCH_KEYED=0: no keying.
        multi = getattr(self.module, "num_branches", 1) > 1
        self.dense_ok = mode == "graph" and multi and self._capture_multibranch()
        self.branch_keyed = (mode == "graph" and multi and self.taskpar is None
                             and os.environ.get("HYDRA_BRANCH_KEYED", "1") == "1")
        if mode == "graph" and multi and not self.dense_ok and not self.branch_keyed:
            self.mode = mode = "eager"
        if world > 1 and mode == "eager" and not isinstance(model, DistributedDataParallel) and self.taskpar is None:
            self.model = DistributedDataParallel(model)
            self.module = self.model.module
        params = [p for p in self.module.parameters() if p.requires_grad]
        if optimizer is None:
            from ..optim.adamw import FusedAdamW

            optimizer = FusedAdamW(params, lr=lr, weight_decay=weight_decay)
        self.opt = optimizer
        self.sync = None
        self.flat_grads = None
        if mode == "graph":
            # captured / padded steps: gradients in one flat buffer; for world > 1 its buckets
            # are all-reduced on a comm stream while backward is still running
            if isinstance(self.model, DistributedDataParallel):
                self.model._sync_enabled = False  # the wrapper's own hooks stand down
                self.model = self.module
            elif self.taskpar is not None:
                self.taskpar.encoder._sync_enabled = False
                self.taskpar.decoder._sync_enabled = False
                self.model = self.module
            elif world > 1:
                _broadcast_state(self.module)
            # one bucket on a single rank unless asked otherwise (the 1-rank RCCL check,
            # tools/gradsync_check.py, uses several to exercise the in-graph bucket order)
            cap = bucket_cap_mb if (world > 1 or bucket_cap_mb is not None) else 1e9
            # task parallel: every rank holds only its own branch (present by construction)
            groups = self._usage_groups(params) if self.taskpar is None else []
            if self.taskpar is not None:
                tp = self.taskpar
                enc_ids = {id(p) for p in tp.encoder.module.parameters()}
                enc = [p for p in params if id(p) in enc_ids]
                dec = [p for p in params if id(p) not in enc_ids]
                self.sync = MultiGradSync([BucketedGradSync(enc, process_group=tp.shared_pg, bucket_cap_mb=cap),
                                           BucketedGradSync(dec, process_group=tp.head_pg, bucket_cap_mb=cap)])
            else:
                self.sync = BucketedGradSync(params, bucket_cap_mb=cap, nflags=len(groups))
            if groups:
                # branch heads absent from a batch keep torch's skip-if-no-grad semantics: the
                # model writes per-branch presence on the device, the sync all-reduces it with
                # the gradients, fused AdamW skips flagged-off parameters
                m = self.module
                m._branch_presence = torch.ones(len(groups), device=dev, dtype=torch.float32)
                self.sync.set_flags(m._branch_presence)
                if hasattr(optimizer, "set_usage_flags"):
                    optimizer.set_usage_flags({p: self.sync.flags[k:k + 1] for k, ps in enumerate(groups)
                                               for p in ps})
                else:
                    import warnings

                    warnings.warn(f"{type(optimizer).__name__} cannot take the captured step's per-branch usage "
                                  "flags: heads of branches absent from a batch still get weight and moment "
                                  "decay (use FusedAdamW, or eager mode, for skip-if-no-grad semantics)",
                                  RuntimeWarning, stacklevel=2)
        elif not isinstance(self.model, DistributedDataParallel) and self.taskpar is None:
            self.flat_grads = FlatGrads(params)
        self.node_bucket, self.edge_bucket = node_bucket, edge_bucket
        self.max_graphs = max_graphs
        # HYDRA_STEP_TIMING=1: accumulate host seconds per graph_step phase
        self.host_times = {} if os.environ.get("HYDRA_STEP_TIMING") == "1" else None
        self.graphs = {}
        self.pool = None
        self.B = None

    def _usage_groups(self, params):
        """Per-branch parameter groups of a multi-branch model (captured dense decode)."""
        m = self.module
        if getattr(m, "num_branches", 1) <= 1 or not hasattr(m, "branch_param_groups"):
            return []
        ids = {id(p) for p in params}
        return [[p for p in g if id(p) in ids] for g in m.branch_param_groups()]

    def _capture_multibranch(self):
        """Multi-branch models capture with a dense decode (every branch head on every row,
        per-row select on the device; ``Base._decode_dense``); conv node heads cannot (their
        BatchNorm would see other branches' nodes).  The dense decode multiplies the head
        work by the branch count, which pays for launch-bound models (MACE multibranch:
        2.4x over eager on MI355X) but not for GEMM-bound ones (the SC25 EGNN-866 with 3 x 889
        node heads: captured 30.6 vs eager 30.1 ms/step), so ``HYDRA_MULTIBRANCH_CAPTURE=auto``
        captures models below 8M parameters; 1 / 0 force it."""
        m = self.module
        if not (hasattr(m, "dense_decode_ok") and m.dense_decode_ok()):
            return False
        flag = os.environ.get("HYDRA_MULTIBRANCH_CAPTURE", "auto")
        if flag in ("0", "1"):
            return flag == "1"
        from ..ops.linear import get_precision

        # bf16: shared-MLP node heads decode branch-grouped (ops.bgemm.branch_mlp: each row
        # through its own branch only), so the captured step wins at any size (EGNN-866:
        # 9.2 ms captured vs 12.1 ms eager on MI355X, profiles/r3_bench_multibranch_egnn.log)
        nh = getattr(m, "config_heads", {}).get("node")
        if get_precision() == "bf16" and (nh is None or nh[0]["architecture"].get("type") == "mlp"):
            return True
        return sum(p.numel() for p in m.parameters()) < 8_000_000

    # ------------------------------------------------------------------ eager
    def _zero(self):
        if self.sync is not None:
            self.sync.release()
        elif isinstance(self.model, DistributedDataParallel) or self.taskpar is not None:
            self.model.zero_grad()
        else:
            self.flat_grads.release()

    def _backward(self, loss, sync=True):
        if self.forces:
            from ..ops.pna import composite_mode

            with composite_mode(True):
                return self._backward_impl(loss, sync)
        return self._backward_impl(loss, sync)

    def _backward_impl(self, loss, sync=True):
        from ..ops.linear import deferred_wgrad

        # tall-linear weight gradients are deferred and computed by one grouped launch pair
        # at the end of backward (ops/linear.py); their grad hooks (bucket all-reduces) fire then
        defer = self.sync is not None or self.flat_grads is not None
        # force steps: only the parameters are backward targets (the positions' second-order
        # gradient terms are never formed)
        inputs = self._train_params() if self.forces else None
        if self.sync is not None:
            self.sync.set_loss(loss)
            if sync:
                self.sync.begin()
            with deferred_wgrad(defer):
                torch.autograd.backward(loss, self._seed(loss), inputs=inputs)
            self.sync.finish()
            return
        with deferred_wgrad(defer):
            torch.autograd.backward(loss, self._seed(loss), inputs=inputs)
        if self.flat_grads is not None:
            self.flat_grads.gather()

    def _train_params(self):
        ps = getattr(self, "_tparams", None)
        if ps is None:
            ps = self._tparams = [p for p in self.module.parameters() if p.requires_grad]
        return ps

    def _seed(self, loss):
        """The backward seed d loss / d loss = 1 as a persistent tensor (an implicit seed is
        a fill launch inside every captured step)."""
        one = getattr(self, "_one", None)
        if one is None or one.device != loss.device or one.dtype != loss.dtype or one.shape != loss.shape:
            if torch.cuda.is_available() and loss.is_cuda and torch.cuda.is_current_stream_capturing():
                return None  # never allocate inside a capture; the warm-up run has created it
            one = self._one = torch.ones_like(loss, memory_format=torch.contiguous_format)
            from ..ops.mlp import mark_unit_seed

            mark_unit_seed(one)
        return one

    def eager(self, store, indices):
        batch = store.batch(indices)
        self._zero()
        loss, tasks = self._loss(batch)
        self._backward(loss)
        self._set_guard(loss)
        self.opt.step()
        return loss.detach(), [t.detach() for t in tasks]

    # ------------------------------------------------------------------ graph
    def bucket_of(self, N, E):
        nb, eb = self.node_bucket, self.edge_bucket
        return (int(math.ceil((N + 2) / nb) * nb), int(math.ceil(max(E, 1) / eb) * eb))

    def prepare(self, store, batch_size, samples=1024, seed=1234, draw=None):
        """Pre-compute the bucket set a random sampler will hit (capture happens lazily).
        ``draw(rng) -> indices``: the sampler (default: uniform without replacement)."""
        self.B = batch_size
        if self.mode != "graph":
            return
        rng = np.random.default_rng(seed)
        seen = set()
        for _ in range(samples):
            idx = draw(rng) if draw is not None else rng.choice(len(store), size=min(batch_size, len(store)),
                                                                 replace=False)
            key = self._key(store, idx)
            if key is not None:
                seen.add(key)
        self.expected = sorted(seen, key=lambda k: tuple(-1 if v is None else v for v in k))

    def precapture(self, store, batch_size, max_draws=2000, seed=4321, draw=None):
        """Capture every bucket ``prepare`` predicted, on real batches drawn at random,
        so no capture (hundreds of ms) lands inside a timed/training region."""
        if self.mode != "graph" or self.device.type != "cuda":
            return
        rng = np.random.default_rng(seed)
        todo = set(getattr(self, "expected", []))
        for _ in range(max_draws):
            if not todo:
                break
            idx = draw(rng) if draw is not None else rng.choice(len(store), size=min(batch_size, len(store)),
                                                                 replace=False)
            key = self._key(store, idx)
            if key in todo and key not in self.graphs:
                self._capture(store, idx, key)
                todo.discard(key)
        self._frozen = bool(self.graphs)

    def _branch_tag(self, store, indices):
        """Branch-keyed capture: the branch id of a single-branch batch, None for a mixed one."""
        if not self.branch_keyed or getattr(store, "dataset_name", None) is None:
            return None
        dn = store.dataset_name[np.asarray(indices, dtype=np.int64)].reshape(-1)
        b = int(dn[0])
        return b if bool((dn == b).all()) else None

    def _key(self, store, indices):
        """Capture key of a batch: its (node, edge) bucket, plus the branch tag for a
        branch-keyed step; None when the batch steps eagerly (mixed, no dense capture)."""
        key = self.bucket_of(*store.sizes_of(indices))
        if not self.branch_keyed:
            return key
        tag = self._branch_tag(store, indices)
        if tag is None and not self.dense_ok:
            return None
        return key + (tag,)

    def _pick(self, N, E, tag=()):
        want = self.bucket_of(N, E) + tag
        if want in self.graphs:
            return want
        cands = [k for k in self.graphs if k[0] >= N + 2 and k[1] >= E and k[2:] == tag]
        # after precapture (or at the cap) a rare unseen bucket replays the captured bucket
        # with the least padded work that fits: extra padding costs microseconds, a capture
        # ~50 ms.  Edge rows cost ~1/avg_degree of a node row (attention, dense maps).
        if cands and (getattr(self, "_frozen", False) or len(self.graphs) >= self.max_graphs):
            return min(cands, key=lambda k: (k[0] - N) + (k[1] - E) / 8.0)
        return want

    def _loss(self, batch):
        if self.forces:
            from ..ops.pna import composite_mode

            batch.pos.requires_grad_(True)
            with composite_mode(True):  # every op on the pos -> E path must be twice differentiable
                pred = self.model(batch)
                return self.module.energy_force_loss(pred, batch)
        if self.model is self.module and hasattr(self.module, "fused_train_loss"):
            out = self.module.fused_train_loss(batch)  # single graph head: head + loss fused
            if out is not None:
                return out
        pred = self.model(batch)
        return batch_loss(self.module, pred, batch)

    def _body_fwd_bwd(self, store, cap, sync=True):
        from ..parallel import gradslots

        self._zero()
        # branch-keyed capture: the batch's single branch is a host constant of the graph
        host_ids = None if getattr(cap, "branch", None) is None else [cap.branch]
        batch = store.assemble(cap.dev_plan, cap.lay, host_ids=host_ids,
                               branch_sorted=store.dataset_name is not None)
        # ops may write gradients straight into the flat buffer's slots (parallel/gradslots.py)
        with gradslots.use(self.sync):
            loss, tasks = self._loss(batch)
            self._backward(loss, sync=sync)
        self._set_guard(loss)
        return loss.detach(), [t.detach() for t in tasks]

    def _set_guard(self, loss):
        """NaN/Inf step guard: optimizers that support it skip the update on the device.

        The guard must be the SAME value on every rank: gradients are all-reduced, so one
        rank's NaN reaches every rank's gradients.  The captured path uses the all-reduced
        guard slot of the gradient buffer (sum of the ranks' losses); the eager DDP path
        all-reduces a copy of the loss."""
        g = loss.detach()
        if self.sync is not None and self.sync.guard_packed:
            g = self.sync.guard
        elif self.world > 1 and isinstance(self.model, DistributedDataParallel):
            import torch.distributed as dist

            g = g.reshape(1).clone()
            dist.all_reduce(g, group=self.model.process_group)
        elif self.world > 1 and self.taskpar is not None:  # eager task parallel: world group
            import torch.distributed as dist

            g = g.reshape(1).clone()
            dist.all_reduce(g, group=self.taskpar.shared_pg)
        if hasattr(self.opt, "guard"):
            self.opt.guard = g
        elif hasattr(getattr(self.opt, "optim", None), "guard"):  # ZeRO wrapper
            self.opt.optim.guard = g

    def _opt_state_tensors(self):
        out = []
        for v in getattr(self.opt, "state", {}).values():
            for t in v.values():
                if torch.is_tensor(t):
                    out.append(t)
        return out

    def _snapshot(self):
        # optimizer state tensors include the per-parameter step counts (FusedAdamW); the
        # device dropout counter is part of the state too: the capture warm-up advances it,
        # and a capture in mid-training must not shift the random stream of the later steps
        # (the captured trajectory then matches the eager padded one step for step)
        from ..ops import rng as _rngmod

        ts = list(self.module.parameters()) + list(self.module.buffers()) + self._opt_state_tensors()
        if self.device.type == "cuda":
            ts.append(_rngmod.counter(self.device))
        return {"pairs": [(t, t.detach().clone()) for t in ts], "ids": {id(t) for t in ts}}

    @torch.no_grad()
    def _restore(self, snap):
        for t, v in snap["pairs"]:
            t.copy_(v)
        for t in self._opt_state_tensors():  # created during warm-up -> fresh (zero) state
            if id(t) not in snap["ids"]:
                t.zero_()

    def _capture(self, store, indices, key):
        """Warm up + capture one bucket.  Parameters, buffers and optimizer state are
        restored afterwards, so the warm-up iterations do not count as training steps."""
        torch.cuda.synchronize()
        if store.dataset_name is not None:
            # the warm-up must see the branch-grouped row order the replayed steps use
            indices = store.branch_order(indices)[0]
        snap = self._snapshot()
        cap = _Captured()
        Np, Ep = key[:2]
        cap.branch = key[2] if len(key) > 2 else None
        cap.lay = store.layout(indices, Np=Np, Ep=Ep, Gp=len(indices) + 1)
        cap.dev_plan = torch.empty(cap.lay.total, dtype=torch.int32, device=self.device)
        # device-side plan: the step uploads only [G, sample ids] and expands the plan in the
        # graph (csrc/assemble.hip store_plan_expand) instead of copying the ~0.6 MB host plan
        cap.seeded = hasattr(store, "device_plan_ok") and store.device_plan_ok(cap.lay)
        n_up = cap.lay.Gp + 1 if cap.seeded else cap.lay.total
        cap.pinned = [torch.empty(n_up, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        if cap.seeded:
            cap.dev_seed = torch.empty(n_up, dtype=torch.int32, device=self.device)
            store.seed(indices, cap.lay, cap.pinned[0].numpy())
            cap.dev_seed.copy_(cap.pinned[0])
            store.plan_device(cap.dev_seed, cap.lay, cap.dev_plan)
        else:
            store.plan(indices, cap.lay, cap.pinned[0].numpy())
            cap.dev_plan.copy_(cap.pinned[0])
        cap.pinned[1].copy_(cap.pinned[0])
        torch.cuda.synchronize()
        # warm-up on the capture stream itself: the parameters' AccumulateGrad nodes are then
        # created on the stream the captured backward runs on (a warm-up on a different stream
        # left them there, and autograd warned of a stream mismatch on every later backward)
        s = self._capture_stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            # warm-up (allocator, kernels, autograd buffers) on real data.  No collective
            # here: ranks capture different buckets at different times (their batches
            # differ), so warm-up must be purely local.  Capture only RECORDS the bucket
            # all-reduces into the graph (RCCL graph capture; user-buffer registration is
            # off, see parallel/distributed.py), nothing is exchanged until replay, where
            # every rank replays exactly one step graph per step.  The warm-up updates are
            # rolled back below.
            for _ in range(2):
                self._body_fwd_bwd(store, cap, sync=False)
                self.opt.step()
        torch.cuda.current_stream().wait_stream(s)
        split = self.world > 1 and not self._graph_collectives()
        from ..ops import rng as _rngmod

        # the dropout counter must exist before capture (created lazily by the first dropout
        # otherwise, and a model without dropout never made it: its H2D init cannot be captured)
        rng_ctr = _rngmod.counter(self.device)
        for j in range(2):
            pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, stream=self._capture_stream()):
                if cap.seeded:  # first node: the device-side plan from the sample ids
                    # the plan kernel reads the ids straight from the pinned host buffer
                    # (HYDRA_SEED_ZEROCOPY=0: an H2D copy node first)
                    zc = os.environ.get("HYDRA_SEED_ZEROCOPY", "1") == "1"
                    if not zc:
                        cap.dev_seed.copy_(cap.pinned[j], non_blocking=True)
                    # the plan launch also advances the dropout counter (the model's per-step
                    # advance is folded into it: one launch less in the step)
                    store.plan_device(cap.pinned[j] if zc else cap.dev_seed, cap.lay, cap.dev_plan, rng=rng_ctr)
                    _rngmod.fold_next_advance(self.device)
                else:  # first node: H2D of the plan
                    cap.dev_plan.copy_(cap.pinned[j], non_blocking=True)
                cap.losses[j], cap.taskss[j] = self._body_fwd_bwd(store, cap, sync=not split)
                if cap.seeded:
                    _rngmod.clear_fold(self.device)
                if not split:
                    self.opt.step()
            cap.graphs[j] = g
            cap.done[j] = torch.cuda.Event()
            if split and j == 0:  # gloo rehearsal on one GPU: [fwd+bwd] -> eager all-reduce -> [optimizer]
                cap.g_opt = torch.cuda.CUDAGraph()
                with torch.cuda.graph(cap.g_opt, pool=pool):
                    self.opt.step()
        cap.hparams = self._opt_hparams()
        self.graphs[key] = cap
        torch.cuda.synchronize()
        self._restore(snap)
        return cap

    def _capture_stream(self):
        """Stream the step graphs are captured on (HYDRA_CAPTURE_PRIORITY: its priority, torch
        convention, lower = higher; default 0 = a normal-priority private stream)."""
        s = getattr(self, "_cap_stream", None)
        if s is None:
            s = self._cap_stream = torch.cuda.Stream(device=self.device,
                                                     priority=int(os.environ.get("HYDRA_CAPTURE_PRIORITY", "0")))
        return s

    def graph_step(self, store, indices):
        N, E = store.sizes_of(indices)
        tag = ()
        if self.branch_keyed:
            b = self._branch_tag(store, indices)
            if b is None and not self.dense_ok:
                return self.eager(store, indices)  # mixed batch, dense decode does not pay
            tag = (b,)
        key = self._pick(N, E, tag)
        cap = self.graphs.get(key)
        if cap is None:
            cap = self._capture(store, indices, key)
            # the capture warm-up already trained on this batch; replay once more as the step
        if not self._sync_opt_hparams(cap):
            # a hyper-parameter baked into the captured update changed: recapture this bucket
            # (the snapshot/restore of _capture keeps the training state unchanged)
            self.graphs.pop(key, None)
            cap = self._capture(store, indices, key)
        tm = self.host_times
        j = cap.next
        cap.next ^= 1
        t0 = time.perf_counter() if tm is not None else 0.0
        ev = cap.done[j]
        ev.synchronize()  # the replay that last read pinned[j] (two steps back) is done
        tw = time.perf_counter() if tm is not None else 0.0
        lay = store.layout(indices, Np=cap.lay.Np, Ep=cap.lay.Ep, Gp=cap.lay.Gp)
        assert lay.total == cap.lay.total
        if cap.seeded:
            store.seed(indices, lay, cap.pinned[j].numpy())
        else:
            store.plan(indices, lay, cap.pinned[j].numpy())
        if tm is not None:
            t1 = time.perf_counter()
        cap.graphs[j].replay()
        ev.record()
        if tm is not None:
            t2 = time.perf_counter()
            tm["plan"] = tm.get("plan", 0.0) + (t1 - tw)
            tm["slot_wait"] = tm.get("slot_wait", 0.0) + (tw - t0)
            tm["replay"] = tm.get("replay", 0.0) + (t2 - t1)
            tm["n"] = tm.get("n", 0) + 1
        if cap.g_opt is not None:
            self.sync.eager_reduce()
            cap.g_opt.replay()
        return cap.losses[j], cap.taskss[j]

    def _opt_hparams(self):
        opt = self.opt
        groups = list(getattr(opt, "param_groups", []))
        inner = getattr(opt, "optim", None)  # ZeRO wrapper: the update runs in the inner optimizer
        return tuple((g.get("lr"), tuple(g.get("betas", ())) if g.get("betas") is not None else None, g.get("eps"),
                      g.get("weight_decay")) for g in groups + (list(inner.param_groups) if inner else []))

    def _sync_opt_hparams(self, cap):
        """Make a replayed step see the optimizer's CURRENT hyper-parameters (a captured step
        never runs the optimizer's host code).  The learning rate of FusedAdamW lives in a
        device scalar and is refreshed here; for any other optimizer, or any other changed
        hyper-parameter, returns False (the bucket is recaptured).  Without this an lr schedule
        such as ReduceLROnPlateau never reached captured training (the CI PNAEq conv-head run
        kept its initial lr 0.02 after the plateau cut it and ended in a bad basin)."""
        opt = self.opt
        inner = getattr(opt, "optim", None)
        if inner is not None and getattr(opt, "param_groups", None):
            for g in inner.param_groups:  # ZeRO wrapper: its step() forwards lr, replays do not
                g["lr"] = opt.param_groups[0]["lr"]
        now = self._opt_hparams()
        if cap.hparams is None or now == cap.hparams:
            return True
        target = inner if inner is not None else opt
        lr_only = [a[1:] for a in now] == [b[1:] for b in cap.hparams]
        if lr_only and hasattr(target, "sync_hparams") and target.sync_hparams():
            cap.hparams = now
            return True
        return False

    def _graph_collectives(self):
        """Collectives can live inside the captured graph only on RCCL ("nccl")."""
        import torch.distributed as dist

        return dist.is_initialized() and dist.get_backend() == "nccl"

    def padded_step(self, store, indices):
        """The captured step's exact computation (static padded bucket shapes) run
        eagerly — the CPU twin of ``graph_step`` used to test the padding logic."""
        N, E = store.sizes_of(indices)
        Np, Ep = self.bucket_of(N, E)
        cap = _Captured()
        if self.branch_keyed:
            cap.branch = self._branch_tag(store, indices)
            if cap.branch is None and not self.dense_ok:
                return self.eager(store, indices)
        lay = store.layout(indices, Np=Np, Ep=Ep, Gp=len(indices) + 1)
        cap.lay = lay
        cap.dev_plan = store.upload(indices, lay)
        loss, tasks = self._body_fwd_bwd(store, cap)  # same bucketed sync as graph_step
        self.opt.step()
        return loss, tasks

    def __call__(self, store, indices):
        if self.mode == "graph":
            if store.dataset_name is not None:
                # graphs grouped by branch (padding last): branch-grouped head GEMMs
                indices = store.branch_order(indices)[0]
            if self.device.type == "cuda":
                return self.graph_step(store, indices)
            return self.padded_step(store, indices)
        return self.eager(store, indices)
