"""Data-parallel gradient synchronisation with bucketed, backward-overlapped all-reduce.

Replaces ``torch.nn.parallel.DistributedDataParallel`` as used by the reference
(``distributed.py:332-351``).  Design for one MI355X node:

* parameters are packed in reverse registration order (≈ the order their
  gradients become ready in backward) into flat fp32 buckets of
  ``bucket_cap_mb``; every ``param.grad`` is a *view* into its bucket, so the
  collective runs on the bucket in place (no pack/unpack copies);
* a post-accumulate-grad hook per parameter counts readiness; a full bucket is
  all-reduced immediately with ``async_op=True`` on the process group (RCCL over
  xGMI for ``nccl``, gloo on CPU), overlapping with the rest of backward;
* a callback queued on the autograd engine flushes buckets whose parameters
  received no gradient (``find_unused_parameters`` semantics) and waits for all
  outstanding collectives before ``backward()`` returns;
* gradients are pre-scaled by 1/world (SUM == AVG, works for gloo too).

GNN parameter counts are small (≈0.1-50 M), so the default bucket size (25 MB)
usually yields 1-3 large collectives per step — the regime where ring
all-reduce over the 7 xGMI links is bandwidth-efficient.
"""
import contextlib
import os

import torch
import torch.distributed as dist
from torch import nn


class _Bucket:
    __slots__ = ("params", "flat", "offsets", "pending", "work", "launched")

    def __init__(self, params, device, dtype):
        self.params = params
        n = sum(p.numel() for p in params)
        self.flat = torch.zeros(n, device=device, dtype=dtype)
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += p.numel()
        self.pending = len(params)
        self.work = None
        self.launched = False


class DistributedDataParallel(nn.Module):
    def __init__(self, module, process_group=None, bucket_cap_mb=25.0, find_unused_parameters=False,
                 broadcast_buffers=True, device_ids=None, output_device=None, gradient_as_bucket_view=True):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world = dist.get_world_size(process_group)
        self.find_unused_parameters = find_unused_parameters
        self.broadcast_buffers = broadcast_buffers
        self._sync_enabled = True
        self._callback_queued = False
        params = [p for p in module.parameters() if p.requires_grad]
        self._broadcast_module_state()
        cap = int(bucket_cap_mb * 1024 * 1024)
        buckets, cur, cur_bytes = [], [], 0
        for p in reversed(params):
            nb = p.numel() * p.element_size()
            if cur and cur_bytes + nb > cap:
                buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            buckets.append(cur)
        self.buckets = []
        self._owner = {}
        for bi, ps in enumerate(buckets):
            b = _Bucket(ps, ps[0].device, ps[0].dtype)
            self.buckets.append(b)
            for p, off in zip(ps, b.offsets):
                p.grad = b.flat[off:off + p.numel()].view_as(p)
                self._owner[p] = bi
                p.register_post_accumulate_grad_hook(self._make_hook(bi, off))

    # ------------------------------------------------------------------ state
    def _src(self):
        """Global rank of the group's first member (torch.distributed takes global src ranks)."""
        if self.process_group is None or self.process_group == dist.group.WORLD:
            return 0
        return dist.get_global_rank(self.process_group, 0)

    def _broadcast_module_state(self):
        if self.world <= 1:
            return
        with torch.no_grad():
            for t in list(self.module.parameters()) + list(self.module.buffers()):
                dist.broadcast(t.data, src=self._src(), group=self.process_group)

    def _sync_buffers(self):
        if self.broadcast_buffers and self.world > 1:
            with torch.no_grad():
                for b in self.module.buffers():
                    dist.broadcast(b.data, src=self._src(), group=self.process_group)

    # ------------------------------------------------------------------ hooks
    def _make_hook(self, bi, off):
        def hook(p):
            if not self._sync_enabled:
                return
            if not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            b = self.buckets[bi]
            # the engine may have replaced the grad tensor (e.g. first accumulation
            # with a non-viewable layout): copy into the bucket view then re-alias
            view = b.flat[off:off + p.numel()].view_as(p)
            if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)
                p.grad = view
            b.pending -= 1
            if b.pending == 0:
                self._launch(b)

        return hook

    def _launch(self, b):
        if b.launched:
            return
        b.launched = True
        if self.world > 1:
            b.flat.div_(self.world)
            b.work = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.process_group, async_op=True)

    def _finalize(self):
        self._callback_queued = False
        for b in self.buckets:
            if not b.launched:
                # parameters that received no gradient contribute zeros
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
            b.launched = False
            b.pending = len(b.params)

    # ------------------------------------------------------------------ API
    def forward(self, *args, **kwargs):
        # Buffers (BN running stats) are broadcast once at construction; per-forward
        # broadcasts would add a collective to every step (see sync_buffers()).
        return self.module(*args, **kwargs)

    def sync_buffers(self):
        self._sync_buffers()

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def zero_grad(self, set_to_none=False):
        for b in self.buckets:
            b.flat.zero_()
        for b in self.buckets:
            for p, off in zip(b.params, b.offsets):
                p.grad = b.flat[off:off + p.numel()].view_as(p)

    def flat_grads(self):
        return [b.flat for b in self.buckets]

    def allreduce_now(self):
        """Synchronous all-reduce of every bucket (used by the graph-captured step)."""
        for b in self.buckets:
            if self.world > 1:
                b.flat.div_(self.world)
                dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.process_group)

    def state_dict(self, *a, **k):
        return super().state_dict(*a, **k)


def default_bucket_cap(nbytes, min_buckets=2):
    """Bucket size in bytes for ``nbytes`` of gradients.  Up to 4 MB (the OC20 PNAPlus+GPS
    headline: 1.7 MB): ONE bucket.  An all-reduce that small is latency-bound over xGMI
    (tens of microseconds whatever its size), and the fused GPS encoder hands back its
    gradients at the end of its backward anyway (tools/overlap_check.py measured its three
    buckets all enqueued after the last backward kernels).  So one collective beats a
    sequence of three.  Medium models: a few buckets, so the first all-reduce starts
    mid-backward.  Large models (> 64 MB): at least 8 buckets of at most 32 MB.  The last
    bucket (the first layers' gradients) is inherently exposed after backward, so it is kept
    small; 4-32 MB rings still run at link bandwidth over xGMI."""
    if nbytes <= 4 * 1024 * 1024:
        return nbytes + 1
    if nbytes > 64 * 1024 * 1024:
        min_buckets = max(min_buckets, 8)
    return min(max(nbytes // min_buckets + 1, 256 * 1024), 32 * 1024 * 1024)


class BucketedGradSync:
    """Gradient all-reduce for the hipGraph-captured training step, overlapped with
    backward (reference DDP ``distributed.py:332-351``).

    All gradients live in ONE flat fp32 buffer laid out in reverse parameter order
    (≈ the order backward produces them) and cut into contiguous buckets.  Backward
    runs with ``p.grad = None`` so autograd hands over each fresh gradient without an
    accumulate kernel; a post-accumulate hook counts the bucket down and, when the
    bucket is complete, a dedicated high-priority comm stream joins the compute stream
    (and the side streams that write gradient slots), packs the bucket (one batched
    copy + the 1/world pre-scale) and launches its all-reduce.  The rest of backward keeps running on the
    compute stream while RCCL moves the bucket over xGMI; ``finish`` joins the comm
    stream back before the optimizer reads the buffer.

    After ``finish`` EVERY parameter holds a gradient (zeros where the step produced none),
    because a captured graph cannot vary the optimizer's parameter set per step.  Parameters
    a step may not reach (heads of branches absent from a batch) get torch's skip-if-no-grad
    semantics back through USAGE FLAGS: ``nflags`` extra slots after the guard slot carry a
    per-group "used this step" value that the model writes on the device (``set_flags``); it
    rides in the last bucket, so after the all-reduce a flag is > 0 iff some rank used the
    group (the reference's DDP ``find_unused_parameters`` + torch AdamW skip), and fused AdamW
    skips flagged-off parameters entirely (``FusedAdamW.set_usage_flags``).

    Captured inside ``torch.cuda.graph`` the event fork/join becomes graph edges, so
    the replayed step is ONE graph launch whose collective nodes run concurrently
    with the remaining backward kernels.  On CPU tensors (gloo) the same code issues
    async collectives and waits for them in ``finish``.
    """

    def __init__(self, params, process_group=None, bucket_cap_mb=None, min_buckets=2, nflags=0):
        self.params = [p for p in params if p.requires_grad]
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        order = list(reversed(self.params))
        total = sum(p.numel() for p in order)
        dev = order[0].device
        # one extra trailing element: the step guard slot.  It rides in the last bucket, so
        # after the all-reduce it holds sum_r loss_r / world — finite iff EVERY rank's loss is
        # finite, the same value on every rank (ranks skip or apply the update together)
        self.nflags = int(nflags)
        self.flat = torch.zeros(total + 1 + self.nflags, device=dev, dtype=order[0].dtype)
        self.total = total
        self.guard = self.flat[total:total + 1]
        self.flags = self.flat[total + 1:total + 1 + self.nflags]  # usage flags (after the reduce)
        self._flag_src = None
        self._loss = None
        nbytes = total * self.flat.element_size()
        if bucket_cap_mb is None:
            cap = default_bucket_cap(nbytes, min_buckets)
        else:
            cap = int(bucket_cap_mb * 1024 * 1024)
        self.offset = {}
        self.buckets = []  # (start, end, [params])
        off, start, cur, cur_b = 0, 0, [], 0
        for p in order:
            nb = p.numel() * self.flat.element_size()
            if cur and cur_b + nb > cap:
                self.buckets.append((start, off, cur))
                start, cur, cur_b = off, [], 0
            self.offset[p] = off
            cur.append(p)
            cur_b += nb
            off += p.numel()
        if cur:
            self.buckets.append((start, off, cur))
        s_, e_, ps_ = self.buckets[-1]
        self.buckets[-1] = (s_, e_ + 1 + self.nflags, ps_)  # + the guard slot (+ usage flags)
        self.bucket_of = {}
        for bi, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self.bucket_of[p] = bi
        self.pending = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.active = False
        self.next = 0
        self.counted = set()
        self.comm = torch.cuda.Stream(device=dev, priority=-1) if dev.type == "cuda" else None
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._hook)
        # gradient slots (parallel/gradslots.py): parameters whose gradient an op wrote straight
        # into its flat slot this step (no pack copy), and the side-stream events behind them
        self.provided = {}
        self.side_events = []
        self.guard_packed = True
        # early flush of deferred grouped weight gradients (ops/linear.py deferred_wgrad): the
        # parameters recorded as deferred this step, and — learned from the previous step —
        # those that must wait for the end-of-backward flush (recorded more than once, or with
        # an ordinary autograd contribution as well: an early flush would reduce their bucket
        # before the last contribution arrived)
        self._deferred = {}
        self._ordinary = set()
        self._in_flush = False
        self._defer_known = False
        self._defer_hold = set()
        self._echoed = set()  # deferred parameters whose None-gradient hook already ran
        self._echo = set()    # flushed early, their op's None-gradient hook still to come
        self._slot_ptr = {p: self.flat.data_ptr() + self.offset[p] * self.flat.element_size() for p in self.params}
        self.attach()

    def slot(self, p):
        """``p``'s view of the flat buffer (None for a parameter this sync does not hold)."""
        o = self.offset.get(p)
        return None if o is None else self.flat[o:o + p.numel()].view_as(p)

    def provide(self, params, event=None):
        """Declare that this step's gradients of ``params`` are (or, after ``event`` on a side
        stream, will be) in their slots: the pack copies skip them, the bucket countdown counts
        them (an op that writes slots returns no autograd gradient for them), and the bucket's
        all-reduce / ``finish`` wait for ``event``."""
        if event is not None:
            self.side_events.append(event)
        for p in params:
            self.provided[id(p)] = p
            if self.active:
                self._count(p)

    def _in_place(self, p):
        if id(p) in self.provided:
            return True
        g = p.grad
        return g is not None and g.is_contiguous() and g.data_ptr() == self._slot_ptr[p]

    # -- grad storage
    def attach(self):
        for p in self.params:
            o = self.offset[p]
            p.grad = self.flat[o:o + p.numel()].view_as(p)

    def release(self):
        for p in self.params:
            p.grad = None

    def zero(self):
        self.flat.zero_()

    # -- sync protocol: begin() before backward, finish() after it
    def set_loss(self, loss):
        """The step's loss: packed into the guard slot with the last bucket."""
        self._loss = loss

    def set_flags(self, src):
        """Device tensor [nflags] of this step's per-group usage (packed with the last bucket)."""
        self._flag_src = src

    def begin(self):
        # HYDRA_GRADSYNC_FORCE=1 exercises the collective path on a 1-rank group (tests)
        self.active = self.world > 1 or (dist.is_initialized() and os.environ.get("HYDRA_GRADSYNC_FORCE") == "1")
        self.pending = [len(ps) for (_, _, ps) in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.next = 0
        self.counted = set()
        for p in list(self.provided.values()):  # slots written during the forward (before begin)
            if self.active:
                self._count(p)

    def note_deferred(self, params):
        """``params`` got a deferred weight-gradient record (not yet computed)."""
        for p in params:
            if p is not None and p in self.offset:
                self._deferred[id(p)] = self._deferred.get(id(p), 0) + 1

    def deferred_flush_ready(self):
        """True when the next bucket in launch order waits only on deferred gradients (none
        of them held back): flushing the recorded problems now lets its all-reduce start
        before the end of backward."""
        if not (self.active and self._defer_known) or self.next >= len(self.buckets):
            return False
        _, _, ps = self.buckets[self.next]
        waiting = False
        for p in ps:
            if id(p) in self.counted:
                continue
            if id(p) in self._defer_hold or id(p) not in self._deferred:
                return False
            waiting = True
        return waiting

    def deferred_held(self, item):
        """A recorded problem that an early flush must leave for the end of backward."""
        return any(p is not None and (id(p) in self._defer_hold or p not in self.offset) for p in item[2:4])

    def expect_echo(self, params):
        """Parameters flushed early: the None-gradient hook of the op that recorded them may
        still arrive (autograd runs it after that op's backward returns) — ignore it once."""
        for p in params:
            if id(p) not in self._echoed:
                self._echo.add(id(p))

    def deferred_flush(self, flushing):
        """Bracket of a deferred flush's post-accumulate hooks (their contributions are the
        deferred ones, not ordinary autograd ones)."""
        self._in_flush = flushing

    def _hook(self, p):
        if not self.active:
            return
        if not self._in_flush and id(p) in self._echo:
            self._echo.discard(id(p))
            self._echoed.add(id(p))
            return
        if p.grad is None:
            self._echoed.add(id(p))
            # autograd runs post-accumulate hooks even for a None contribution: an op that
            # deferred this weight gradient (ops/linear.py deferred_wgrad) or wrote it into its
            # slot (provide) returned None.  A deferred gradient arrives with the flush, a
            # provided one was counted by provide(); counting it now would launch the bucket's
            # all-reduce before the gradient exists.  (A parameter with no gradient at all this
            # step is reduced as zeros by finish().)
            return
        if not self._in_flush:
            self._ordinary.add(id(p))
        self._count(p)

    def _count(self, p):
        bi = self.bucket_of[p]
        if id(p) in self.counted:
            # a second gradient contribution (a parameter used by both a deferred grouped
            # weight gradient and an ordinary op): fine until its bucket has been reduced
            if self.launched[bi]:
                raise RuntimeError("gradient contribution arrived after its bucket was all-reduced")
            return
        self.counted.add(id(p))
        self.pending[bi] -= 1
        # launch in bucket-index order only: every rank then issues the identical
        # collective sequence whatever order its autograd engine finished buckets in
        while self.next < len(self.buckets) and self.pending[self.next] == 0:
            self._launch(self.next)
            self.next += 1

    def _zeros(self, n):
        """A read-only all-zero source of n elements: slices of one persistent buffer (a
        per-step torch.zeros was a fill launch per parameter without a gradient)."""
        z = getattr(self, "_zsrc", None)
        if z is None or z.numel() < n:
            if self.flat.is_cuda and torch.cuda.is_current_stream_capturing():
                return torch.zeros(n, device=self.flat.device, dtype=self.flat.dtype)
            z = self._zsrc = torch.zeros(max(n, max(p.numel() for p in self.params)), device=self.flat.device,
                                         dtype=self.flat.dtype)
        return z[:n]

    def _pack(self, bi):
        """Copy the bucket's gradients into the flat buffer: one batched copy per contiguous run
        of parameters whose gradient is not already in its slot (one run, one launch, in the
        common case)."""
        s, e, ps = self.buckets[bi]
        runs, start, cur, extra = [], None, [], []
        for p in ps:
            if self._in_place(p):
                g = p.grad
                if id(p) in self.provided and g is not None and g.data_ptr() != self._slot_ptr[p]:
                    extra.append(p)  # a second, autograd-returned contribution of a slot-written gradient
                if cur:
                    runs.append((start, cur))
                    cur = []
                continue
            if not cur:
                start = self.offset[p]
            cur.append(p.grad.reshape(-1) if p.grad is not None else self._zeros(p.numel()))
        self.guard_packed = self.active or self.world > 1 or self.nflags > 0
        if e == self.total + 1 + self.nflags and self.guard_packed:
            # the guard slot (+ usage flags) rides with the last bucket's reduce; a lone rank
            # without flags reads the loss itself (TrainStep._set_guard) and packs nothing here
            if not cur:
                start = self.total
            loss = self._loss
            cur.append(loss.detach().reshape(1).to(self.flat.dtype) if loss is not None else
                       torch.zeros(1, device=self.flat.device, dtype=self.flat.dtype))
            if self.nflags:
                f = self._flag_src
                cur.append(f.detach().reshape(-1).to(self.flat.dtype) if f is not None else
                           torch.ones(self.nflags, device=self.flat.device, dtype=self.flat.dtype))
        if cur:
            runs.append((start, cur))
        for start, gs in runs:
            n = sum(g.numel() for g in gs)
            out = self.flat[start:start + n]
            if len(gs) == 1:
                out.copy_(gs[0])
            else:
                torch.cat(gs, out=out)
        for p in extra:
            self.slot(p).add_(p.grad.view_as(p))
        return self.flat[s:e]

    def _launch(self, bi):
        if self.launched[bi]:
            return
        self.launched[bi] = True
        if self.comm is None:
            buf = self._pack(bi)
            buf.mul_(1.0 / self.world)
            self.works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            return
        # pack, pre-scale and reduce all run on the comm stream AFTER it joined the compute
        # stream and every side-stream slot writer: the guard's loss and the head twin's weight
        # gradients come from side streams, so a pack / scale on the compute stream could read
        # or scale a slot before its writer finished.  The packed sources (p.grad, the loss, the
        # usage flags) stay referenced until finish() joins this stream back.
        self.comm.wait_stream(torch.cuda.current_stream())
        for ev in self.side_events:  # slot writers on side streams
            self.comm.wait_event(ev)
        with torch.cuda.stream(self.comm):
            buf = self._pack(bi)
            buf.mul_(1.0 / self.world)
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)

    def eager_reduce(self):
        """Average the packed flat buffer over the group with one blocking all-reduce (the
        split gloo rehearsal of the captured step: collectives outside the graph)."""
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)
            dist.all_reduce(self.flat, group=self.group)

    def finish(self):
        """Flush buckets never completed (parameters without a gradient), join the comm
        stream, re-attach the flat views as ``p.grad``."""
        if self.active:
            for bi in range(len(self.buckets)):
                if not self.launched[bi]:
                    self._launch(bi)
            if self.comm is not None:
                torch.cuda.current_stream().wait_stream(self.comm)
            for w in self.works:
                w.wait()
        else:
            if self.flat.is_cuda:  # the loss / slots written on side streams, before the pack reads them
                for ev in self.side_events:
                    torch.cuda.current_stream().wait_event(ev)
            for bi in range(len(self.buckets)):
                self._pack(bi)
        if self.flat.is_cuda:
            for ev in self.side_events:
                torch.cuda.current_stream().wait_event(ev)
        self.side_events = []
        self.provided = {}
        self.works = []
        if self.active:
            self._defer_hold = {k for k, c in self._deferred.items() if c > 1 or k in self._ordinary}
            self._defer_known = True
        self._deferred = {}
        self._ordinary = set()
        self._echoed = set()
        self._echo = set()
        self.active = False
        self.attach()


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, group, world):
        cnt = torch.tensor([x.shape[0]], dtype=x.dtype, device=x.device)
        stats = torch.cat([x.sum(0), (x * x).sum(0), cnt])
        dist.all_reduce(stats, group=group)
        F = x.shape[1]
        n = stats[-1]
        mean = stats[:F] / n
        var = stats[F:2 * F] / n - mean * mean
        invstd = torch.rsqrt(var + eps)
        xhat = (x - mean) * invstd
        ctx.save_for_backward(xhat, invstd, weight, n)
        ctx.group = group
        y = xhat * weight + bias if weight is not None else xhat
        return y, mean, var * n / (n - 1).clamp(min=1)

    @staticmethod
    def backward(ctx, dy, _dm, _dv):
        xhat, invstd, weight, n = ctx.saved_tensors
        F = xhat.shape[1]
        g = torch.cat([dy.sum(0), (dy * xhat).sum(0)])
        dbias_local, dweight_local = g[:F].clone(), g[F:].clone()
        dist.all_reduce(g, group=ctx.group)
        sdy, sdyx = g[:F], g[F:]
        w = weight if weight is not None else torch.ones_like(sdy)
        dx = (dy - sdy / n - xhat * sdyx / n) * invstd * w
        return dx, (dweight_local if weight is not None else None), (dbias_local if weight is not None else None), \
            None, None, None


class SyncBatchNorm(nn.Module):
    """Cross-rank batch statistics (all-reduce of [sum, sumsq, count]); SURVEY §2.5 C4."""

    def __init__(self, bn, group=None):
        super().__init__()
        self.module = bn
        self.group = group

    def forward(self, x, num_valid=None):
        bn = self.module
        if not bn.training or not dist.is_initialized():
            return torch.nn.functional.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                                                  bn.training, bn.momentum, bn.eps)
        y, mean, uvar = _SyncBNFn.apply(x, bn.weight, bn.bias, bn.eps, self.group, dist.get_world_size())
        with torch.no_grad():
            bn.running_mean.mul_(1 - bn.momentum).add_(bn.momentum * mean.detach())
            bn.running_var.mul_(1 - bn.momentum).add_(bn.momentum * uvar.detach())
            bn.num_batches_tracked.add_(1)
        return y


def convert_sync_batchnorm(model, group=None):
    from ..models.layers import BatchNorm

    for name, m in list(model.named_modules()):
        if isinstance(m, BatchNorm):
            m.module_sync = None
            bn = m.module
            m.forward = SyncBatchNorm(bn, group).forward
    return model


class MultiGradSync:
    """Several :class:`BucketedGradSync` over disjoint parameter subsets, each on its own
    process group and comm stream, driven as one (the captured task-parallel step,
    reference ``MultiTaskModelMP.py:172-276``: the shared encoder all-reduces over WORLD,
    each branch decoder over its branch group).  Inside the step graph the two bucket
    streams become two sets of collective nodes overlapping the rest of backward.

    The first sync is the global one: it carries the step guard (loss) and the usage
    flags, so every rank takes the same skip decision.  All syncs share ONE comm stream:
    two communicators' kernels in flight at once can deadlock when one rank's GPU runs
    them in the other order; on a shared stream every rank issues its branch group's
    buckets, then the world's, in the same autograd order."""

    def __init__(self, syncs):
        self.syncs = list(syncs)
        for s in self.syncs[1:]:
            s.comm = self.syncs[0].comm
        self.guard = self.syncs[0].guard
        self.nflags = self.syncs[0].nflags
        self.flags = self.syncs[0].flags

    @property
    def guard_packed(self):
        return self.syncs[0].guard_packed

    def set_loss(self, loss):
        self.syncs[0].set_loss(loss)

    def set_flags(self, src):
        self.syncs[0].set_flags(src)

    def slot(self, p):
        for s in self.syncs:
            v = s.slot(p)
            if v is not None:
                return v
        return None

    def provide(self, params, event=None):
        for i, s in enumerate(self.syncs):
            mine = [p for p in params if p in s.offset]
            if mine:
                s.provide(mine, event)
            elif i == 0 and event is not None:
                # the side stream also produced the loss the guard holder packs
                s.side_events.append(event)

    def note_deferred(self, params):
        for s in self.syncs:
            s.note_deferred(params)

    def deferred_flush_ready(self):
        return any(s.deferred_flush_ready() for s in self.syncs)

    def deferred_held(self, item):
        """A recorded problem that an early flush must leave for the end of backward."""
        return any(p is not None and (id(p) in self._defer_hold or p not in self.offset) for p in item[2:4])

    def expect_echo(self, params):
        """Parameters flushed early: the None-gradient hook of the op that recorded them may
        still arrive (autograd runs it after that op's backward returns) — ignore it once."""
        for p in params:
            if id(p) not in self._echoed:
                self._echo.add(id(p))

    def deferred_flush(self, flushing):
        for s in self.syncs:
            s.deferred_flush(flushing)

    def deferred_held(self, item):
        # a problem is flushed early only when no sync holds it (each sync sees its own params)
        ps = [p for p in item[2:4] if p is not None]
        for s in self.syncs:
            mine = [p for p in ps if p in s.offset]
            if any(id(p) in s._defer_hold for p in mine):
                return True
        return not all(any(p in s.offset for s in self.syncs) for p in ps)

    def expect_echo(self, params):
        for s in self.syncs:
            s.expect_echo([p for p in params if p in s.offset])

    def begin(self):
        for s in self.syncs:
            s.begin()

    def finish(self):
        for s in self.syncs:
            s.finish()

    def release(self):
        for s in self.syncs:
            s.release()

    def attach(self):
        for s in self.syncs:
            s.attach()

    def zero(self):
        for s in self.syncs:
            s.zero()

    def eager_reduce(self):
        for s in self.syncs:
            s.eager_reduce()
