"""Linear layers: library / fused-engine fp32 paths and the bf16 MFMA engine.

``linear_act`` computes ``act(sum_p X_p W_p^T + b) (+ residual)``.

Precision (``set_precision`` / ``Training.precision``):
* ``"fp32"`` (default; the reference's numerics): library GEMM forward + data gradient,
  split-K weight-gradient kernel (csrc/linear.hip, deferred + grouped inside the training
  engine's backward), and the one-launch concat-linear forward of csrc/gemm.hip
  (v_mfma_f32_16x16x4_f32, exact fp32) for node-sized multi-input sums;
* ``"bf16"``: single-input maps above ``BF16_MIN_MACS`` run on the bf16 MFMA engine
  (csrc/bgemm.hip via ``ops.bgemm.BF16Linear``): operands rounded to bf16, fp32
  accumulation, fp32 storage and master weights.  Narrow or small maps stay fp32.

CPU tensors, non-fp32 dtypes and composite mode (double backward for force
training) use ``F.linear``.
"""
import os

import torch
import torch.nn.functional as F

from .. import _native
from ..parallel import gradslots as _gradslots
from . import pna as _mode

_PREC = {"fp32": 0, "bf16": 1}
_state = {"prec": _PREC.get(os.environ.get("HYDRA_PRECISION", "fp32"), 0)}

ACT_NONE, ACT_RELU = 0, 1


def set_precision(name):
    """Global GEMM compute precision: "fp32" or "bf16"."""
    _state["prec"] = _PREC[name]


def get_precision():
    return "bf16" if _state["prec"] == 1 else "fp32"


class precision:
    """Context manager: ``with precision("bf16"): ...``."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = _state["prec"]
        _state["prec"] = _PREC[self.name]

    def __exit__(self, *a):
        _state["prec"] = self.prev


def _row_contig(t):
    return t if (t.stride(-1) == 1 or t.shape[-1] == 1) else t.contiguous()


# ---- deferred weight gradients -------------------------------------------------------
# Inside ``deferred_wgrad()`` (the training engine wraps its backward in it) the tall
# linears do not launch their own split-K weight-gradient pair: they record
# (dY, X, W, b) and return no dW/db; on exit ONE grouped launch pair computes every
# recorded weight gradient and writes / accumulates it into ``W.grad`` / ``b.grad``
# (csrc/linear.hip, ``linear_wgrad_grouped``), then runs the parameters'
# post-accumulate-grad hooks (the bucketed all-reduce of the captured step).
_defer = {"on": False, "items": [], "early": 0}  # early: flushes triggered by a waiting bucket


def _can_defer(W, b):
    return _defer["on"] and not torch.is_grad_enabled() and isinstance(W, torch.nn.Parameter) and \
        (b is None or isinstance(b, torch.nn.Parameter))


class deferred_wgrad:
    def __init__(self, enabled=True):
        self.enabled = enabled and os.environ.get("HYDRA_DEFER_WGRAD", "1") == "1"

    def __enter__(self):
        self.prev = _defer["on"]
        _defer["on"] = self.enabled
        return self

    def __exit__(self, *exc):
        _defer["on"] = self.prev
        if exc[0] is None:
            flush_deferred_wgrads()
        else:
            _defer["items"].clear()
        return False


def _record(item):
    """Record one deferred weight-gradient problem.  Under a step's gradient sync whose next
    bucket now waits only on deferred problems, flush everything recorded so far at once
    (``BucketedGradSync.deferred_flush_ready``): that bucket's all-reduce then overlaps the
    rest of backward instead of starting after the end-of-backward flush."""
    _defer["items"].append(item)
    s = _gradslots.active()
    if s is None or not hasattr(s, "note_deferred"):
        return
    s.note_deferred(item[2:4])
    if os.environ.get("HYDRA_EARLY_WGRAD_FLUSH", "1") == "1" and s.deferred_flush_ready():
        _defer["early"] += 1
        held = s.deferred_held
        flushed = [p for it in _defer["items"] if not held(it) for p in it[2:4] if p is not None]
        flush_deferred_wgrads(keep=held)
        s.expect_echo(flushed)


def _span(it):
    k0 = it[4] if len(it) > 4 else 0  # column block [k0, k0 + K) of W (row programs)
    return k0, k0 + it[1].shape[1]


def _conflict(a, b):
    """Two deferred problems write the same output elements (same weight columns / bias)."""
    if a[2] is b[2]:
        (a0, a1), (b0, b1) = _span(a), _span(b)
        if a0 < b1 and b0 < a1:
            return True
    return a[3] is not None and a[3] is b[3]


def flush_deferred_wgrads(keep=None):
    """Compute every recorded weight gradient (grouped launches) and run the parameters'
    post-accumulate hooks.  ``keep(item)`` True: leave that problem recorded for a later flush
    (an early flush skips parameters whose bucket must wait for the end of backward)."""
    items = _defer["items"]
    if keep is not None:
        _defer["items"] = [it for it in items if keep(it)]
        items = [it for it in items if not keep(it)]
    else:
        _defer["items"] = []
    if not items:
        return
    # one launch covers problems with disjoint outputs (column blocks of one weight included);
    # a weight / bias recorded twice (shared weights) goes to a later launch so its
    # accumulation is ordered
    rounds = []
    for it in items:
        for r in rounds:
            if not any(_conflict(it, o) for o in r):
                r.append(it)
                break
        else:
            rounds.append([it])
    touched = []
    for r in rounds:
        # a weight without a gradient yet whose column blocks in this launch cover all its
        # columns is written directly (no zero fill, no accumulation)
        cover = {}
        for it in r:
            cover.setdefault(id(it[2]), [it[2], []])[1].append(_span(it))
        fresh = set()
        for key, (W, spans) in cover.items():
            if W.grad is None:
                spans = sorted(spans)
                pos = 0
                for a0, a1 in spans:
                    if a0 != pos:
                        break
                    pos = a1
                if pos == W.shape[1]:
                    fresh.add(key)
        dys, xs, dws, dbs, acc = [], [], [], [], []
        for it in r:
            dy, x, W, b = it[:4]
            k0, k1 = _span(it)
            full = k0 == 0 and k1 == W.shape[1]
            a = not (id(W) in fresh and (b is None or b.grad is None))
            if W.grad is None:
                # the step's flat-buffer slot when it provides one (parallel/gradslots.py)
                sl = _gradslots.slots([W])
                if sl is not None:
                    W.grad = sl[0] if id(W) in fresh else sl[0].zero_()
                else:
                    W.grad = torch.empty_like(W) if id(W) in fresh else torch.zeros_like(W)
            if b is not None and b.grad is None:
                sl = _gradslots.slots([b])
                if sl is not None:
                    b.grad = sl[0] if not a else sl[0].zero_()
                else:
                    b.grad = torch.empty_like(b) if not a else torch.zeros_like(b)
            if a and id(W) in fresh:
                # (a fresh weight block paired with an already-accumulating bias: the block's
                # columns must start from zero too)
                W.grad[:, k0:k1].zero_()
            dys.append(dy)
            xs.append(x)
            dws.append(W.grad if full else W.grad[:, k0:k1])
            dbs.append(b.grad if b is not None else torch.empty(0, device=dy.device))
            acc.append(1 if a else 0)
            touched += [W] + ([b] if b is not None else [])
        if dys[0].is_cuda:
            _native.ops().linear_wgrad_grouped(dys, xs, dws, dbs, acc)
        else:  # CPU twin (multi-rank gloo tests of the flush / bucket protocol)
            _cpu_grouped(dys, xs, dws, dbs, acc)

    s = _gradslots.active()
    mark = s is not None and hasattr(s, "deferred_flush")
    if mark:
        s.deferred_flush(True)
    try:
        seen = set()
        for p in touched:
            if id(p) not in seen:
                seen.add(id(p))
                _run_post_hooks(p)
    finally:
        if mark:
            s.deferred_flush(False)


@torch.no_grad()
def _cpu_grouped(dys, xs, dws, dbs, acc):
    for dy, x, dw, db, a in zip(dys, xs, dws, dbs, acc):
        gw = dy.t() @ x
        dw.add_(gw) if a else dw.copy_(gw)
        if db.numel():
            gb = dy.sum(0)
            db.add_(gb) if a else db.copy_(gb)


def _run_post_hooks(p):
    hooks = getattr(p, "_post_accumulate_grad_hooks", None)
    if hooks:
        for h in hooks.values():
            h(p)


class _TallLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        ctx.params = (W, b)
        return F.linear(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dx = dy @ W if ctx.needs_input_grad[0] else None
        dW = db = None
        Wp, bp = ctx.params
        if ctx.needs_input_grad[1] and (not ctx.has_b or ctx.needs_input_grad[2]) and _can_defer(Wp, bp):
            _record((dy, x, Wp, bp))
            return dx, None, None
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            dW, db = _native.ops().linear_wgrad(dy, x, ctx.has_b)
            if not ctx.has_b:
                db = None
        return dx, dW, db


class _WGrad2(torch.autograd.Function):
    """dW = dy^T x (+ db = sum_n dy) on the split-K weight-gradient kernel, differentiable once
    more: the weight gradient formed inside a create_graph backward (force training's first
    pass) stays part of the second pass's graph."""

    @staticmethod
    def forward(ctx, dy, x, has_b):
        ctx.save_for_backward(dy, x)
        dW, db = _native.ops().linear_wgrad(dy.contiguous(), x.contiguous(), has_b)
        return dW, db

    @staticmethod
    def backward(ctx, gW, gb):
        dy, x = ctx.saved_tensors
        d_dy = x @ gW.t() if gW is not None else None
        if gb is not None and gb.numel():
            d_dy = gb.expand(dy.shape[0], -1) if d_dy is None else d_dy + gb
        d_x = dy @ gW if gW is not None else None
        return d_dy, d_x, None


class _MM2(torch.autograd.Function):
    """dx = dy @ W recorded by a create_graph backward: its own weight gradient dy^T h (an
    edge- or node-length reduction, the second-order term of force training) runs on the
    split-K kernel instead of a library GEMM that picks 2 workgroups for K ~ 10^4."""

    @staticmethod
    def forward(ctx, dy, W, Wp=None):
        ctx.save_for_backward(dy, W)
        ctx.param = Wp  # the Parameter (deferral needs it: W may be a view or detached alias)
        return dy @ W

    @staticmethod
    def backward(ctx, h):
        dy, W = ctx.saved_tensors
        d_dy = h @ W.t() if ctx.needs_input_grad[0] else None
        d_W = None
        if ctx.needs_input_grad[1]:
            # dW[o, i] = sum_n dy[n, o] h[n, i]: the kernel's dY^T X with (dY, X) = (dy, h);
            # inside the step's backward it joins the deferred grouped launch
            Wp = ctx.param
            if Wp is not None and _can_defer(Wp, None):
                _record((dy, h.contiguous(), Wp, None))
            else:
                d_W, _ = _native.ops().linear_wgrad(dy.contiguous(), h.contiguous(), False)
        return d_dy, d_W, None


class _LinearC(torch.autograd.Function):
    """Composite-mode (force training) linear: twice differentiable like F.linear, with every
    weight gradient of both backward passes on the split-K kernel (``_WGrad2`` / ``_MM2``)."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        ctx.params = (W, b)
        return F.linear(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        Wp, bp = ctx.params
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = _MM2.apply(dy, W, Wp if isinstance(Wp, torch.nn.Parameter) else None) if torch.is_grad_enabled() \
                else dy @ W
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            if torch.is_grad_enabled():
                dW, db = _WGrad2.apply(dy, x, ctx.has_b)
            elif ctx.needs_input_grad[1] and (not ctx.has_b or ctx.needs_input_grad[2]) and _can_defer(Wp, bp):
                _record((dy, x, Wp, bp))  # the step's deferred grouped weight-gradient launch
                return dx, None, None
            else:
                dW, db = _native.ops().linear_wgrad(dy.contiguous(), x.contiguous(), ctx.has_b)
            if not ctx.has_b:
                db = None
        return dx, dW, db


def _composite_tall(x, W, b):
    """The composite-mode linear takes the split-K weight gradients (GPU fp32, tall input)."""
    return (_mode._state["composite"] and "linear" not in _mode._state["off"] and _COMPOSITE_SK and x.is_cuda
            and x.dtype == torch.float32 and W.dtype == torch.float32 and x.dim() == 2 and x.shape[0] >= MIN_ROWS
            and torch.is_grad_enabled() and (x.requires_grad or W.requires_grad))


# HYDRA_COMPOSITE_SPLITK=0: composite-mode linears on plain F.linear (autograd's library GEMMs)
_COMPOSITE_SK = os.environ.get("HYDRA_COMPOSITE_SPLITK", "1") == "1"


class _TallLinearRelu(torch.autograd.Function):
    """relu(x W^T + b) with the ReLU in the library GEMM's epilogue (torch._addmm_activation:
    no separate [M, O] activation pass); backward masks dy by y > 0, then as _TallLinear."""

    @staticmethod
    def forward(ctx, x, W, b):
        y = torch._addmm_activation(b, x, W.t())
        ctx.save_for_backward(x, W, y)
        ctx.params = (W, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, y = ctx.saved_tensors
        dz = torch.ops.aten.threshold_backward(dy, y, 0.0)
        dx = dz @ W if ctx.needs_input_grad[0] else None
        Wp, bp = ctx.params
        if ctx.needs_input_grad[1] and ctx.needs_input_grad[2] and _can_defer(Wp, bp):
            _record((dz, x, Wp, bp))
            return dx, None, None
        dW = db = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dW, db = _native.ops().linear_wgrad(dz, x, True)
        return dx, dW, db


# HYDRA_LINEAR_RELU_EPI=0: tall linear + ReLU as two launches (GEMM, then the activation)
_RELU_EPI = os.environ.get("HYDRA_LINEAR_RELU_EPI", "1") == "1"


class _ColBlockLinear(torch.autograd.Function):
    """y = x @ W[:, k0:k0+K]^T for a column block of a (concat-)linear weight: the block's
    weight gradient joins the deferred grouped launch as a column-block problem (``_span``)
    instead of autograd's slice backward (a zero-filled full gradient plus a library GEMM
    with a ~10^4-row reduction dimension on a handful of workgroups)."""

    @staticmethod
    def forward(ctx, x, W, k0):
        K = x.shape[1]
        w = W[:, k0:k0 + K]
        ctx.save_for_backward(x, W)
        ctx.k0 = k0
        return F.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        k0, K = ctx.k0, x.shape[1]
        w = W[:, k0:k0 + K]
        dx = dy @ w if ctx.needs_input_grad[0] else None
        dW = None
        if ctx.needs_input_grad[1]:
            if _can_defer(W, None):
                _record((dy, x, W, None, k0))
            else:
                dW = torch.zeros_like(W)
                g, _ = _native.ops().linear_wgrad(dy.contiguous(), x.contiguous(), False)
                dW[:, k0:k0 + K] = g
        return dx, dW, None


def linear_cols(x, W, k0):
    """``F.linear(x, W[:, k0:k0 + x.shape[1]])`` — one column block of a concat-linear weight
    (GPU fp32 tall inputs: grouped deferred weight gradient; otherwise plain autograd)."""
    if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[0] >= MIN_ROWS and \
            torch.is_grad_enabled() and W.requires_grad and _mode.fused("linear"):
        return _ColBlockLinear.apply(x.contiguous(), W, int(k0))
    return F.linear(x, W[:, k0:k0 + x.shape[1]])


_EDGE_LINEAR = os.environ.get("HYDRA_EDGE_LINEAR", "1") == "1"


def _edge_linear_ok(xs, ws, b):
    return (_EDGE_LINEAR and len(xs) <= 3 and all(t.is_cuda and t.dtype == torch.float32 for t in list(xs) + list(ws))
            and all(x.dim() == 2 and x.stride(1) == 1 for x in xs) and sum(w.shape[1] for w in ws) <= 188
            and (b is None or b.dtype == torch.float32))


def _dgrad(dy, w):
    """dX = dY @ W of an edge-sized linear (library GEMM: the edge-linear kernel measured
    on par, 9.5 us per call at 23k x 64 @ 64 x 64 on MI355X, and was removed)."""
    return dy @ w


class _TallLinearSum(torch.autograd.Function):
    """y = sum_k x_k @ W_k^T + b  (one output, several inputs; e.g. a concat-linear
    split into its column blocks so the concat is never materialised)."""

    @staticmethod
    def forward(ctx, b, *xw):
        xs, ws = xw[0::2], xw[1::2]
        ctx.save_for_backward(*xs, *ws)
        ctx.k = len(xs)
        ctx.has_b = b is not None
        ctx.params = (b, tuple(ws))
        if _edge_linear_ok(xs, ws, b):
            # one pass (csrc/linear.hip edge_linear_fwd) instead of bias copy + GEMM + addmm
            return _native.ops().edge_linear_fwd(list(xs), list(ws), b)
        y = F.linear(xs[0], ws[0], b)
        for x, w in zip(xs[1:], ws[1:]):
            y = torch.addmm(y, x, w.t())
        return y

    @staticmethod
    def backward(ctx, dy):
        t = ctx.saved_tensors
        xs, ws = t[:ctx.k], t[ctx.k:]
        grads = []
        db = None
        bp, wps = ctx.params
        if all(ctx.needs_input_grad[2 + 2 * j] for j in range(ctx.k)) and \
                (not ctx.has_b or ctx.needs_input_grad[0]) and all(_can_defer(w, None) for w in wps) and \
                _can_defer(wps[0], bp) and len({id(w) for w in wps}) == len(wps):
            for j, (x, w) in enumerate(zip(xs, ws)):
                _record((dy, x, wps[j], bp if j == 0 else None))
                grads += [_dgrad(dy, w) if ctx.needs_input_grad[1 + 2 * j] else None, None]
            return (None, *grads)
        # non-leaf weights (e.g. the PNA weight-prep outputs): all k weight gradients of this
        # sum in ONE grouped launch pair (they share dY)
        need_w = [bool(ctx.needs_input_grad[2 + 2 * j]) for j in range(ctx.k)]
        want_b = ctx.has_b and ctx.needs_input_grad[0]
        dws = [torch.empty(w.shape, device=w.device, dtype=w.dtype) if (need_w[j] or (want_b and j == 0)) else None
               for j, w in enumerate(ws)]
        if want_b:
            db = torch.empty(ws[0].shape[0], device=dy.device, dtype=dy.dtype)
        sel = [j for j in range(ctx.k) if dws[j] is not None]
        if sel:
            _native.ops().linear_wgrad_grouped(
                [dy] * len(sel), [xs[j] for j in sel], [dws[j] for j in sel],
                [db if (want_b and j == 0) else torch.empty(0, device=dy.device) for j in sel], [0] * len(sel))
        for j, (x, w) in enumerate(zip(xs, ws)):
            dx = _dgrad(dy, w) if ctx.needs_input_grad[1 + 2 * j] else None
            grads += [dx, dws[j] if need_w[j] else None]
        return (db, *grads)


class _EngineSumF32(_TallLinearSum):
    """fp32 concat-linear: one engine launch forward (instead of one GEMM per input block),
    library dgrad + split-K wgrad backward."""

    @staticmethod
    def forward(ctx, b, *xw):
        xs, ws = xw[0::2], xw[1::2]
        ctx.save_for_backward(*xs, *ws)
        ctx.k = len(xs)
        ctx.has_b = b is not None
        ctx.params = (b, tuple(ws))
        return _native.ops().mm_fwd([_row_contig(x) for x in xs], [_row_contig(w) for w in ws], b, None, 0, 0)


MIN_ROWS = 1024  # below this the library GEMM is already latency-bound and fine
# HYDRA_ENGINE_FWD1=1: single-input tall fp32 forwards on the engine instead of the library GEMM
# (A/B on MI355X, profiles/r5_ab_engine_fwd1.log: DimeNet 3.12 -> 3.44 ms, SchNet 0.404 -> 0.427 ms: off)
_ENGINE_FWD1 = os.environ.get("HYDRA_ENGINE_FWD1", "0") == "1"
BF16_MIN_MACS = int(os.environ.get("HYDRA_BF16_MIN_MACS", str(1 << 26)))
ENGINE_SUM_MAX_ROWS = 8192  # fp32 multi-input sums above this use the library GEMM pair


def _engine_ok(tensors):
    return _mode.fused("linear") and all(
        t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 for t in tensors)


def linear_act(pairs, b=None, act=ACT_NONE, residual=None):
    """``act(sum_k x_k @ W_k^T + b) (+ residual)`` for 1-3 (x_k, W_k) pairs.

    bf16 precision: single-input maps above BF16_MIN_MACS run on the bf16 MFMA engine
    (csrc/bgemm.hip, ``ops.bgemm.BF16Linear``).  fp32: measured on MI355X
    (tools/bench_mm.py, profiles/r2_bench_mm.log) the library GEMM is faster for the
    plain single-input forward and the dgrad of these shapes, and the engine's in-launch
    split-K reduction loses to a separate reduce launch whenever the grid has more than a
    few dozen workgroups (agent-scope release fences under load), so fp32 uses: library
    GEMM forward + dgrad, split-K weight-gradient kernel + reduce, and the engine only for
    multi-input concat-linear forwards (one launch instead of one per input block)."""
    assert not (act == ACT_RELU and residual is not None), "residual is added after the activation: relu+residual unsupported"
    xs = [p[0] for p in pairs]
    ws = [p[1] for p in pairs]
    engine = len(pairs) <= 3 and _engine_ok(xs + ws) and xs[0].shape[0] > 0 and \
        (residual is None or (residual.is_cuda and residual.dtype == torch.float32))
    # bf16 precision pays only where the GEMM is big enough to be compute-bound: below
    # BF16_MIN_MACS (QM9-sized SchNet maps, ~1-20 M MACs) the launch-bound library fp32
    # path is faster than rounding into the MFMA engine (measured on MI355X: QM9 SchNet
    # 72.5 k graphs/s fp32 vs 44.9 k with every map on the bf16 engine), and fp32 is the
    # more accurate of the two, so small maps stay fp32 in bf16 mode
    bf16 = _state["prec"] == 1 and \
        sum(x.shape[0] * w.shape[0] * w.shape[1] for x, w in zip(xs, ws)) >= BF16_MIN_MACS
    if engine and bf16 and len(pairs) == 1 and residual is None and min(ws[0].shape) >= 16:
        # wide maps (the SC25 EGNN decoder heads, 866 -> 889 -> ...): the bf16 MFMA engine
        # of csrc/bgemm.hip (padded bf16 operands, fp32 accumulate, fused bias/ReLU,
        # split-row weight gradient with the bias gradient from the ones lane)
        from . import bgemm

        return bgemm.bf16_linear(xs[0], ws[0], b, act)
    # narrow maps (e.g. an 866 -> 1 projection) and multi-input sums stay on the fp32 path
    tall = engine and xs[0].shape[0] >= MIN_ROWS and torch.is_grad_enabled() and \
        any(t.requires_grad for t in xs + ws + ([b] if b is not None else []))
    if len(pairs) == 1 and _composite_tall(xs[0], ws[0], b):
        # force training: split-K weight gradients in both passes; the activation and the
        # residual stay twice-differentiable torch ops
        y = _LinearC.apply(xs[0], ws[0], b)
        if act == ACT_RELU:
            y = torch.relu(y)
        return y if residual is None else y + residual
    if (len(pairs) == 1 and tall and act == ACT_RELU and b is not None and residual is None and _RELU_EPI
            and not _ENGINE_FWD1):
        return _TallLinearRelu.apply(xs[0], ws[0], b)
    if len(pairs) == 1:
        if tall and _ENGINE_FWD1 and xs[0].shape[0] < ENGINE_SUM_MAX_ROWS * 4:
            y = _EngineSumF32.apply(b, xs[0], ws[0])  # HYDRA_ENGINE_FWD1=1: engine forward (A/B knob)
        else:
            y = _TallLinear.apply(xs[0], ws[0], b) if tall else F.linear(xs[0], ws[0], b)
    elif tall:
        flat = []
        for x, w in zip(xs, ws):
            flat += [x, w]
        # fp32 concat-linear: the engine's one-launch forward wins on node-sized inputs; on
        # edge-sized ones (PNAPlus radial term, 23k x 65 -> 64) the library GEMM + addmm pair
        # is ~2x faster on MI355X (30-40 us vs ~14 us, profiles/r2_rocprof_headline_sequence.txt)
        y = (_EngineSumF32 if xs[0].shape[0] < ENGINE_SUM_MAX_ROWS else _TallLinearSum).apply(b, *flat)
    else:
        y = F.linear(xs[0], ws[0], b)
        for x, w in zip(xs[1:], ws[1:]):
            y = y + F.linear(x, w)
    if act == ACT_RELU:
        y = torch.relu(y)
    if residual is not None:
        y = y + residual
    return y


def linear(x, W, b=None, act=ACT_NONE):
    if x.dim() != 2:
        sh = x.shape
        return linear(x.reshape(-1, sh[-1]), W, b, act).view(*sh[:-1], W.shape[0])
    return linear_act([(x, W)], b, act)


def linear_sum(pairs, b=None):
    """sum_k F.linear(x_k, W_k) + b in one launch (no concatenation)."""
    return linear_act(pairs, b)
