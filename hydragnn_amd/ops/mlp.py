"""Fused Linear/ReLU chains for the graph-level heads (``csrc/mlp.hip``).

Reference: the per-branch shared MLP + per-head MLP of ``Base._multihead``
(``hydragnn/models/Base.py:246-287``) applied to pooled graph features.  On the
GPU a chain of up to 8 Linear(+ReLU) layers of width <= 128 over <= 1024 rows is
one forward and two backward launches; anything else (CPU, other activations,
composite/double-backward mode) runs the modules as written.
"""
import os

import torch
from torch import nn

from .. import _native
from ..parallel import gradslots as _gradslots
from . import pna as _mode
from . import streams as _streams

MAX_ROWS = 1024
ROWS = 4  # rows per workgroup (csrc/mlp.hip kMlpRows)
MAX_DIM = 128
MAX_LAYERS = 8
MAX_LDS = 159 * 1024


def _lds_ok(G, dims):
    """LDS footprint of the fused kernels (``csrc/mlp.hip`` fwd_lds / bwd_lds)."""
    w = sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
    md = max(dims) + 1
    fwd = 4 * (w + 2 * ROWS * md)
    bwd = 4 * (w + ROWS * (sum(dims[1:]) + dims[0] + md))
    return max(fwd, bwd) <= MAX_LDS


class _FusedMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, relu, *params):
        out, acts = _native.ops().mlp_fwd(x, params[0::2], params[1::2], relu)
        ctx.save_for_backward(x, acts, *params)
        ctx.relu = relu
        return out

    @staticmethod
    def backward(ctx, dout):
        x, acts, *params = ctx.saved_tensors
        dx, dWs, dbs = _native.ops().mlp_bwd(dout, x, acts, params[0::2], params[1::2], ctx.relu)
        grads = []
        for dW, db in zip(dWs, dbs):
            grads += [dW, db]
        return (dx, None, *grads)


def _chain(seqs):
    """[(Linear, relu_after)] for Sequentials made only of Linear and ReLU, else None."""
    layers = []
    for s in seqs:
        for m in s:
            if isinstance(m, nn.Linear):
                if m.bias is None:
                    return None
                layers.append([m, False])
            elif isinstance(m, nn.ReLU) and layers and not layers[-1][1]:
                layers[-1][1] = True
            else:
                return None
    return layers


def sequential_chain(x, *seqs):
    """``seqs[-1](...seqs[0](x))`` — fused on the GPU when the chain qualifies."""
    if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and _mode.fused("mlp") \
            and 0 < x.shape[0] <= MAX_ROWS:
        layers = _chain(seqs)
        dims = [x.shape[1]] + [m.weight.shape[0] for m, _ in layers] if layers else []
        if layers and len(layers) <= MAX_LAYERS and max(dims) <= MAX_DIM and _lds_ok(x.shape[0], dims) and \
                all(m.weight.dtype == torch.float32 for m, _ in layers):
            params = []
            for m, _ in layers:
                params += [m.weight, m.bias]
            return _FusedMLP.apply(x.contiguous(), [int(r) for _, r in layers], *params)
    for s in seqs:
        x = s(x)
    return x


# ---------------------------------------------------------------- head + loss
HL_MAX_LDS = 150 * 1024
_KIND = {"mse": 0, "mae": 1, "rmse": 2, "smooth_l1": 3}


def _hl_lds(G, dims):
    """LDS footprint of ``csrc/mlp.hip`` head_loss kernels (hl_layout): every matrix is
    [rows padded to 16][cols padded to 16, + 1]."""
    r16 = lambda v: (v + 15) // 16 * 16
    ld = lambda c: r16(c) + 1
    Gp = r16(G)
    w = sum(r16(dims[i + 1]) * ld(dims[i]) + r16(dims[i + 1]) for i in range(len(dims) - 1))
    acts = sum(Gp * ld(d) for d in dims[1:])
    # + targets [G][out] and the row mask [Gp]
    return 4 * (w + Gp * ld(dims[0]) + acts + 2 * Gp * ld(max(dims)) + G * dims[-1] + Gp)


def head_loss_layers(seqs, G, in_dim, kind):
    """[(Linear, relu)] when ``seqs`` + a masked ``kind`` loss over G rows fit the one-
    workgroup head+loss kernels, else None."""
    if kind not in _KIND or not _mode.fused("headloss") or not _mode.fused("mlp") or G < 1:
        return None
    layers = _chain(seqs)
    if not layers or len(layers) > MAX_LAYERS:
        return None
    dims = [in_dim] + [m.weight.shape[0] for m, _ in layers]
    if max(dims) > MAX_DIM or _hl_lds(G, dims) > HL_MAX_LDS:
        return None
    if any(m.weight.dtype != torch.float32 or not m.weight.is_cuda for m, _ in layers):
        return None
    return layers


def mark_unit_seed(t):
    """Declare ``t`` a persistent all-ones backward seed (the training step's d loss / d loss):
    a fused head+loss whose upstream gradient IS this tensor returns its precomputed
    gradients without a scaling launch."""
    t._hydra_unit_seed = True
    return t


class _HeadLoss(torch.autograd.Function):
    """loss = masked_loss(MLP(x), target) as one forward and one backward launch; with
    ``fused`` (training), the forward launch also computes every gradient for a unit
    upstream gradient (``head_loss_fused``) and the backward only scales them by ``g`` —
    nothing at all when ``g`` is the step's unit seed (``mark_unit_seed``)."""

    @staticmethod
    def forward(ctx, x, target, mask, kind, relu, fused, *params):
        ctx.fused = fused
        ctx.set_materialize_grads(False)  # no zero-filled gradient for pred
        ctx.slotted = False
        if fused:
            sl = _side_slots(x, kind, params)
            if sl is not None:
                return _HeadLoss._forward_side(ctx, x, target, mask, kind, relu, params, sl)
            out = _native.ops().head_loss_fused(x, params[0::2], params[1::2], relu, target, mask, kind)
            stats, pred = out[0], out[1]
            ctx.grads = out[2:]
            ctx.mark_non_differentiable(pred)
            return stats[0], pred
        stats, pred, acts = _native.ops().head_loss_fwd(x, params[0::2], params[1::2], relu, target, mask, kind)
        ctx.save_for_backward(x, acts, target, mask, stats, *params)
        ctx.kind, ctx.relu = kind, relu
        ctx.mark_non_differentiable(pred)
        return stats[0], pred

    @staticmethod
    def _forward_side(ctx, x, target, mask, kind, relu, params, sl):
        """Training step with gradient slots: the critical path gets only dx (the forward and
        input-gradient chains, ``head_loss_dx``); the same kernel in full mode runs on a side
        stream and writes predictions, the loss and every weight gradient — straight into the
        step's flat gradient slots — overlapped with the encoder's backward."""
        ops = _native.ops()
        Ws, bs = params[0::2], params[1::2]
        main = torch.cuda.current_stream(x.device)
        side = _streams.side_stream(x.device, 4)
        # the twin is forked BEFORE the dx launch: a hipGraph node with two successors on
        # different streams delays both (~7 us), and the dx launch's successor is the encoder
        # backward (the critical path)
        side.wait_stream(main)
        for t in (x, target, mask):
            if t is not None:
                t.record_stream(side)
        with torch.cuda.stream(side):
            out = ops.head_loss_fused(x, Ws, bs, relu, target, mask, kind, None, sl, False)
        ev = torch.cuda.Event()
        ev.record(side)
        dx = ops.head_loss_dx(x, Ws, bs, relu, target, mask, kind)
        stats, pred = out[0], out[1]
        # loss / predictions are read after the step's gradient join (finish): the main stream
        # waits for the side stream there; until then keep their memory out of reuse
        stats.record_stream(main)
        pred.record_stream(main)
        _gradslots.provide(list(params), ev)
        ctx.slotted = True
        ctx.dx = dx
        ctx.nparams = len(params)
        ctx.mark_non_differentiable(pred)
        return stats[0], pred

    @staticmethod
    def backward(ctx, g, _gpred):
        if ctx.slotted:
            dx = ctx.dx
            ctx.dx = None
            if g is None:
                return (None,) * (6 + ctx.nparams)
            if not getattr(g, "_hydra_unit_seed", False):
                raise RuntimeError("head_loss: slotted gradients need the step's unit backward seed")
            return (dx, None, None, None, None, None) + (None,) * ctx.nparams
        if ctx.fused:
            grads = ctx.grads
            ctx.grads = None
            if g is None:
                return (None,) * (6 + len(grads) - 1)
            if not getattr(g, "_hydra_unit_seed", False):
                grads = [t * g for t in grads]
            return (grads[0], None, None, None, None, None, *grads[1:])
        x, acts, target, mask, stats, *params = ctx.saved_tensors
        out = _native.ops().head_loss_bwd(g.reshape(1).contiguous(), x, acts, params[0::2], params[1::2], ctx.relu,
                                          target, mask, stats, ctx.kind)
        return (out[0], None, None, None, None, None, *out[1:])


_side_state = {"ok": True}


def _side_slots(x, kind, params):
    """Gradient slots for the head's parameters when the side-stream split applies (training
    step under ``parallel.gradslots.use``, CUDA, not RMSE — its dx needs the batch loss), else
    None.  ``HYDRA_HEADLOSS_SIDE``: ``auto`` (default) follows the caller's hint (``head_loss``
    ``side``: on for the fused GPS encoder, where the twin overlaps the multi-stream backward;
    measured off for launch-bound steps such as QM9 SchNet: 0.51 vs 0.57-0.67 ms/step), ``1``
    always, ``0`` never."""
    mode = os.environ.get("HYDRA_HEADLOSS_SIDE", "auto")
    if not x.is_cuda or kind == _KIND["rmse"] or mode == "0" or (mode != "1" and not _side_state["ok"]):
        return None
    if not _streams.enabled(x):
        return None
    return _gradslots.slots(params)


def head_loss(x, layers, target, mask, kind, fused=None, side=True):
    """(loss, pred) of a masked-loss graph head over the pooled features ``x``.  ``fused``
    (default: when grad mode is on; ``HYDRA_HEADLOSS_FUSED=0`` disables): gradients computed
    inside the forward launch (see ``_HeadLoss``).  ``side``: the side-stream split may apply
    (see ``_side_slots``)."""
    params = []
    for m, _ in layers:
        params += [m.weight, m.bias]
    if fused is None:
        fused = torch.is_grad_enabled() and os.environ.get("HYDRA_HEADLOSS_FUSED", "1") == "1"
    prev = _side_state["ok"]
    _side_state["ok"] = bool(side)
    try:
        return _HeadLoss.apply(x.contiguous(), target.contiguous(), None if mask is None else mask.contiguous(),
                               _KIND[kind], [int(r) for _, r in layers], bool(fused), *params)
    finally:
        _side_state["ok"] = prev
