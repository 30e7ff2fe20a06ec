"""Host side of the bf16 MFMA GEMM engine (``csrc/bgemm.hip``).

Padded-bf16 convention (see the kernel file): an activation with ``K`` valid columns is
a bf16 ``[rows, Kp]`` matrix, ``Kp = pad(K)``, zero pad columns except the *ones lane*
at column ``K`` (value 1.0); padded weights are bf16 ``[Np, Kp]`` (and ``[Kp, Np]``
transposed images for the data-gradient products) with zero padding.  A weight-gradient
product ``dY^T X`` then carries the bias gradient in its column ``K``.

``BF16Linear`` is the bf16-precision ``linear`` for wide maps (>= ``BF16_MIN_MACS``):
fp32 in / fp32 out at the module boundary, bf16 MFMA inside (operands rounded to bf16,
fp32 accumulation), backward = one data-gradient NT GEMM and one split-M weight-gradient
TN GEMM + slab reduce (bias gradient from the ones lane).
"""
import torch

from .. import _native

ACT = {"none": 0, "relu": 1, "silu": 2}


def pad64(k):
    return (k + 64) // 64 * 64  # strictly greater than k: room for the ones lane


def pad128(k):
    return (k + 128) // 128 * 128


def padded(rows, k, dev, pad=pad128):
    return torch.empty((rows, pad(k)), device=dev, dtype=torch.bfloat16)


def cast_pad(x, kp=None, gate=None, ones=True, out=None):
    """fp32 [M, K] -> padded bf16 [M, kp] (ones lane at column K), optionally zeroed where
    ``gate`` (padded bf16) <= 0 (ReLU derivative)."""
    M, K = x.shape
    if out is None:
        out = torch.empty((M, kp or pad128(K)), device=x.device, dtype=torch.bfloat16)
    _native.ops().bg_cast_pad(x if x.stride(1) == 1 else x.contiguous(), out, gate, K if ones else -1)
    return out


def weight_images(Ws, kps=None, nps=None, need=(True, True)):
    """bf16 padded images of fp32 weights ``W [N, K]`` (one batched launch): returns a list
    of (Wb [Np, Kp], WbT [Kp, Np]) (either may be None per ``need``)."""
    srcs, d, dt, out = [], [], [], []
    for i, W in enumerate(Ws):
        N, K = W.shape
        kp = kps[i] if kps else pad128(K)
        np_ = nps[i] if nps else pad128(N - 1)
        e = torch.empty(0, device=W.device, dtype=torch.bfloat16)
        wb = torch.empty((np_, kp), device=W.device, dtype=torch.bfloat16) if need[0] else None
        wt = torch.empty((kp, np_), device=W.device, dtype=torch.bfloat16) if need[1] else None
        srcs.append(W if W.stride(1) == 1 else W.contiguous())
        d.append(wb if wb is not None else e)
        dt.append(wt if wt is not None else e)
        out.append((wb, wt))
    _native.ops().bg_cast_weights(srcs, d, dt)
    return out


def nt(A, B, K, N, *, A2=None, k1=None, bias=None, act=0, gate=None, addg=None, addg_idx=None, outf=None, beta=0.0,
       outb=None, ones_col=-1, rowvec=None, rowdot=None, bm=None):
    """epi(A @ B^T): A [M, >=K] padded bf16 (or [A | A2] concatenated at column k1), B
    [Np, >=K] padded bf16 weight image; writes ``outf`` (fp32, first N columns) and/or
    ``outb`` (padded bf16, all Np columns)."""
    if bm is None:
        # >= ~2 workgroups per CU: big row counts take the 256-row tile (half the B
        # traffic), node-sized ones the 64-row tile
        tiles_n = B.shape[0] // 128
        M = A.shape[0]
        bm = 256 if (M + 255) // 256 * tiles_n >= 512 else (128 if (M + 127) // 128 * tiles_n >= 512 else 64)
    _native.ops().bg_nt(A, A2, K if k1 is None else k1, B, K, N, bias, act, gate, addg, addg_idx, outf, beta, outb,
                        ones_col, rowvec, rowdot, bm)


_slabs = {}


def _slab(dev, numel):
    key = (dev, torch.cuda.current_stream(dev).stream_id if dev.type == "cuda" else 0)
    s = _slabs.get(key)
    if s is None or s.numel() < numel or torch.cuda.is_current_stream_capturing():
        # captured steps own their workspace (graph memory pool); eager calls reuse one
        s = torch.empty(max(numel, 1 << 20), device=dev, dtype=torch.float32)
        if not torch.cuda.is_current_stream_capturing():
            _slabs[key] = s
    return s


def splits_for(M, tiles):
    """Row splits of a weight-gradient product: ~2 workgroups per CU, >= 2 K-steps each."""
    s = max(1, min(64, (512 + tiles - 1) // tiles))
    while s > 1 and M / s < 128:
        s //= 2
    return s


def wgrad(G, X, Np, Kp, outs, *, X2=None, kc1=None, beta=0.0):
    """Weight gradients ``G^T [X | X2]`` ([Np, Kp] fp32, split over rows) reduced into
    ``outs``: a list of (out [N, K] fp32 view, row0, bias_out or None, bias_col[, col0])."""
    M = G.shape[0]
    S = splits_for(M, (Np // 128) * (Kp // 128))
    slab = _slab(G.device, S * Np * Kp)
    _native.ops().bg_tn(G, X, X2, Kp if kc1 is None else kc1, Np, Kp, slab, S)
    for o in outs:
        out, n0, bias_out, bias_col = o[:4]
        k0 = o[4] if len(o) > 4 else 0
        _native.ops().bg_slab_reduce(slab, S, Np, Kp, n0, k0, out.shape[0], out.shape[1], out, beta, bias_col,
                                     bias_out)


def _accum_grad(p, g):
    """fresh tensor for ``p.grad`` accumulation target (beta = 1 when a grad exists)."""
    if p.grad is None:
        p.grad = torch.empty_like(p)
        return p.grad, 0.0
    return p.grad, 1.0


class BF16Linear(torch.autograd.Function):
    """``act(x W^T + b)`` with bf16 MFMA operands and fp32 in/out (see module doc)."""

    @staticmethod
    def forward(ctx, x, W, b, act):
        M, K = x.shape
        N = W.shape[0]
        kp, np_ = pad128(K), pad128(N - 1)
        xb = cast_pad(x, kp)
        (wb, _), = weight_images([W], [kp], [np_], need=(True, False))
        y = torch.empty((M, N), device=x.device, dtype=torch.float32)
        yb = torch.empty((M, np_), device=x.device, dtype=torch.bfloat16) if act == 1 else None
        nt(xb, wb, kp, N, bias=b, act=act, outf=y, outb=yb)
        ctx.save_for_backward(xb, W, yb)
        ctx.dims = (K, N, kp, np_, act, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, W, yb = ctx.saved_tensors
        K, N, kp, np_, act, has_b = ctx.dims
        M = xb.shape[0]
        # gradient at the pre-activation, padded bf16 (ReLU derivative from the saved output)
        g = cast_pad(dy, np_, gate=yb if act == 1 else None, ones=False)
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            (_, wt), = weight_images([W], [kp], [np_], need=(False, True))
            dx = torch.empty((M, K), device=dy.device, dtype=torch.float32)
            nt(g, wt, np_, K, outf=dx)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dW = torch.empty_like(W)
            db = torch.empty(N, device=dy.device, dtype=torch.float32) if has_b else None
            wgrad(g, xb, np_, kp, [(dW, 0, db, K)])
        return dx, dW, db, None


def bf16_linear(x, W, b=None, act=0):
    return BF16Linear.apply(x, W, b, act)
