"""Host side of the bf16 MFMA GEMM engine (``csrc/bgemm.hip``).

Padded-bf16 convention (see the kernel file): an activation with ``K`` valid columns is
a bf16 ``[rows, Kp]`` matrix, ``Kp = pad(K)``, zero pad columns except the *ones lane*
at column ``K`` (value 1.0); padded weights are bf16 ``[Np, Kp]`` (and ``[Kp, Np]``
transposed images for the data-gradient products) with zero padding.  A weight-gradient
product ``dY^T X`` then carries the bias gradient in its column ``K``.

``BF16Linear`` is the bf16-precision ``linear`` for wide maps (>= ``BF16_MIN_MACS``):
fp32 in / fp32 out at the module boundary, bf16 MFMA inside (operands rounded to bf16,
fp32 accumulation), backward = one data-gradient NT GEMM and one split-M weight-gradient
TN GEMM whose last-arriving split block reduces each tile (bias gradient from the ones lane).
"""
import os

import torch

from .. import _native

ACT = {"none": 0, "relu": 1, "silu": 2}
GEMM_TILE = 1064  # NT kernel: 64-row tile, global_load_lds staging (1000 + rows; 64/128/256 = register staging)


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


stats = {"nt": 0}  # bf16 MFMA GEMM launches issued (incl. recorded into captured graphs)


def nt(A, B, K, N, *, A2=None, k1=None, bias=None, act=0, gate=None, addg=None, addg_idx=None, outf=None, beta=0.0,
       outb=None, ones_col=-1, rowvec=None, rowdot=None, bm=None):
    """epi(A @ B^T): A [M, >=K] padded bf16 (or [A | A2] concatenated at column k1), B
    [Np, >=K] padded bf16 weight image; writes ``outf`` (fp32, first N columns) and/or
    ``outb`` (padded bf16, all Np columns)."""
    if bm is None:
        # the glds-staged 64-row tile measured fastest on every EGNN shape on MI355X
        # (profiles/r3_bench_bgemm.log: 752 TF/s at 35k x 896 x 896 vs 571 for hipBLASLt)
        bm = GEMM_TILE
    stats["nt"] += 1
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


_counters = {}
_FUSED_TN_REDUCE = os.environ.get("HYDRA_TN_FUSED_REDUCE", "0") == "1"


def _counter_buf(dev, n):
    """Per-tile arrival counters of the fused TN reduce (zero between products: the last
    block of each tile resets its counter).  Shared by every product on one stream."""
    key = (dev, torch.cuda.current_stream(dev).stream_id)
    c = _counters.get(key)
    if c is None or c.numel() < n:
        c = torch.zeros(max(n, 1 << 14), device=dev, dtype=torch.int32)
        _counters[key] = c
    return c


def tn_reduce(G, X, Np, Kp, slab, S, outs, *, X2=None, kc1=None, boff=None, beta=0.0):
    """``slab = G^T [X | X2]`` split over rows, reduced in the same launch into ``outs``:
    (out, n0, k0, N, K, bias_out or None, bias_col) per destination (up to 3)."""
    groups = 1 if boff is None else boff.numel() - 1
    if not _FUSED_TN_REDUCE:
        # measured on MI355X (EGNN-866 bf16, profiles/r3_rocprof_cfg_multibranch_egnn_bf16_*):
        # the in-launch last-arriver reduce made tn_kernel 4.6x slower (30 -> 138 us per call,
        # device-scope release/acquire per split block under load) than the GEMM + one
        # slab_reduce launch per destination (12 us), so the separate reduce is the default
        _native.ops().bg_tn(G, X, X2, Kp if kc1 is None else kc1, Np, Kp, slab, S, boff, [], [], [], 0.0, None)
        for out, n0, k0, N, K, bias_out, bias_col in outs:
            _native.ops().bg_slab_reduce(slab, S, Np, Kp, n0, k0, N, K, out, beta, bias_col, bias_out, groups)
        return
    cnt = _counter_buf(G.device, groups * (Np // 128) * (Kp // 128))
    meta = []
    for o in outs:
        meta += [o[1], o[2], o[3], o[4], o[6]]
    _native.ops().bg_tn(G, X, X2, Kp if kc1 is None else kc1, Np, Kp, slab, S, boff, [o[0] for o in outs],
                        [o[5] for o in outs], meta, beta, cnt)


def splits_for(M, tiles):
    """Row splits of a weight-gradient product: ~1.5 workgroups per CU and >= 8 K-steps
    (512 rows) per split (fewer slabs for the reduce to read)."""
    return max(1, min(64, (384 + tiles - 1) // tiles, M // 512))


def wgrad(G, X, Np, Kp, outs, *, X2=None, kc1=None, beta=0.0):
    """Weight gradients ``G^T [X | X2]`` ([Np, Kp] fp32, split over rows) reduced into
    ``outs``: a list of (out [N, K] fp32 view, row0, bias_out or None, bias_col[, col0])."""
    M = G.shape[0]
    S = splits_for(M, (Np // 128) * (Kp // 128))
    slab = _slab(G.device, S * Np * Kp)
    dst = []
    for o in outs:
        out, n0, bias_out, bias_col = o[:4]
        k0 = o[4] if len(o) > 4 else 0
        dst.append((out, n0, k0, out.shape[0], out.shape[1], bias_out, bias_col))
    tn_reduce(G, X, Np, Kp, slab, S, dst, X2=X2, kc1=kc1, beta=beta)


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


# ---------------------------------------------------------------- branch-grouped heads
def _chain_layers(seq):
    """[(Linear, relu_after)] of a Sequential made of Linear (+bias) and ReLU, else None."""
    out = []
    for m in seq:
        if isinstance(m, torch.nn.Linear) and m.bias is not None:
            out.append([m, False])
        elif isinstance(m, torch.nn.ReLU) and out and not out[-1][1]:
            out[-1][1] = True
        else:
            return None
    return out


def branch_offsets(bid, nb):
    """Row offsets [nb + 1] (int32, on the device, no host sync) of rows sorted by branch."""
    cnt = (bid.view(-1, 1) == torch.arange(nb, device=bid.device, dtype=bid.dtype).view(1, -1)).sum(0)
    return torch.cat([torch.zeros(1, device=bid.device, dtype=torch.int64), torch.cumsum(cnt, 0)]).to(torch.int32)


class _BranchMLP(torch.autograd.Function):
    """Per-branch MLP chains over rows sorted by branch: every layer is ONE grouped NT GEMM
    (each row tile runs against its branch's weight image; a tile straddling a branch
    boundary runs once per branch present) and its weight gradients ONE grouped TN GEMM
    over each branch's own rows.  Replaces the captured step's dense decode (every branch
    head on every row, then a per-row select)."""

    @staticmethod
    def forward(ctx, x, bid, boff, dims, relu, nb, *params):
        M = x.shape[0]
        L = len(dims) - 1
        dev = x.device
        kps = [pad128(d) for d in dims]  # padded width of each layer's input / output
        imgs, imgTs, biases = [], [], []
        srcs, d, dt = [], [], []
        for l in range(L):
            img = torch.empty((nb, kps[l + 1], kps[l]), device=dev, dtype=torch.bfloat16)
            imgT = torch.empty((nb, kps[l], kps[l + 1]), device=dev, dtype=torch.bfloat16)
            for b in range(nb):
                srcs.append(params[(l * 2) * nb + b])
                d.append(img[b])
                dt.append(imgT[b])
            imgs.append(img)
            imgTs.append(imgT)
            biases.append(torch.stack([params[(l * 2 + 1) * nb + b] for b in range(nb)]).contiguous())
        _native.ops().bg_cast_weights(srcs, d, dt)
        h = cast_pad(x, kps[0])
        hs = [h]
        out = None
        for l in range(L):
            last = l == L - 1
            Np = kps[l + 1]
            if last:
                out = torch.empty((M, dims[-1]), device=dev, dtype=torch.float32)
                _native.ops().bg_nt(h, None, kps[l], imgs[l][0], kps[l], dims[l + 1], biases[l], int(relu[l]), None,
                                    None, None, out, 0.0, None, -1, None, None, GEMM_TILE, bid, imgs[l][0].numel(),
                                    dims[l + 1])
            else:
                hn = torch.empty((M, Np), device=dev, dtype=torch.bfloat16)
                _native.ops().bg_nt(h, None, kps[l], imgs[l][0], kps[l], dims[l + 1], biases[l], int(relu[l]), None,
                                    None, None, None, 0.0, hn, dims[l + 1], None, None, GEMM_TILE, bid, imgs[l][0].numel(),
                                    dims[l + 1])
                h = hn
                hs.append(h)
        ctx.save_for_backward(bid, boff, *hs)
        ctx.imgTs, ctx.dims, ctx.relu, ctx.nb, ctx.kps = imgTs, dims, relu, nb, kps
        ctx.shapes = [tuple(p.shape) for p in params]
        return out

    @staticmethod
    def backward(ctx, dout):
        bid, boff, *hs = ctx.saved_tensors
        dims, relu, nb, kps, imgTs = ctx.dims, ctx.relu, ctx.nb, ctx.kps, ctx.imgTs
        L = len(dims) - 1
        M = dout.shape[0]
        dev = dout.device
        grads = [None] * (2 * L * nb)
        # gradient at the last pre-activation
        g = cast_pad(dout, kps[L], gate=None, ones=False) if not relu[L - 1] else None
        if g is None:
            raise NotImplementedError("branch MLP ending in an activation")
        dx = None
        S = splits_for(max(1, M // nb), (kps[L] // 128) * (kps[L - 1] // 128))
        for l in range(L - 1, -1, -1):
            Np, Kp = kps[l + 1], kps[l]
            slab = _slab(dev, nb * S * Np * Kp)
            # every branch's weight and bias gradient in the same grouped launch
            dW = torch.empty((nb, dims[l + 1], dims[l]), device=dev, dtype=torch.float32)
            db = torch.empty((nb, dims[l + 1]), device=dev, dtype=torch.float32)
            tn_reduce(g, hs[l], Np, Kp, slab, S, [(dW.view(-1, dims[l]), 0, 0, dims[l + 1], dims[l], db.view(-1),
                                                   dims[l])], boff=boff)
            for b in range(nb):
                grads[(l * 2) * nb + b] = dW[b]
                grads[(l * 2 + 1) * nb + b] = db[b]
            if l > 0:
                gn = torch.empty((M, Kp), device=dev, dtype=torch.bfloat16)
                _native.ops().bg_nt(g, None, Np, imgTs[l][0], Np, dims[l], None, 0, hs[l] if relu[l - 1] else None,
                                    None, None, None, 0.0, gn, -1, None, None, GEMM_TILE, bid, imgTs[l][0].numel(), 0)
                g = gn
            elif ctx.needs_input_grad[0]:
                dx = torch.empty((M, dims[0]), device=dev, dtype=torch.float32)
                _native.ops().bg_nt(g, None, Np, imgTs[0][0], Np, dims[0], None, 0, None, None, None, dx, 0.0, None,
                                    -1, None, None, GEMM_TILE, bid, imgTs[0][0].numel(), 0)
        ctx.imgTs = None
        return (dx, None, None, None, None, None, *grads)


def branch_mlp(x, seqs, bid, boff):
    """Rows of ``x`` (sorted by branch id ``bid``, int32, values in [0, len(seqs))) through
    their branch's Linear/ReLU chain ``seqs[bid]``; None when the chains do not qualify."""
    chains = [_chain_layers(s) for s in seqs]
    if any(c is None for c in chains) or len({len(c) for c in chains}) != 1:
        return None
    c0 = chains[0]
    dims = [x.shape[1]] + [m.out_features for m, _ in c0]
    relu = [r for _, r in c0]
    for c in chains:
        if [m.out_features for m, _ in c] != dims[1:] or [r for _, r in c] != relu or \
                c[0][0].in_features != dims[0]:
            return None
    if relu[-1] or min(dims[1:]) < 1:
        return None
    nb = len(seqs)
    params = []
    for l in range(len(c0)):
        params += [chains[b][l][0].weight for b in range(nb)]
        params += [chains[b][l][0].bias for b in range(nb)]
    return _BranchMLP.apply(x, bid, boff, dims, relu, nb, *params)
