"""Branch-stacked MLP read-out (``csrc/branch_mlp.hip``): every row of a multi-branch batch
runs the head MLP of its own branch, one launch forward and one backward plus one grouped
weight-gradient launch pair — the captured step's dense multi-branch decode (reference
``hydragnn/models/MACEStack.py:365-400``, ``mace_utils/modules/blocks.py:417-767``)
without evaluating every branch on every row.

A chain is described per branch as steps ``(W, trans, bias, act, scale)``: ``W`` the weight
PARAMETER (``trans`` 0: [O, I] as ``nn.Linear``; 1: [I, O] elements, the e3nn ``x @ W``
layout of an o3.Linear to scalars), ``bias`` a parameter or None, ``act`` an activation
module or None, ``scale`` the layer's input scale.  Weight gradients are written straight
into the step's gradient slots when it provides them (parallel/gradslots.py)."""
import torch
from torch import nn

from .. import _native
from ..parallel import gradslots as _gradslots

_ACT = {nn.ReLU: 1, nn.SiLU: 2, nn.Tanh: 3, nn.Sigmoid: 4}
_PTAB = {}


def act_code(m):
    if m is None:
        return 0
    return _ACT.get(type(m))


def eligible(x, chains):
    """Native path: GPU fp32 rows, <= 8 branches / layers, widths <= 128, known activations,
    identical layer shapes across branches."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2):
        return False
    nb = len(chains)
    if not (1 <= nb <= 8) or not (1 <= len(chains[0]) <= 8):
        return False
    for c in chains:
        if len(c) != len(chains[0]):
            return False
        for (W, tr, b, act, sc), (W0, tr0, b0, act0, sc0) in zip(c, chains[0]):
            if W.shape != W0.shape or tr != tr0 or (b is None) != (b0 is None) or act_code(act) is None or \
                    act_code(act) != act_code(act0) or sc != sc0 or W.dtype != torch.float32 or not W.is_cuda:
                return False
    return True


def _dims(chains, in_dim):
    dims = [in_dim]
    for (W, tr, b, act, sc) in chains[0]:
        O = W.numel() // dims[-1]
        dims.append(O)
    return dims


def _ptab(chains, dev):
    key = tuple((W.data_ptr(), 0 if b is None else b.data_ptr()) for c in chains for (W, _, b, _, _) in c)
    t = _PTAB.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("branch_mlp: pointer table first built inside graph capture")
        L, nb = len(chains[0]), len(chains)
        tab = [[[0] * nb for _ in range(L)] for _ in range(2)]
        for q, c in enumerate(chains):
            for l, (W, _, b, _, _) in enumerate(c):
                tab[0][l][q] = W.data_ptr()
                tab[1][l][q] = 0 if b is None else b.data_ptr()
        t = torch.tensor(tab, dtype=torch.int64, device=dev)
        _PTAB[key] = t
    return t


class _BranchMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rid, acc, meta, *params):
        L, nb, dims, acts, trans, scales, hd, ptab, layout = meta
        res = _native.ops().branch_mlp_fwd(x, rid, ptab, nb, dims, acts, trans, scales, hd,
                                           None if acc is None else acc.contiguous())
        out, hs, zs = res[0], res[1:1 + L], res[1 + L:1 + 2 * L]
        ctx.save_for_backward(x, rid, *hs, *zs)
        ctx.meta = meta
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, g):
        L, nb, dims, acts, trans, scales, hd, ptab, layout = ctx.meta
        t = ctx.saved_tensors
        x, rid, hs, zs = t[0], t[1], t[2:2 + L], t[2 + L:2 + 2 * L]
        ops = _native.ops()
        res = ops.branch_mlp_bwd(g.contiguous(), x, rid, ptab, nb, dims, acts, trans, scales, hd, list(zs))
        dx, slabs = res[0], res[1:]
        params = ctx.params
        sl = _gradslots.slots(list(params))
        grads = list(sl) if sl is not None else [torch.empty_like(p) for p in params]
        dys, xs, dws, dbs = [], [], [], []
        empty = torch.empty(0, device=g.device, dtype=g.dtype)
        for l in range(L):
            I, O = dims[l], dims[l + 1]
            for q in range(nb):
                wi, bi = layout[l][q]
                if trans[l]:  # dW [I, O] = h^T dz (no bias)
                    dys.append(hs[l])
                    xs.append(slabs[l][q])
                    dws.append(grads[wi].view(I, O))
                    dbs.append(empty)
                else:
                    dys.append(slabs[l][q])
                    xs.append(hs[l])
                    dws.append(grads[wi].view(O, I))
                    dbs.append(grads[bi].view(O) if bi is not None else empty)
        ops.linear_wgrad_grouped(dys, xs, dws, dbs, [0] * len(dys))
        if sl is not None:
            _gradslots.provide(list(params))
            pg = [None] * len(params)
        else:
            pg = grads
        return (dx if ctx.needs_input_grad[0] else None, None, g if ctx.needs_input_grad[2] else None, None, *pg)


def branch_mlp(x, rid, chains, hd, acc=None):
    """``out[r] = chain_{rid[r]}(x[r])[:hd]`` (rows with rid < 0: zero), plus ``acc`` [R, hd]
    when given (summed read-outs: no separate add).  ``rid`` int32 [R]."""
    L, nb = len(chains[0]), len(chains)
    if x.stride(1) != 1:  # a column slice of wider rows is read in place (row stride)
        x = x.contiguous()
    dims = _dims(chains, x.shape[1])
    acts = [act_code(s[3]) for s in chains[0]]
    trans = [int(s[1]) for s in chains[0]]
    scales = [float(s[4]) for s in chains[0]]
    params, layout = [], []
    for l in range(L):
        row = []
        for q in range(nb):
            W, _, b, _, _ = chains[q][l]
            wi = len(params)
            params.append(W)
            bi = None
            if b is not None:
                bi = len(params)
                params.append(b)
            row.append((wi, bi))
        layout.append(row)
    meta = (L, nb, dims, acts, trans, scales, int(hd), _ptab(chains, x.device), layout)
    return _BranchMLP.apply(x, rid, acc, meta, *params)
