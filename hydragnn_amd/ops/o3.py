"""Minimal O(3)-equivariant toolkit for MACE (replaces the e3nn pieces the reference
uses: ``o3.SphericalHarmonics``, ``o3.Linear``, ``o3.TensorProduct`` (uvu),
``nn.FullyConnectedNet``, and MACE's ``SymmetricContraction`` / ``U_matrix_real``;
reference ``hydragnn/utils/model/mace_utils/*``, ``irreps_tools.py``).

Conventions (self-consistent; e3nn is not installed here, so bit-parity with e3nn's
basis/sign choices is *unpinned* and equivariance is verified by rotation tests):

* real spherical harmonics, component normalisation (sum_m Y_lm^2 = 2l+1 on the
  unit sphere), m ordered -l..l, built from polynomials in (x, y, z) (smooth,
  differentiable to any order for force training);
* Wigner-D matrices of this basis are fitted numerically (least squares on random
  points), Wigner-3j tensors are the unit-norm invariant of D1 x D2 x D3 (null space
  over two generic rotations, sign fixed by the first significant entry);
* irreps are lists of (mul, l, parity) with parity (-1)^l for everything MACE
  builds here ("natural" parity), flat layout per irrep block = [mul, 2l+1]
  (e3nn layout).
"""
import itertools
import math
import os
from functools import lru_cache

import numpy as np
import torch
from torch import nn


# ----------------------------------------------------------------------------- irreps
class Irreps:
    """Ordered list of (mul, l, p) blocks; flat layout mul-major within a block."""

    def __init__(self, blocks):
        self.blocks = [(int(m), int(l), int(p)) for m, l, p in blocks if m > 0]

    @staticmethod
    def natural(mul, lmax, lmin=0):
        return Irreps([(mul, l, (-1) ** l) for l in range(lmin, lmax + 1)])

    @staticmethod
    def sh(lmax):
        return Irreps([(1, l, (-1) ** l) for l in range(lmax + 1)])

    @property
    def dim(self):
        return sum(m * (2 * l + 1) for m, l, _ in self.blocks)

    def count(self, l, p):
        return sum(m for m, ll, pp in self.blocks if ll == l and pp == p)

    @property
    def num_irreps(self):
        return sum(m for m, _, _ in self.blocks)

    @property
    def lmax(self):
        return max(l for _, l, _ in self.blocks)

    def slices(self):
        out, o = [], 0
        for m, l, p in self.blocks:
            d = m * (2 * l + 1)
            out.append((o, o + d))
            o += d
        return out

    def simplify(self):
        """Merge consecutive blocks with the same (l, p)."""
        out = []
        for m, l, p in self.blocks:
            if out and out[-1][1] == l and out[-1][2] == p:
                out[-1] = (out[-1][0] + m, l, p)
            else:
                out.append((m, l, p))
        return Irreps(out)

    def sort(self):
        """Stable sort by (l, -p-ish) like e3nn (l ascending, even before odd); returns (irreps, perm)."""
        key = [(l, -p, i) for i, (_, l, p) in enumerate(self.blocks)]
        order = sorted(range(len(self.blocks)), key=lambda i: key[i])
        inv = [0] * len(order)
        for new, old in enumerate(order):
            inv[old] = new
        return Irreps([self.blocks[i] for i in order]), inv

    def __iter__(self):
        return iter(self.blocks)

    def __len__(self):
        return len(self.blocks)

    def __add__(self, other):
        return Irreps(self.blocks + other.blocks)

    def __repr__(self):
        return " + ".join(f"{m}x{l}{'e' if p == 1 else 'o'}" for m, l, p in self.blocks)


def create_irreps_string(n, ell):
    """Reference ``irreps_tools.create_irreps_string``: n x l, parity (-1)^l, l = 0..ell."""
    return Irreps.natural(n, ell)


# ----------------------------------------------------------------------------- spherical harmonics
class _SHFused(torch.autograd.Function):
    """One-launch real SH of [E, 3] edge vectors (csrc/sphharm.hip, l <= 4); the backward
    re-evaluates the recurrences in forward-mode dual numbers (one launch).  Double
    backward (force training) takes the composite path via ``composite_mode``."""

    @staticmethod
    def forward(ctx, vec, lmax, normalize, eps):
        from .. import _native

        ctx.save_for_backward(vec)
        ctx.cfg = (lmax, normalize, eps)
        return _native.ops().sh_fwd(vec, lmax, eps, normalize)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        (vec,) = ctx.saved_tensors
        lmax, normalize, eps = ctx.cfg
        return _native.ops().sh_bwd(g, vec, lmax, eps, normalize), None, None, None


def spherical_harmonics(lmax, vec, normalize=True, eps=0.0):
    """Real SH, component normalisation, [..., (lmax+1)^2] with m = -l..l per l."""
    from .pna import fused

    if (vec.is_cuda and vec.dtype == torch.float32 and vec.dim() == 2 and vec.shape[1] == 3 and 0 <= lmax <= 4
            and fused("sh")):
        return _SHFused.apply(vec.contiguous(), int(lmax), bool(normalize), float(eps))
    if normalize:
        vec = vec / (torch.linalg.vector_norm(vec, dim=-1, keepdim=True) + eps)
    x, y, z = vec[..., 0], vec[..., 1], vec[..., 2]
    A = [torch.ones_like(x)]
    B = [torch.zeros_like(x)]
    for m in range(lmax):
        A.append(x * A[m] - y * B[m])
        B.append(x * B[m] + y * A[m])
    # reduced associated Legendre Q[l][m] (P_l^m / (1-z^2)^{m/2}, no Condon-Shortley phase)
    Q = [[None] * (lmax + 1) for _ in range(lmax + 1)]
    for m in range(lmax + 1):
        Q[m][m] = torch.full_like(z, float(np.prod(np.arange(2 * m - 1, 0, -2)) if m > 0 else 1.0))
        if m + 1 <= lmax:
            Q[m + 1][m] = (2 * m + 1) * z * Q[m][m]
        for l in range(m + 2, lmax + 1):
            Q[l][m] = ((2 * l - 1) * z * Q[l - 1][m] - (l + m - 1) * Q[l - 2][m]) / (l - m)
    out = []
    for l in range(lmax + 1):
        for m in range(-l, l + 1):
            am = abs(m)
            c = math.sqrt((2 * l + 1) * math.factorial(l - am) / math.factorial(l + am))
            if m == 0:
                out.append(c * Q[l][0])
            elif m > 0:
                out.append(c * math.sqrt(2.0) * Q[l][am] * A[am])
            else:
                out.append(c * math.sqrt(2.0) * Q[l][am] * B[am])
    return torch.stack(out, -1)


def _rand_rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    return np.array([[a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c)],
                     [2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b)],
                     [2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d]])


def wigner_D(l, R):
    """D^l(R) in the real SH basis above: Y_l(R x) = D Y_l(x)."""
    rng = np.random.default_rng(1234 + l)
    X = rng.normal(size=(max(64, 8 * (2 * l + 1)), 3))
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    Xt = torch.tensor(X, dtype=torch.float64)
    Rt = torch.tensor(R, dtype=torch.float64)
    sl = slice(l * l, (l + 1) * (l + 1))
    Y = spherical_harmonics(l, Xt)[:, sl]
    YR = spherical_harmonics(l, Xt @ Rt.T)[:, sl]
    D = torch.linalg.lstsq(Y, YR).solution.T
    return D.numpy()


@lru_cache(maxsize=None)
def _rotations():
    rng = np.random.default_rng(7)
    return [_rand_rot(rng) for _ in range(2)]


@lru_cache(maxsize=None)
def wigner_3j(l1, l2, l3):
    """Unit-norm invariant tensor [2l1+1, 2l2+1, 2l3+1] (zeros if it does not exist)."""
    if not (abs(l1 - l2) <= l3 <= l1 + l2):
        return torch.zeros(2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1, dtype=torch.float64)
    rows = []
    n = (2 * l1 + 1) * (2 * l2 + 1) * (2 * l3 + 1)
    for R in _rotations():
        K = np.kron(np.kron(wigner_D(l1, R), wigner_D(l2, R)), wigner_D(l3, R))
        rows.append(K - np.eye(n))
    M = np.concatenate(rows, 0)
    _, s, vt = np.linalg.svd(M)
    v = vt[-1]
    assert s[-1] < 1e-6 * max(1.0, s[0]), f"no 3j invariant for ({l1},{l2},{l3})"
    v = v / np.linalg.norm(v)
    i = int(np.argmax(np.abs(v) > 1e-6))
    if v[i] < 0:
        v = -v
    return torch.tensor(v.reshape(2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1), dtype=torch.float64)


# ----------------------------------------------------------------------------- layers
def element_index(elem, num_elements):
    """SegIndex grouping nodes by element (CSR over ``num_elements`` segments with a stable
    sort permutation) so per-element weight tables are *gathered* (``seg.gather``: an
    embedding lookup whose backward is a deterministic segment-sum) instead of multiplying
    a materialised [N, num_elements] one-hot.  Device-only ops (no host sync): capturable."""
    from . import segment as seg

    elem = elem.view(-1)
    if elem.is_cuda and 0 < num_elements <= 1024 and elem.numel() > 0:
        # one launch (csrc/segment.hip elem_csr: stable counting sort in one wave)
        from .. import _native

        from . import devcheck

        idx32, rowptr, perm = _native.ops().elem_csr(elem, int(num_elements),
                                                     devcheck.flag(elem.device, "elem_range"))
        devcheck.debug_check("elem_range", elem.device)
        return seg.SegIndex(idx32, rowptr, perm, num_elements)
    counts = torch.zeros(num_elements, dtype=torch.float32, device=elem.device).index_add_(
        0, elem.long(), torch.ones(elem.shape[0], dtype=torch.float32, device=elem.device))  # exact integer sums
    rowptr = torch.cat([counts.new_zeros(1), counts.cumsum(0)]).to(torch.int32)
    perm = torch.sort(elem, stable=True).indices.to(torch.int32)
    return seg.SegIndex(elem.to(torch.int32), rowptr, perm, num_elements)


def _il_wgrad(x, g, W, jobs, maxd, wscale):
    """Weight gradient of one native o3.Linear; written straight into the weight's slot of
    the step's flat gradient buffer when there is one (then None is returned)."""
    from .. import _native
    from ..parallel import gradslots as _gs

    sl = _gs.slots([W])
    dW = _native.ops().irreps_linear_wgrad(x, g, jobs, wscale, maxd, None if sl is None else sl[0].view(-1))
    if sl is not None:
        _gs.provide([W])
        return None
    return dW


class _IrrepsLinear(torch.autograd.Function):
    """Native o3.Linear (csrc/irreps_linear.hip): forward and input gradient are the same
    column-table kernel in two orientations; the weight gradient is a split node reduction
    (first-order; composite mode runs the torch path).  An optional residual ``res`` is
    added in the forward kernel's epilogue (its gradient is the output gradient itself)."""

    @staticmethod
    def forward(ctx, x, W, fwd, bwd, jobs, maxd, wscale, res=None):
        from .. import _native

        x = x.contiguous()
        ctx.save_for_backward(x, W)
        ctx.tabs = (bwd, jobs, maxd, wscale)
        return _native.ops().irreps_linear(x, W, fwd[0], fwd[1], res)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        x, W = ctx.saved_tensors
        bwd, jobs, maxd, wscale = ctx.tabs
        g = g.contiguous()
        dx = _native.ops().irreps_linear(g, W, bwd[0], bwd[1]) if ctx.needs_input_grad[0] else None
        dW = _il_wgrad(x, g, W, jobs, maxd, wscale) if ctx.needs_input_grad[1] else None
        return dx, dW, None, None, None, None, None, (g if ctx.needs_input_grad[7] else None)


class _IrrepsLinearMulti(torch.autograd.Function):
    """Several native o3.Linears reading the same rows x (the skip / up / down linears of a
    MACE interaction).  Forward: one launch each, as separately.  Backward: the input
    gradient is ONE chain of transposed-orientation launches, each adding the previous
    partial sum in its epilogue, instead of a launch each plus an autograd add per extra
    consumer (csrc/irreps_linear.hip ``res``)."""

    @staticmethod
    def forward(ctx, x, tabs, *Ws):
        from .. import _native

        ctx.set_materialize_grads(False)
        x = x.contiguous()
        ctx.save_for_backward(x, *Ws)
        ctx.tabs = tabs
        return tuple(_native.ops().irreps_linear(x, W, t[0][0], t[0][1]) for W, t in zip(Ws, tabs))

    @staticmethod
    def backward(ctx, *gs):
        from .. import _native

        x, *Ws = ctx.saved_tensors
        ops = _native.ops()
        dx, dWs = None, []
        for W, t, g, need in zip(Ws, ctx.tabs, gs, ctx.needs_input_grad[2:]):
            if g is None:
                dWs.append(None)
                continue
            g = g.contiguous()
            (_fwd, bwd, jobs, maxd, wscale) = t
            if ctx.needs_input_grad[0]:
                dx = ops.irreps_linear(g, W, bwd[0], bwd[1], dx)
            dWs.append(_il_wgrad(x, g, W, jobs, maxd, wscale) if need else None)
        if dx is None and ctx.needs_input_grad[0]:
            dx = torch.zeros_like(x)
        return (dx, None, *dWs)


def linear_multi(lins, x):
    """``[lin(x) for lin in lins]`` for o3.Linears sharing the input rows; native: one fused
    input-gradient chain (``_IrrepsLinearMulti``)."""
    if all(lin.native_ok(x) for lin in lins):
        tabs = []
        for lin in lins:
            fwd, bwd, jobs, maxd = lin._native_tables(x.device)
            tabs.append((fwd, bwd, jobs, maxd, lin.wscale))
        return list(_IrrepsLinearMulti.apply(x, tuple(tabs), *[lin.weight for lin in lins]))
    return [lin(x) for lin in lins]


class O3Linear(nn.Module):
    """e3nn ``o3.Linear`` semantics: per (l, p) channel mixing, N(0,1) weights scaled by
    1/sqrt(fan_in) in the forward ("element" path normalisation), no bias."""

    def __init__(self, irreps_in, irreps_out):
        super().__init__()
        self.irreps_in, self.irreps_out = irreps_in, irreps_out
        self.paths = []
        numel = 0
        for io, (mo, lo, po) in enumerate(irreps_out.blocks):
            ins = [ii for ii, (mi, li, pi) in enumerate(irreps_in.blocks) if li == lo and pi == po]
            fan = sum(irreps_in.blocks[ii][0] for ii in ins)
            for ii in ins:
                mi = irreps_in.blocks[ii][0]
                self.paths.append((ii, io, numel, mi, mo, 1.0 / math.sqrt(fan)))
                numel += mi * mo
        self.weight = nn.Parameter(torch.randn(numel))
        self.sl_in, self.sl_out = irreps_in.slices(), irreps_out.slices()
        # per-element path normalisation: ONE multiply of the whole weight vector per forward
        # and one split into path views (per-path slices would cost a zero-fill + copy each
        # in backward, and a multiply each way per path)
        scale = torch.empty(numel)
        for _, _, off, mi, mo, a in self.paths:
            scale[off:off + mi * mo] = a
        self.register_buffer("wscale", scale, persistent=False)

    def scale_paths(self, f):
        """Multiply every path normalisation by the constant ``f`` (a scale folded in from a
        neighbouring linear op); keeps the torch scale vector and the native tables in step."""
        self.paths = [(ii, io, off, mi, mo, a * f) for ii, io, off, mi, mo, a in self.paths]
        self.wscale.mul_(f)
        self._ntabs = None

    # ---- native (HIP) path: csrc/irreps_linear.hip, one launch forward, two backward
    def _native_tables(self, dev):
        t = getattr(self, "_ntabs", None)
        if t is not None and t[0] == dev:
            return t[1]
        import numpy as np

        def bits(a):
            return int(np.array([a], dtype=np.float32).view(np.int32)[0])

        def orient(transposed):
            # column table over the orientation's OUTPUT columns, paths grouped by output block
            oblocks = self.irreps_in.blocks if transposed else self.irreps_out.blocks
            osl = self.sl_in if transposed else self.sl_out
            prow, cols = [], []
            for ob, (m, l, _) in enumerate(oblocks):
                d = 2 * l + 1
                p0 = len(prow)
                for ii, io, off, mi, mo, a in self.paths:
                    if (ii if transposed else io) != ob:
                        continue
                    if transposed:  # dX: reduce over o, weight index off + i * mo + o
                        prow.append([self.sl_out[io][0], mo, off, 1, mo, d, bits(a)])
                    else:
                        prow.append([self.sl_in[ii][0], mi, off, mo, 1, d, bits(a)])
                p1 = len(prow)
                for u in range(m):
                    for c in range(d):
                        cols.append([p0, p1, u, c])
                assert len(cols) == osl[ob][1]
            return (torch.tensor(prow, dtype=torch.int32, device=dev).reshape(-1, 7),
                    torch.tensor(cols, dtype=torch.int32, device=dev).reshape(-1, 4))

        jobs = []
        for ii, io, off, mi, mo, a in self.paths:
            d = 2 * self.irreps_in.blocks[ii][1] + 1
            for i0 in range(0, mi, 64):
                for o0 in range(0, mo, 64):
                    jobs.append([self.sl_in[ii][0], self.sl_out[io][0], mi, mo, d, off, i0, o0])
        fwd, bwd = orient(False), orient(True)
        tabs = (fwd, bwd, torch.tensor(jobs, dtype=torch.int32, device=dev).reshape(-1, 8),
                max([2 * l + 1 for _, l, _ in self.irreps_in.blocks] + [1]))
        self._ntabs = (dev, tabs)
        return tabs

    def native_ok(self, x):
        from . import pna as _mode

        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] == self.irreps_in.dim
                and 0 < x.shape[1] <= 4096 and self.irreps_out.dim <= 4096 and len(self.paths) > 0
                and self.irreps_in.lmax <= 4
                and _mode.fused("o3linear"))

    def path_weights(self):
        """[mi, mo] normalised weight of every path (views of one scaled vector)."""
        if not self.paths:
            return []
        w = self.weight * self.wscale
        if len(self.paths) == 1:
            _, _, _, mi, mo, _ = self.paths[0]
            return [w.view(mi, mo)]
        return [t.view(mi, mo) for t, (_, _, _, mi, mo, _) in
                zip(torch.split(w, [p[3] * p[4] for p in self.paths]), self.paths)]

    def lookup(self, elem_si):
        """forward(one_hot(elem)) for a single scalar input block (the MACE node embedding):
        one row gather of the weight table per node."""
        from . import segment as seg

        (mi, li, _), = self.irreps_in.blocks
        assert li == 0 and all(l == 0 for _, l, _ in self.irreps_out.blocks), "lookup: scalar irreps only"
        cols = []
        ws = self.path_weights()
        for io in range(len(self.irreps_out.blocks)):
            W = None
            for (ii, o, off, m_in, mo, a), Wp in zip(self.paths, ws):
                if o == io:
                    W = Wp
            cols.append(W if W is not None else self.weight.new_zeros(mi, self.irreps_out.blocks[io][0]))
        table = torch.cat(cols, 1) if len(cols) > 1 else cols[0]
        if table.is_cuda:  # backward = one GEMM over the element one-hot (few, long segments)
            return elem_si.onehot_t(table.dtype).t() @ table
        return seg.gather(table, elem_si)

    def forward(self, x, residual=None):
        """``linear(x) (+ residual)``; natively the residual is added in the kernel epilogue."""
        from .linear import linear

        if self.native_ok(x) and (residual is None or residual.shape == (x.shape[0], self.irreps_out.dim)):
            fwd, bwd, jobs, maxd = self._native_tables(x.device)
            return _IrrepsLinear.apply(x, self.weight, fwd, bwd, jobs, maxd, self.wscale, residual)
        if residual is not None:
            return self.forward(x) + residual
        N = x.shape[0]
        outs = [None] * len(self.irreps_out.blocks)
        # input blocks by ONE split (backward: one concat; per-block slices would zero-fill
        # and copy a full-width gradient each); a scalar-only input may be just its first block
        sizes = [b - a for a, b in self.sl_in]
        if x.shape[1] == sizes[0] and all(p[0] == 0 for p in self.paths):
            xs = [x]
        else:
            xs = torch.split(x, sizes, 1) if len(sizes) > 1 else [x]
        for (ii, io, off, mi, mo, a), W in zip(self.paths, self.path_weights()):
            l = self.irreps_in.blocks[ii][1]
            d = 2 * l + 1
            xi = xs[ii].reshape(N, mi, d)
            if d == 1:  # scalars: a plain [N, mi] x [mi, mo] GEMM
                y = linear(xi.reshape(N, mi), W.t()).view(N, mo, 1)
            else:  # one (N*d, mi) x (mi, mo) GEMM instead of an N-batched tiny bmm
                y = linear(xi.transpose(1, 2).reshape(N * d, mi), W.t()).view(N, d, mo).transpose(1, 2)
            outs[io] = y if outs[io] is None else outs[io] + y
        res = []
        for io, (mo, lo, _) in enumerate(self.irreps_out.blocks):
            o = outs[io]
            if o is None:
                o = x.new_zeros(N, mo, 2 * lo + 1)
            res.append(o.reshape(N, -1))
        return res[0] if len(res) == 1 else torch.cat(res, -1)


def _silu_2mom():
    z = np.linspace(-12, 12, 200001)
    pdf = np.exp(-z * z / 2) / math.sqrt(2 * math.pi)
    s = z / (1 + np.exp(-z))
    return 1.0 / math.sqrt(np.trapezoid(s * s * pdf, z))


_SILU_C = _silu_2mom()


class _TallMM(torch.autograd.Function):
    """x @ W for edge-sized x and a [in, out] weight: the weight gradient x^T dY (K = edges)
    takes the split-K wgrad kernel of csrc/linear.hip, written straight in the weight's
    layout (a library GEMM picks a handful of workgroups for this shape)."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return x @ W

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        from . import linear as _lin

        x, W = ctx.saved_tensors
        dx = g @ W.t() if ctx.needs_input_grad[0] else None
        if ctx.needs_input_grad[1] and _lin._can_defer(W, None):
            # the step's grouped weight-gradient flush: dy^T x with the roles swapped is
            # x^T g = dW in the e3nn [in, out] layout (a full-width "column block" of W)
            _lin._record((x, g.contiguous(), W, None))
            return dx, None
        dW = _native.ops().linear_wgrad(x, g.contiguous(), False)[0] if ctx.needs_input_grad[1] else None
        return dx, dW


class _ScaledSilu(torch.autograd.Function):
    """silu(s x) in one HIP launch each way (csrc/conv_misc.hip scaled_silu_*); first order."""

    @staticmethod
    def forward(ctx, x, s):
        from .. import _native

        ctx.save_for_backward(x)
        ctx.s = s
        return _native.ops().scaled_silu_fwd(x, s)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        (x,) = ctx.saved_tensors
        g = g.contiguous()
        if g.data_ptr() % 16:  # the kernel reads float4s: a sliced view can be misaligned
            g = g.clone()
        return _native.ops().scaled_silu_bwd(g, x, ctx.s), None


def scaled_silu(x, s):
    from . import pna as _mode

    if x.is_cuda and x.dtype == torch.float32 and x.numel() % 4 == 0 and _mode.fused("mlp"):
        xc = x.contiguous()
        if xc.data_ptr() % 16 == 0:  # float4 loads (a contiguous row slice can start mid-vector)
            return _ScaledSilu.apply(xc, float(s))
    return torch.nn.functional.silu(x * s)


def _mm_tall(x, W):
    from . import pna as _mode
    from .linear import MIN_ROWS

    if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[0] >= MIN_ROWS and \
            _mode.fused("linear") and torch.is_grad_enabled():
        return _TallMM.apply(x, W)
    return x @ W


def _seg():
    from . import segment

    return segment


class _FCNFirstSplit(torch.autograd.Function):
    """First layer of the MACE radial FCN over cat[edge_feats, down[src], down[dst]] with the
    concatenation split at node level: y = silu(s (ef W_e + (down W_s)[src] + (down W_d)[dst]))
    where W1 = [W_e; W_s; W_d] ([nef + 2 nd, nd], e3nn x @ W layout).  Forward: one node-level
    batched GEMM, one tall GEMM, one gather + silu pass (csrc/conv_misc.hip edge_gather_silu);
    backward: one pass for dz, two CSR segment sums for dA / dB, ONE grouped weight-gradient
    launch pair for the three row blocks of dW1 (written in place), one batched GEMM for
    d down.  First order (composite mode keeps the torch chain)."""

    @staticmethod
    def forward(ctx, ef, down, W1, s, src_si, dst_si):
        from .. import _native

        nef, nd = ef.shape[1], down.shape[1]
        # [2, N, nd] = down @ W_s, down @ W_d: one batched GEMM over the row blocks of W1[nef:]
        # with a stride-0 batch operand (the [N, 2 nd] side-by-side form needed a transposing
        # copy of the weight every step); edge_gather_silu takes either layout
        ab = torch.bmm(down.unsqueeze(0).expand(2, -1, -1), W1[nef:].view(2, nd, nd))
        et = ef @ W1[:nef]
        ctx.save_for_backward(ef, down, W1, ab, et)
        ctx.cfg = (s, src_si, dst_si)
        return _native.ops().edge_gather_silu_fwd(ab, src_si.index, dst_si.index, et, s)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        ops = _native.ops()
        ef, down, W1, ab, et = ctx.saved_tensors
        s, src_si, dst_si = ctx.cfg
        nef, nd = ef.shape[1], down.shape[1]
        dz = ops.edge_gather_silu_bwd(g, ab, src_si.index, dst_si.index, et, s)
        seg = _seg()
        # CSR sums (they stop at the batch's real edge count when the index carries a limit)
        dA, dB = seg.segment_sum(dz, src_si), seg.segment_sum(dz, dst_si)
        dW1 = None
        if ctx.needs_input_grad[2]:
            dW1 = torch.empty_like(W1)
            e = torch.empty(0, device=g.device, dtype=g.dtype)
            # row blocks of dW1 = x_block^T dy_block (the grouped kernel's dy^T x with roles swapped)
            ops.linear_wgrad_grouped([ef, down, down], [dz, dA, dB], [dW1[:nef], dW1[nef:nef + nd], dW1[nef + nd:]],
                                     [e, e, e], [0, 0, 0])
        ddown = None
        if ctx.needs_input_grad[1]:
            ddown = torch.addmm(dA @ W1[nef:nef + nd].t(), dB, W1[nef + nd:].t())
        def_ = dz @ W1[:nef].t() if ctx.needs_input_grad[0] else None
        return def_, ddown, dW1, None, None, None


class _LinSilu(torch.autograd.Function):
    """One hidden layer of the radial FCN, ``silu(s (x @ W))``, in one HIP launch each way
    (csrc/resmlp.hip lin_act with the e3nn [in, out] weight layout and the pre-scale s); the
    weight gradient x^T dz joins the step's deferred grouped weight-gradient launch."""

    @staticmethod
    def forward(ctx, x, W, s):
        from .. import _native

        y, Z = _native.ops().lin_act_fwd(x, W, None, None, None, s, True)
        ctx.save_for_backward(x, Z, W)
        ctx.s = s
        return y

    @staticmethod
    def backward(ctx, g):
        from .. import _native
        from . import linear as _lin

        x, Z, W = ctx.saved_tensors
        dx, dz, _ = _native.ops().lin_act_bwd(g.contiguous(), Z, W, None, False, ctx.s, True)
        dW = None
        if ctx.needs_input_grad[1]:
            if _lin._can_defer(W, None):
                _lin._record((x, dz, W, None))  # dy^T x with the roles swapped: x^T dz = dW [in, out]
            else:
                dW = x.t() @ dz
        return dx, dW, None


# measured on MI355X (multibranch MACE, same box A/B): 12.61-12.68k with the fused hidden
# layers vs 12.74-12.76k with library GEMM + scaled silu, so the fusion is opt-in
_FCN_LINACT = os.environ.get("HYDRA_FCN_LINACT", "0") == "1"


def _lin_silu_ok(x, W):
    from . import pna as _mode

    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.is_contiguous() and W.shape[0] <= 64
            and W.shape[1] <= 64 and _mode.fused("linear") and _FCN_LINACT)


class FullyConnectedNet(nn.Module):
    """e3nn ``nn.FullyConnectedNet`` with silu: no biases, N(0,1) weights, 1/sqrt(fan_in),
    second-moment-normalised activation between layers."""

    def __init__(self, dims):
        super().__init__()
        self.dims = list(dims)
        self.weights = nn.ParameterList([nn.Parameter(torch.randn(a, b)) for a, b in zip(dims[:-1], dims[1:])])
        # True: the last layer's 1/sqrt(fan_in) is left to the consumer (a linear one folds it
        # into its own constants: the MACE convolution's output linear)
        self.defer_last_scale = False

    def last_scale(self):
        """The constant the last layer's output still needs with ``defer_last_scale``: its
        1/sqrt(fan_in) times the previous activation's normalisation."""
        return (_SILU_C if len(self.weights) > 1 else 1.0) / math.sqrt(self.weights[-1].shape[0])

    def forward_split(self, edge_feats, down, src_si, dst_si):
        """``forward(cat[edge_feats, down[src], down[dst]])`` with the first layer's
        concatenation split at node level (``_FCNFirstSplit``) on the GPU."""
        from . import pna as _mode

        W1 = self.weights[0]
        nd = down.shape[1]
        if (down.is_cuda and down.dtype == torch.float32 and len(self.weights) > 1 and nd % 4 == 0 and
                W1.shape[0] == edge_feats.shape[1] + 2 * nd and _mode.fused("linear")):
            x = _FCNFirstSplit.apply(edge_feats.contiguous(), down.contiguous(), W1, 1.0 / math.sqrt(W1.shape[0]),
                                     src_si, dst_si)
            return self.forward(x, start=1, carry=_SILU_C)
        return self.forward(torch.cat([edge_feats, _seg().gather(down, src_si), _seg().gather(down, dst_si)], -1))

    def forward(self, x, start=0, carry=1.0):
        # the activation normalisation C and the next layer's 1/sqrt(fan_in) are ONE multiply
        # of the pre-activation (same values as scaling after each step)
        n = len(self.weights)
        for i, W in enumerate(self.weights):
            if i < start:
                continue
            s = carry / math.sqrt(W.shape[0])
            if i < n - 1 and _lin_silu_ok(x, W):
                x = _LinSilu.apply(x, W, s)  # GEMM + scaled silu, one launch each way
                carry = _SILU_C
                continue
            x = _mm_tall(x, W)
            if i < n - 1:
                x = scaled_silu(x, s)
                carry = _SILU_C
            elif not self.defer_last_scale:
                x = x * s  # (deferred: s == last_scale(), applied by the consumer)
        return x


def tp_uvu_instructions(irreps1, irreps2, target):
    """Reference ``tp_out_irreps_with_instructions``: all (l1 x l2 -> l3) with l3 (and
    parity) in target; output blocks sorted; instructions (i1, i2, i_out)."""
    out, ins = [], []
    tgt = {(l, p) for _, l, p in target.blocks}
    for i, (m1, l1, p1) in enumerate(irreps1.blocks):
        for j, (_, l2, p2) in enumerate(irreps2.blocks):
            for l3 in range(abs(l1 - l2), l1 + l2 + 1):
                p3 = p1 * p2
                if (l3, p3) in tgt:
                    ins.append((i, j, len(out)))
                    out.append((m1, l3, p3))
    irr = Irreps(out)
    srt, perm = irr.sort()
    ins = sorted([(a, b, perm[k]) for a, b, k in ins], key=lambda t: t[2])
    return srt, ins


class _TPUVU(torch.autograd.Function):
    """HIP uvu tensor product (first-order autograd; composite mode uses the einsum path)."""

    @staticmethod
    def forward(ctx, x1, x2, w, ins, cg, out_dim):
        from .. import _native

        ctx.save_for_backward(x1, x2, w, ins, cg)
        return _native.ops().tp_uvu_fwd(x1, x2, w, ins, cg, out_dim)

    @staticmethod
    def backward(ctx, go):
        from .. import _native

        x1, x2, w, ins, cg = ctx.saved_tensors
        g1, g2, gw = _native.ops().tp_uvu_bwd(go, x1, x2, w, ins, cg)
        return g1, g2, gw, None, None, None


class _TPConv(torch.autograd.Function):
    """Fused MACE convolution: out[n] = sum_{e: dst_e = n} TP(x1[src_e], Y_e, w_e)
    (csrc/equivariant.hip tp_conv_*; first-order autograd)."""

    @staticmethod
    def forward(ctx, x1, y, w, ins, cg, out_dim, src_si, dst_si):
        from .. import _native

        ctx.save_for_backward(x1, y, w, ins, cg)
        ctx.si = (src_si, dst_si)
        return _native.ops().tp_conv_fwd(x1, y, w, ins, cg, src_si.index, dst_si.rowptr, out_dim)

    @staticmethod
    def backward(ctx, go):
        from .. import _native

        x1, y, w, ins, cg = ctx.saved_tensors
        src_si, dst_si = ctx.si
        need_gy = ctx.needs_input_grad[1]  # edge attributes: no gradient in energy training
        g1, gy, gw = _native.ops().tp_conv_bwd(go, x1, y, w, ins, cg, src_si.index, dst_si.index, src_si.rowptr,
                                               src_si.perm, need_gy)
        return g1, (gy if need_gy else None), gw, None, None, None, None, None


class TensorProductUVU(nn.Module):
    """Channel-wise ("uvu") tensor product with per-edge external weights:
    out[e, u, m3] (block k) = sqrt(2 l3 + 1) sum_v w[e, k, u, v] sum_{m1 m2} C[m1 m2 m3] x1[e, u, m1] x2[e, v, m2]."""

    def __init__(self, irreps1, irreps2, irreps_out, instructions):
        super().__init__()
        self.irreps1, self.irreps2, self.irreps_out = irreps1, irreps2, irreps_out
        self.ins = instructions
        self.sl1, self.sl2 = irreps1.slices(), irreps2.slices()
        self.weight_numel = 0
        self.woff = []
        for i, j, k in instructions:
            m1, l1, _ = irreps1.blocks[i]
            m2, l2, _ = irreps2.blocks[j]
            l3 = irreps_out.blocks[k][1]
            self.woff.append((self.weight_numel, m1, m2))
            self.weight_numel += m1 * m2
            self.register_buffer(f"cg_{l1}_{l2}_{l3}", wigner_3j(l1, l2, l3).float() * math.sqrt(2 * l3 + 1),
                                 persistent=False)

        # native (HIP) path tables: the second operand carries one channel per l (spherical
        # harmonics), which is the case the fused kernel implements (csrc/equivariant.hip)
        # (the fused kernels compile every (l1, l2, l3) body with l <= 3)
        self.native_ok = all(m2 == 1 for _, _, m2 in self.woff) and max(irreps1.lmax, irreps2.lmax, irreps_out.lmax) <= 3
        rows, cgs, cgoff = [], [], 0
        so = irreps_out.slices()
        for (i, j, k), (off, m1, m2) in zip(instructions, self.woff):
            l1, l2, l3 = irreps1.blocks[i][1], irreps2.blocks[j][1], irreps_out.blocks[k][1]
            rows.append([l1, l2, l3, m1, self.sl1[i][0], self.sl2[j][0], off, so[k][0], cgoff])
            c = getattr(self, f"cg_{l1}_{l2}_{l3}").reshape(-1)
            cgs.append(c)
            cgoff += c.numel()
        self.register_buffer("_ins", torch.tensor(rows, dtype=torch.int32), persistent=False)
        self.register_buffer("_cg", torch.cat(cgs) if cgs else torch.zeros(0), persistent=False)

    def forward(self, x1, x2, w):
        from . import pna as _mode

        if x1.is_cuda and self.native_ok and x1.dtype == torch.float32 and _mode.fused("tp"):
            return _TPUVU.apply(x1, x2, w, self._ins, self._cg, self.irreps_out.dim)
        return self.forward_reference(x1, x2, w)

    def conv(self, x1_nodes, x2, w, src_si, dst_si):
        """sum over each destination's edges of TP(x1_nodes[src], x2, w) (MACE message +
        aggregation): one fused kernel on the GPU, gather / TP / segment-sum otherwise."""
        from . import pna as _mode
        from . import segment as seg

        if x1_nodes.is_cuda and self.native_ok and x1_nodes.dtype == torch.float32 and _mode.fused("tpconv") and \
                dst_si.perm is None:
            return _TPConv.apply(x1_nodes.contiguous(), x2.contiguous(), w.contiguous(), self._ins, self._cg,
                                 self.irreps_out.dim, src_si, dst_si)
        return seg.segment_sum(self(seg.gather(x1_nodes, src_si), x2, w), dst_si)

    def forward_reference(self, x1, x2, w):
        E = x1.shape[0]
        outs = [None] * len(self.irreps_out.blocks)
        for (i, j, k), (off, m1, m2) in zip(self.ins, self.woff):
            l1, l2, l3 = self.irreps1.blocks[i][1], self.irreps2.blocks[j][1], self.irreps_out.blocks[k][1]
            a = x1[:, self.sl1[i][0]:self.sl1[i][1]].reshape(E, m1, 2 * l1 + 1)
            b = x2[:, self.sl2[j][0]:self.sl2[j][1]].reshape(E, m2, 2 * l2 + 1)
            C = getattr(self, f"cg_{l1}_{l2}_{l3}")
            ww = w[:, off:off + m1 * m2].view(E, m1, m2)
            bv = torch.einsum("evj,euv->euj", b, ww) if m2 > 1 else b * ww  # [E, u, 2l2+1]
            y = torch.einsum("eui,euj,ijk->euk", a, bv, C)
            outs[k] = y.reshape(E, -1)
        return torch.cat(outs, -1)


# ----------------------------------------------------------------------------- symmetric contraction
@lru_cache(maxsize=None)
def u_matrix(lmax_in, L, nu):
    """Basis of symmetric equivariant maps Sym^nu(V) -> V_L, V = (+)_{l<=lmax_in} V_l with
    parity (-1)^l, output parity (-1)^L.  Returns [2L+1, d, ..., d (nu), K] (float64)."""
    d = (lmax_in + 1) ** 2
    # coupling paths: (l, parity, tensor [2l+1, d^k])
    paths = []
    for l in range(lmax_in + 1):
        T = torch.zeros(2 * l + 1, d, dtype=torch.float64)
        T[:, l * l:(l + 1) * (l + 1)] = torch.eye(2 * l + 1, dtype=torch.float64)
        paths.append((l, (-1) ** l, T))
    for step in range(nu - 1):
        remaining = nu - 2 - step  # factors still to couple after this one
        new = []
        for lp, pp, T in paths:
            for l in range(lmax_in + 1):
                for lo in range(abs(lp - l), lp + l + 1):
                    if abs(lo - L) > remaining * lmax_in:  # can no longer reach L
                        continue
                    C = wigner_3j(lp, l, lo) * math.sqrt(2 * lo + 1)
                    E = torch.zeros(2 * l + 1, d, dtype=torch.float64)
                    E[:, l * l:(l + 1) * (l + 1)] = torch.eye(2 * l + 1, dtype=torch.float64)
                    # T'[mo, prev..., i] = sum_{mp, m} C[mp, m, mo] T[mp, prev] E[m, i]
                    Tn = torch.einsum("abo,ap,bi->opi", C, T, E).reshape(2 * lo + 1, -1)
                    new.append((lo, pp * (-1) ** l, Tn))
        paths = new
    sel = [T for l, p, T in paths if l == L and p == (-1) ** L]
    if not sel:
        return torch.zeros((2 * L + 1,) + (d,) * nu + (0,), dtype=torch.float64)
    X = torch.stack([T.reshape((2 * L + 1,) + (d,) * nu) for T in sel], 0)  # [P, M, d..]
    perms = list(itertools.permutations(range(nu)))
    Xs = sum(X.permute(0, 1, *[2 + q for q in pm]) for pm in perms) / len(perms)
    Mx = Xs.reshape(Xs.shape[0], -1)
    U, s, Vt = torch.linalg.svd(Mx, full_matrices=False)
    keep = s > 1e-8 * max(1.0, float(s[0]) if s.numel() else 1.0)
    B = Vt[keep]  # [K, M*d^nu] orthonormal rows
    K = B.shape[0]
    return B.T.reshape((2 * L + 1,) + (d,) * nu + (K,))


class Contraction(nn.Module):
    def __init__(self, lmax_in, L, correlation, num_features, num_elements):
        super().__init__()
        self.L, self.correlation = L, correlation
        self.d = (lmax_in + 1) ** 2
        self.weights = nn.ParameterList()
        for nu in range(1, correlation + 1):
            U = u_matrix(lmax_in, L, nu).float()
            self.register_buffer(f"U_{nu}", U, persistent=False)
            K = U.shape[-1]
            self.weights.append(nn.Parameter(torch.randn(num_elements, K, num_features) / max(K, 1)))

    def forward(self, x, elem):
        """x [N, H, d]; elem [N] element index -> [N, H, 2L+1]."""
        N, H, d = x.shape
        out = None
        for nu in range(self.correlation, 0, -1):
            U = getattr(self, f"U_{nu}")
            K = U.shape[-1]
            P = U.reshape(-1, K)  # [M d^nu, K]
            if K > 0:
                # per-element weights: one-hot(elem) @ W as a GEMM (its backward is a GEMM too,
                # not a sort-based index_put), then one (N*H, K) x (K, M d^nu) GEMM
                Wt = self.weights[nu - 1]
                if not torch.is_tensor(elem):  # element SegIndex: per-node row gather of the table
                    from . import segment as seg

                    W = seg.gather(Wt.reshape(Wt.shape[0], -1), elem).view(N, K, H)
                elif elem.dim() == 2:  # one-hot / soft assignment [N, num_elements]
                    W = (elem @ Wt.reshape(Wt.shape[0], -1)).view(N, K, H)
                else:
                    W = Wt[elem]
                W = W.transpose(1, 2).reshape(N * H, K)
                c = (W @ P.t()).view(N, H, -1)
            else:
                c = x.new_zeros(N, H, P.shape[0])
            out = c if out is None else out + c
            # contract the last input index with x: broadcast multiply + reduce (no tiny bmm)
            out = (out.view(N, H, -1, d) * x.unsqueeze(2)).sum(-1)
        return out  # [N, H, 2L+1]


class _SymConNative(torch.autograd.Function):
    """csrc/symcon.hip: the whole product basis (every L, every nu) in one launch each
    way; per-element weight gradients by a CSR segment sum over the element index."""

    @staticmethod
    def forward(ctx, x, elem_si, ents, grps, out_cols, shapes, *weights):
        from .. import _native

        ne = weights[0].shape[0]
        Wcat = torch.cat([w for w in weights], 1).contiguous()  # [ne, Ktot, H]
        ctx.save_for_backward(x, Wcat, ents, grps)
        ctx.elem_si, ctx.shapes, ctx.ne = elem_si, shapes, ne
        ctx.params = weights
        return _native.ops().symcon_fwd(x.contiguous(), elem_si.index, Wcat, ents, grps, out_cols)

    @staticmethod
    def backward(ctx, gout):
        from .. import _native
        from . import segment as seg

        x, Wcat, ents, grps = ctx.saved_tensors
        dx, dWn = _native.ops().symcon_bwd(gout, x, ctx.elem_si.index, Wcat, ents, grps)
        N, Ktot, H = dWn.shape
        # per-element reduction over nodes: few, long segments (every node of an element,
        # padding nodes included) -> one GEMM with the element one-hot (a CSR walk of the
        # longest segment was 80+ us per layer on MI355X)
        oh = ctx.elem_si.onehot_t(dWn.dtype)
        from ..parallel import gradslots as _gs

        sl = _gs.slots(list(ctx.params))
        if sl is not None:
            # every weight's gradient GEMM writes its own slot of the step's flat buffer (the
            # column blocks of one GEMM were strided views: a contiguous copy each, then the pack)
            o = 0
            for K, w in zip(ctx.shapes, sl):
                torch.mm(oh, dWn[:, o:o + K].reshape(N, K * H), out=w.view(ctx.ne, K * H))
                o += K
            _gs.provide(list(ctx.params))
            return (dx, None, None, None, None, None, *([None] * len(ctx.shapes)))
        dW = (oh @ dWn.view(N, Ktot * H)).view(ctx.ne, Ktot, H)
        grads, o = [], 0
        for K in ctx.shapes:
            grads.append(dW[:, o:o + K])
            o += K
        return (dx, None, None, None, None, None, *grads)


class SymmetricContraction(nn.Module):
    """MACE product basis: per output irrep L of ``irreps_out``, sum_{nu<=correlation}
    sum_k W_{nu,k}(element) U_{nu,k} . x^{(x) nu}, channel-wise."""

    def __init__(self, lmax_in, irreps_out, correlation, num_features, num_elements):
        super().__init__()
        self.irreps_out = irreps_out
        self.correlation = correlation
        self.contractions = nn.ModuleList([Contraction(lmax_in, l, correlation, num_features, num_elements)
                                           for _, l, _ in irreps_out.blocks])
        self._tables = None

    def _native_tables(self, H, dev):
        """Entry table of the non-zero U coefficients (i0, i1, i2, weight row, value bits)
        grouped by output column (base, 2L+1, M, first, end), for csrc/symcon.hip."""
        if self._tables is not None and self._tables[0].device == dev and self._tables[3] == H:
            return self._tables
        ents, grps = [], []
        koff, base = 0, 0
        for c in self.contractions:
            L = c.L
            ks = []
            for nu in range(1, c.correlation + 1):
                ks.append(koff)
                koff += getattr(c, f"U_{nu}").shape[-1]
            for M in range(2 * L + 1):
                e0 = len(ents)
                for nu in range(1, c.correlation + 1):
                    U = getattr(c, f"U_{nu}")[M]  # [d]*nu + [K]
                    nz = torch.nonzero(U.abs() > 1e-12)
                    for row in nz.tolist():
                        idx, k = row[:-1], row[-1]
                        v = float(U[tuple(row)])
                        i = idx + [-1] * (3 - len(idx))
                        ents.append([i[0], i[1], i[2], ks[nu - 1] + k, v])
                grps.append([base, 2 * L + 1, M, e0, len(ents)])
            base += H * (2 * L + 1)
        e = torch.tensor([r[:4] for r in ents], dtype=torch.int32).view(-1, 4)
        vals = torch.tensor([r[4] for r in ents], dtype=torch.float32).view(-1, 1).view(torch.int32)
        self._tables = (torch.cat([e, vals], 1).contiguous().to(dev), torch.tensor(grps, dtype=torch.int32).to(dev),
                        base, H)
        return self._tables

    def native_ok(self, x, elem):
        from . import pna as _mode

        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and x.shape[2] <= 16 and
                self.correlation <= 3 and _mode.fused("symcon") and not torch.is_tensor(elem))

    def forward(self, x, elem):
        """``elem``: an element SegIndex (``element_index``), element indices [N], or a
        one-hot / soft assignment [N, num_elements]."""
        N = x.shape[0]
        if torch.is_tensor(elem) and elem.dim() == 1:
            elem = element_index(elem, self.contractions[0].weights[0].shape[0])
        if self.native_ok(x, elem):
            ents, grps, cols, _ = self._native_tables(x.shape[1], x.device)
            weights = [w for c in self.contractions for w in c.weights]
            return _SymConNative.apply(x, elem, ents, grps, cols, [w.shape[1] for w in weights], *weights)
        return torch.cat([c(x, elem).reshape(N, -1) for c in self.contractions], -1)
