"""Row programs: node-level compute chains compiled into ONE interpreter launch per mode,
with forward, first-order and second-order derivative programs generated here.

Force training (forces = -dE/dpos, then the loss gradient w.r.t. the parameters; reference
``Base.energy_force_loss``, ``Base.py:582-636``) differentiates every op twice.  Op-by-op
(torch composite) that is ~7 launches per Linear and ~4 per pointwise op; a PAINN layer
alone is ~400 launches per training step.  A *row program* is a straight-line chain of
row-local ops (linears, activations, products, norms over the 3 Cartesian components,
masks) over node rows; this module

* records the forward chain (``Prog`` builder),
* builds the forward-mode **dual** program (``dual``): primal values + tangents,
* builds the reverse-mode **adjoint** program of any program (``reverse``), with dead-
  adjoint elimination and weight-gradient records,

so that for a chain ``y = f(x; W)``:

* ``VJP``  = reverse(f) seeded with ``ybar``                -> ``xbar``, ``Wbar``
* ``VVJP`` = reverse(dual(f)) seeded with ``adj(y') = g``    -> ``J h`` (= dual tangent out),
  ``d/dx [g . J(x) h]``, ``d/dW [g . J h]`` — the backward of the VJP (double backward).

Programs run on the device in ``csrc/rowprog.hip`` (one interpreter kernel: 16-row
blocks, MFMA fp32 linears, weight gradients through the grouped MFMA wgrad), and on the
CPU in ``run_torch`` (the fp64-checkable twin of the kernel).

Value layout: every value is [N, nc * w] fp32 (nc = 1 scalar features, nc = 3 the
Cartesian components of a vector feature, component-major: column c * w + f, i.e. the
memory layout of a contiguous [N, 3, w] tensor).
"""
import torch

# elementwise opcodes (device values in csrc/rowprog.hip)
E_COPY, E_MUL, E_MUL3, E_ACT, E_DOT3, E_NORM3, E_SINV, E_MASK, E_ZERO = range(9)
ACTS = {"identity": 0, "relu": 1, "silu": 2, "tanh": 3, "sigmoid": 4}


class Val:
    """A value: a root slot or a column slice (c0, w) of a root (per component)."""

    __slots__ = ("id", "w", "nc", "root", "c0", "name")
    _n = 0

    def __init__(self, w, nc=1, root=None, c0=0, name=""):
        Val._n += 1
        self.id = Val._n
        self.w, self.nc, self.root, self.c0, self.name = int(w), int(nc), root, int(c0), name

    @property
    def base(self):
        return self.root if self.root is not None else self

    def slice(self, c0, w):
        b = self.base
        return Val(w, self.nc, b, self.c0 + c0, name=f"{b.name}[{self.c0 + c0}:{self.c0 + c0 + w}]")

    @property
    def full(self):
        return self.root is None

    def __repr__(self):
        return f"<{self.name or self.id}:{self.nc}x{self.w}>"


class Weight:
    """A linear weight W [O, K] (torch parameter index ``pid``) and optional bias."""

    __slots__ = ("pid", "O", "K", "bid")

    def __init__(self, pid, O, K, bid=None):
        self.pid, self.O, self.K, self.bid = pid, O, K, bid


class Prog:
    """Straight-line row program.  Instructions:

    ('lin', y, [(x, W, k0)], trans, bias_pid|None, acc)
        trans=True:  y[o] (+)= sum_i sum_k x_i[k] W_i[o, k0_i + k]  (+ b[o])  (x W^T)
        trans=False: y[k] (+)= sum_i sum_o x_i[o] W_i[o, k0_i + k]           (x W)
      per Cartesian component when the values are vectors (nc = 3; no bias then).
    ('ew', op, y, a, b, c, arg, coef, acc)
        y (+)= coef * op(a, b, c); scalar operands broadcast over components.
    """

    def __init__(self):
        self.ins = []
        self.inputs = []
        self.outputs = []

    # -- builder
    def input(self, w, nc=1, name=""):
        v = Val(w, nc, name=name)
        self.inputs.append(v)
        return v

    def lin(self, xs, W, bias=True, name="", trans=True, y=None, acc=False):
        """xs: list of (x, k0) pairs sharing the weight ``W`` (column blocks of one W)."""
        nc = xs[0][0].nc
        O = W.O if trans else xs[0][0].w
        if y is None:
            y = Val(O if trans else W.K, nc, name=name)
        self.ins.append(("lin", y, [(x, W, k0) for x, k0 in xs], trans,
                         W.bid if (bias and trans and W.bid is not None) else None, acc))
        return y

    def ew(self, op, a, b=None, c=None, arg=0, coef=1.0, nc=None, w=None, name="", y=None, acc=False):
        if y is None:
            if nc is None:
                nc = 1 if op in (E_DOT3, E_NORM3) else max(t.nc for t in (a, b, c) if t is not None)
            y = Val(w or a.w, nc, name=name)
        self.ins.append(("ew", op, y, a, b, c, arg, float(coef), acc))
        return y

    def act(self, x, kind, name=""):
        return self.ew(E_ACT, x, arg=ACTS[kind] * 4 + 0, name=name)

    def mul(self, a, b, name=""):
        return self.ew(E_MUL, a, b, name=name)

    def add(self, *terms, name=""):
        y = self.ew(E_COPY, terms[0], nc=max(t.nc for t in terms), name=name)
        for t in terms[1:]:
            self.ew(E_COPY, t, y=y, acc=True)
        return y

    def dot3(self, a, b, name=""):
        return self.ew(E_DOT3, a, b, name=name)

    def norm3(self, a, name=""):
        return self.ew(E_NORM3, a, name=name)

    def mask(self, x, name=""):
        return self.ew(E_MASK, x, name=name)


def _act_code(arg):
    return arg // 4, arg % 4  # (kind, derivative order)


# ----------------------------------------------------------------------------- dual
def dual(prog, tin):
    """Forward-mode dual of ``prog``: returns (program, tangent map) where the program
    computes every primal value and the tangent of every value reachable from the seeded
    inputs ``tin`` ({input Val: tangent Val}).  Weights carry no tangent."""
    out = Prog()
    out.inputs = list(prog.inputs) + list(tin.values())
    tan = {}  # base Val id -> tangent root Val
    tinit = set()  # base ids whose tangent root has been written

    def t_of(v):
        tb = tan.get(v.base.id)
        if tb is None or v.base.id not in tinit:
            return None
        return tb if v.full else tb.slice(v.c0, v.w)

    def t_target(y):
        """(tangent Val of y, accumulate flag of the first write into it)."""
        b = y.base
        if b.id not in tan:
            tan[b.id] = Val(b.w, b.nc, name=f"d({b.name})")
        tb = tan[b.id]
        ty = tb if y.full else tb.slice(y.c0, y.w)
        if b.id in tinit:
            return ty, True
        tinit.add(b.id)
        if not y.full:
            out.ins.append(("ew", E_ZERO, tb, None, None, None, 0, 1.0, False))
            return ty, True
        return ty, False

    for k, v in tin.items():
        tan[k.base.id] = v
        tinit.add(k.base.id)
    for ins in prog.ins:
        out.ins.append(ins)
        if ins[0] == "lin":
            _, y, xs, trans, bias, acc = ins
            txs = [(t_of(x), W, k0) for x, W, k0 in xs if t_of(x) is not None]
            if not txs:
                continue
            ty, a0 = t_target(y)
            out.ins.append(("lin", ty, txs, trans, None, a0))
            continue
        _, op, y, a, b, c, arg, coef, acc = ins
        if op == E_ZERO:
            continue
        ta, tb, tc = (t_of(t) if t is not None else None for t in (a, b, c))
        if ta is None and tb is None and tc is None:
            continue
        terms = []  # (op, a, b, c, arg, coef) tangent contributions
        if op == E_COPY:
            terms.append((E_COPY, ta, None, None, 0, coef))
        elif op in (E_MUL, E_MUL3):
            fs = [a, b] + ([c] if op == E_MUL3 else [])
            ts = [ta, tb] + ([tc] if op == E_MUL3 else [])
            for i, t in enumerate(ts):
                if t is not None:
                    f2 = list(fs)
                    f2[i] = t
                    terms.append((op, f2[0], f2[1], f2[2] if op == E_MUL3 else None, 0, coef))
        elif op == E_ACT:
            kind, order = _act_code(arg)
            assert order <= 1 and c is None, "dual of a second derivative / 3-factor activation is not needed"
            # y = coef s^(o)(a) [* b]  ->  y' = coef s^(o+1)(a) a' [* b] + coef s^(o)(a) b'
            if ta is not None:
                terms.append((E_ACT, a, ta, b, kind * 4 + order + 1, coef))
            if tb is not None:
                terms.append((E_ACT, a, tb, None, kind * 4 + order, coef))
        elif op == E_DOT3:
            assert tc is None
            if ta is not None:
                terms.append((E_DOT3, ta, b, c, 0, coef))
            if tb is not None:
                terms.append((E_DOT3, a, tb, c, 0, coef))
        elif op == E_NORM3:
            # n = |a|: n' = (a . a') / n  (0 where n = 0)
            r = _emit(out, E_SINV, y, nc=1)
            terms.append((E_DOT3, a, ta, r, 0, coef))
        elif op == E_SINV:
            # r = 1/a: r' = -r^2 a'
            terms.append((E_MUL3, y, y, ta, 0, -coef))
        elif op == E_MASK:
            terms.append((E_MASK, ta, None, None, 0, coef))
        else:
            raise NotImplementedError(op)
        ty, a0 = t_target(y)
        for i, (o2, a2, b2, c2, arg2, cf) in enumerate(terms):
            out.ins.append(("ew", o2, ty, a2, b2, c2, arg2, cf, a0 if i == 0 else True))
    out.outputs = list(prog.outputs)
    return out, {k: tan[k] for k in tan if k in tinit}


def _emit(prog, op, a, b=None, c=None, arg=0, coef=1.0, nc=None):
    return prog.ew(op, a, b, c, arg=arg, coef=coef, nc=nc)


# ----------------------------------------------------------------------------- reverse
def _deps(prog):
    """Forward dependency sets: base id -> set of input base ids / ('W', pid) it depends on."""
    dep = {}
    for v in prog.inputs:
        dep[v.base.id] = {v.base.id}
    for ins in prog.ins:
        if ins[0] == "lin":
            _, y, xs, trans, bias, acc = ins
            s = set(dep.get(y.base.id, set()))
            for x, W, k0 in xs:
                s |= dep.get(x.base.id, set())
                s.add(("W", W.pid))
            if bias is not None:
                s.add(("W", bias))
        else:
            _, op, y, a, b, c, arg, coef, acc = ins
            s = set(dep.get(y.base.id, set()))
            for t in (a, b, c):
                if t is not None:
                    s |= dep.get(t.base.id, set())
        dep[y.base.id] = s
    return dep


def reverse(prog, seeds, wanted, want_weights=True):
    """Reverse-mode adjoint program of ``prog``.

    seeds: {Val: adjoint Val} on program values (outputs); wanted: input Vals whose
    adjoints are returned.  Returns (adjoint program, {wanted input: adjoint Val or None},
    wgrads) with wgrads a list of ('w', pid, k0, G, X, trans) / ('b', pid, G) records:
    W[:, k0:k0+K] += G^T X (trans) or W[:, k0:k0+K] += X^T G (not trans), b += sum G."""
    dep = _deps(prog)
    target = {v.base.id for v in wanted}
    useful_cache = {}

    def useful(v):
        i = v.base.id
        r = useful_cache.get(i)
        if r is None:
            d = dep.get(i, set())
            r = bool(d & target) or (want_weights and any(isinstance(t, tuple) for t in d))
            useful_cache[i] = r
        return r

    out = Prog()
    adj = {}  # base id -> adjoint root Val
    init = set()  # base ids whose adjoint has been written
    wg = []

    read = set()
    for ins in prog.ins:
        for t in _reads(ins):
            read.add(t.base.id)
    out.inputs = list(seeds.values())
    for v, a in seeds.items():
        assert v.full
        if v.base.id in read:
            # other instructions will accumulate into this adjoint: never write the seed tensor
            c = Val(v.w, v.nc, name=f"adj({v.name})")
            out.ins.append(("ew", E_COPY, c, a, None, None, 0, 1.0, False))
            a = c
        adj[v.base.id] = a
        init.add(v.base.id)

    def a_of(v):
        r = adj.get(v.base.id)
        if r is None:
            return None
        return r if v.full else r.slice(v.c0, v.w)

    def contrib(v, op, a, b=None, c=None, arg=0, coef=1.0):
        """adj(v) += coef * op(a, b, c)."""
        if not useful(v):
            return
        bid = v.base.id
        if bid not in adj:
            bv = v.base
            adj[bid] = Val(bv.w, bv.nc, name=f"adj({bv.name})")
        first = bid not in init
        if first and not v.full:
            out.ins.append(("ew", E_ZERO, adj[bid], None, None, None, 0, 1.0, False))
            first = False
        init.add(bid)
        out.ins.append(("ew", op, a_of(v), a, b, c, arg, float(coef), not first))

    def contrib_lin(x, W, k0, g, trans):
        if not useful(x):
            return
        bid = x.base.id
        if bid not in adj:
            bv = x.base
            adj[bid] = Val(bv.w, bv.nc, name=f"adj({bv.name})")
        first = bid not in init
        if first and not x.full:
            out.ins.append(("ew", E_ZERO, adj[bid], None, None, None, 0, 1.0, False))
            first = False
        init.add(bid)
        out.ins.append(("lin", a_of(x), [(g, W, k0)], not trans, None, not first))

    for ins in reversed(prog.ins):
        if ins[0] == "lin":
            _, y, xs, trans, bias, acc = ins
            g = a_of(y)
            if g is None or y.base.id not in init:
                continue
            for x, W, k0 in xs:
                contrib_lin(x, W, k0, g, trans)
                if want_weights:
                    wg.append(("w", W.pid, k0, g, x, trans))
            if bias is not None and want_weights:
                wg.append(("b", bias, g))
            if not acc and y.full:
                # y was (re)defined here: earlier writers of y are not its producers
                pass
            continue
        _, op, y, a, b, c, arg, coef, acc = ins
        g = a_of(y)
        if g is None or y.base.id not in init:
            continue
        if op == E_ZERO:
            continue
        if op == E_COPY:
            contrib(a, E_COPY, g, coef=coef) if a.nc == y.nc else contrib(a, E_DOT3, g, _ones(out, y), coef=coef)
        elif op == E_MUL:
            _mul_adj(out, contrib, y, g, a, b, None, coef)
        elif op == E_MUL3:
            _mul_adj(out, contrib, y, g, a, b, c, coef)
        elif op == E_ACT:
            kind, order = _act_code(arg)
            # y = coef s^(o)(a) [* b [* c]]
            # a_bar += coef s^(o+1)(a) g [* b [* c]]    (summed over components if a is scalar)
            if b is None:
                contrib(a, E_ACT, a, g, None, kind * 4 + order + 1, coef)
            else:
                # y = coef s^(o)(a) * b (* c): treat as product of three factors
                _act_prod_adj(out, contrib, y, g, a, b, c, kind, order, coef)
        elif op == E_DOT3:
            # y = coef sum_c a_c b_c [* c_s]
            if c is None:
                contrib(a, E_MUL, g, b, coef=coef)
                contrib(b, E_MUL, g, a, coef=coef)
            else:
                contrib(a, E_MUL3, g, b, c, coef=coef)
                contrib(b, E_MUL3, g, a, c, coef=coef)
                contrib(c, E_DOT3, a, b, g, coef=coef)
        elif op == E_NORM3:
            # n = |a|: a_bar += g a / n
            r = _emit(out, E_SINV, y, nc=1)
            contrib(a, E_MUL3, g, a, r, coef=coef)
        elif op == E_SINV:
            contrib(a, E_MUL3, g, y, y, coef=-coef)
        elif op == E_MASK:
            contrib(a, E_MASK, g, coef=coef)
        else:
            raise NotImplementedError(op)
    res = {}
    for v in wanted:
        r = adj.get(v.base.id)
        res[v] = (r if v.full else r.slice(v.c0, v.w)) if r is not None and v.base.id in init else None
    return out, res, wg


def _ones(prog, like):
    raise NotImplementedError("broadcast COPY adjoint")


def _mul_adj(out, contrib, y, g, a, b, c, coef):
    """y = coef * a * b [* c] (scalar factors broadcast over components): every factor f
    gets coef * g * (other factors), summed over the components when f is a scalar
    factor of a vector product."""
    fs = [t for t in (a, b, c) if t is not None]
    for i, f in enumerate(fs):
        ops = [g] + [t for j, t in enumerate(fs) if j != i]
        if f.nc == y.nc:
            contrib(f, E_MUL if len(ops) == 2 else E_MUL3, *ops, coef=coef)
            continue
        vec = [t for t in ops if t.nc == 3]
        sca = [t for t in ops if t.nc == 1]
        if len(vec) != 2 or len(sca) > 1:
            raise NotImplementedError("component reduction needs exactly two vector operands")
        contrib(f, E_DOT3, vec[0], vec[1], sca[0] if sca else None, coef=coef)


def _act_prod_adj(out, contrib, y, g, a, b, c, kind, order, coef):
    """y = coef * s^(o)(a) * b [* c]."""
    # a_bar += coef s^(o+1)(a) * g * b [* c]
    if c is None:
        if a.nc == y.nc:
            contrib(a, E_ACT, a, g, b, kind * 4 + order + 1, coef)
        else:
            raise NotImplementedError("activation of a scalar gating a vector")
        # b_bar += coef s^(o)(a) * g
        if b.nc == y.nc:
            contrib(b, E_ACT, a, g, None, kind * 4 + order, coef)
        else:
            raise NotImplementedError
    else:
        raise NotImplementedError("three-factor activation product")


# ----------------------------------------------------------------------------- composition
def _reads(ins):
    if ins[0] == "lin":
        return [x for x, _, _ in ins[2]] + ([ins[1]] if ins[5] else [])
    _, op, y, a, b, c, arg, coef, acc = ins
    return [t for t in (a, b, c) if t is not None] + ([y] if acc else [])


def _writes(ins):
    return ins[1] if ins[0] == "lin" else ins[2]


def concat_pruned(head, tail, keep_out=()):
    """``head`` instructions followed by ``tail``, with head instructions whose results are
    never read (by a later kept head instruction or any tail instruction) and are not in
    ``keep_out`` removed: the backward programs recompute only the forward values they use."""
    need = {v.base.id for v in keep_out}
    for ins in tail:
        for t in _reads(ins):
            need.add(t.base.id)
    kept = []
    for ins in reversed(head):
        y = _writes(ins)
        if y.base.id in need:
            kept.append(ins)
            for t in _reads(ins):
                need.add(t.base.id)
    out = Prog()
    out.ins = list(reversed(kept)) + list(tail)
    return out


# ----------------------------------------------------------------------------- torch executor
def _act(x, kind, order):
    if kind == 0:  # identity
        return x if order == 0 else (torch.ones_like(x) if order == 1 else torch.zeros_like(x))
    if kind == 1:  # relu
        if order == 0:
            return torch.relu(x)
        return (x > 0).to(x.dtype) if order == 1 else torch.zeros_like(x)
    if kind == 2:  # silu
        s = torch.sigmoid(x)
        if order == 0:
            return x * s
        if order == 1:
            return s * (1 + x * (1 - s))
        return s * (1 - s) * (2 + x * (1 - 2 * s))
    if kind == 3:  # tanh
        t = torch.tanh(x)
        if order == 0:
            return t
        if order == 1:
            return 1 - t * t
        return -2 * t * (1 - t * t)
    if kind == 4:  # sigmoid
        s = torch.sigmoid(x)
        if order == 0:
            return s
        if order == 1:
            return s * (1 - s)
        return s * (1 - s) * (1 - 2 * s)
    raise ValueError(kind)


def _get(env, v, N):
    t = env[v.base.id]
    b = v.base
    t3 = t.view(N, b.nc, b.w)
    return t3[:, :, v.c0:v.c0 + v.w]


def _bc(t, nc):
    return t if t.shape[1] == nc else t.expand(-1, nc, -1)


def run_torch(prog, env, weights, mask, N, dtype=None):
    """Execute ``prog`` over all rows (CPU twin of the device interpreter).

    env: {base Val id: tensor [N, nc * w]} holding the inputs; allocated values are added.
    weights: list of tensors indexed by Weight.pid / bias pid; mask: [N] (0/1) or None."""
    dev = next(iter(env.values())).device
    dtype = dtype or next(iter(env.values())).dtype

    def alloc(v):
        b = v.base
        if b.id not in env:
            env[b.id] = torch.zeros(N, b.nc * b.w, device=dev, dtype=dtype)

    for ins in prog.ins:
        if ins[0] == "lin":
            _, y, xs, trans, bias, acc = ins
            alloc(y)
            acc_t = None
            for x, W, k0 in xs:
                xv = _get(env, x, N)
                Wt = weights[W.pid]
                if trans:
                    Wb = Wt[:, k0:k0 + x.w]
                    r = torch.einsum("nck,ok->nco", xv, Wb)
                else:
                    Wb = Wt[:, k0:k0 + y.w]
                    r = torch.einsum("nco,ok->nck", xv, Wb)
                acc_t = r if acc_t is None else acc_t + r
            if bias is not None:
                acc_t = acc_t + weights[bias].view(1, 1, -1)
            yv = _get(env, y, N)
            if acc:
                yv += acc_t
            else:
                yv.copy_(acc_t)
            continue
        _, op, y, a, b, c, arg, coef, acc = ins
        alloc(y)
        yv = _get(env, y, N)
        if op == E_ZERO:
            yv.zero_()
            continue
        A = _get(env, a, N)
        B = _get(env, b, N) if b is not None else None
        C = _get(env, c, N) if c is not None else None
        nc = y.nc
        if op == E_COPY:
            r = _bc(A, nc)
        elif op == E_MUL:
            r = _bc(A, nc) * _bc(B, nc)
        elif op == E_MUL3:
            r = _bc(A, nc) * _bc(B, nc) * _bc(C, nc)
        elif op == E_ACT:
            kind, order = _act_code(arg)
            r = _act(_bc(A, nc), kind, order)
            if B is not None:
                r = r * _bc(B, nc)
            if C is not None:
                r = r * _bc(C, nc)
        elif op == E_DOT3:
            r = (A * B).sum(1, keepdim=True)
            if C is not None:
                r = r * C
        elif op == E_NORM3:
            n2 = (A * A).sum(1, keepdim=True)
            r = torch.sqrt(n2)
        elif op == E_SINV:
            r = torch.where(A > 0, 1.0 / torch.where(A > 0, A, torch.ones_like(A)), torch.zeros_like(A))
        elif op == E_MASK:
            m = mask.view(N, 1, 1).to(A.dtype) if mask is not None else torch.ones(N, 1, 1, dtype=A.dtype,
                                                                                   device=A.device)
            r = A * m
        else:
            raise NotImplementedError(op)
        if coef != 1.0:
            r = r * coef
        if acc:
            yv += r
        else:
            yv.copy_(r)
    return env


def wgrads_torch(wg, env, N, weights, grads):
    """Apply weight-gradient records (``reverse``) into ``grads`` (list aligned with weights,
    tensors or None)."""
    for rec in wg:
        if rec[0] == "w":
            _, pid, k0, G, X, trans = rec
            g = _get(env, G, N).reshape(N * G.nc, G.w)
            x = _get(env, X, N).reshape(N * X.nc, X.w)
            if trans:  # y = x W^T: W[:, k0:k0+K] += G^T X
                d = g.t() @ x
                sl = (slice(None), slice(k0, k0 + X.w))
            else:  # y = x W (y width K): W[:, k0:k0+K] += X^T G
                d = x.t() @ g
                sl = (slice(None), slice(k0, k0 + G.w))
            if grads[pid] is None:
                grads[pid] = torch.zeros_like(weights[pid])
            grads[pid][sl] += d
        else:
            _, pid, G = rec
            g = _get(env, G, N).reshape(N * G.nc, G.w)
            if grads[pid] is None:
                grads[pid] = torch.zeros_like(weights[pid])
            grads[pid] += g.sum(0)
    return grads


# ----------------------------------------------------------------------------- device compile
INS_INTS = 64
OPD_INTS = 12  # per operand: present, global kind, global index, gld, LDS offset, lld, cs, c0, w, nc


LDS_FLOATS = 160 * 1024 // 4  # one workgroup per CU may take all of it
BUF_INTS = 6
# buffer kinds of the interpreter: global workspace, external pointer, LDS only,
# LDS + global-workspace mirror, LDS + external-pointer mirror
B_WS, B_PTR, B_LDS, B_LDS_WS, B_LDS_PTR = range(5)


def _substitute(prog, old_root, new_root):
    """Reads of ``old_root`` (and its slices) -> ``new_root`` in a copy of the instruction list."""
    def sub(v):
        if v is None or v.base is not old_root:
            return v
        return new_root if v.full else new_root.slice(v.c0, v.w)

    out = []
    for ins in prog:
        if ins[0] == "lin":
            _, y, xs, trans, bias, acc = ins
            out.append(("lin", y, [(sub(x), W, k0) for x, W, k0 in xs], trans, bias, acc))
        else:
            _, op, y, a, b, c, arg, coef, acc = ins
            out.append(("ew", op, y, sub(a), sub(b), sub(c), arg, coef, acc))
    return out


def compile_device(prog, ext_roots, n_weights, inputs=(), keep_global=(), lds_budget=None):
    """Lower ``prog`` to the interpreter's tables (csrc/rowprog.hip).

    ext_roots: root Vals held in external tensors, in pointer-table order after the
    ``n_weights`` weight pointers.  ``inputs`` (ext roots the program only reads) are staged
    into LDS by a copy right before their first use; every value lives in the workgroup's
    LDS for its live range (first-fit by liveness), mirrored to its global home when it is
    an external output or ``keep_global`` (read later by the weight-gradient launch).
    Values that do not fit stay in the global workspace.  Returns (ins int32 [n, INS_INTS],
    bufs int32 [nb, BUF_INTS], global workspace floats per row, LDS floats per row,
    {root id: buffer index})."""
    import numpy as np

    ext = {v.id: k for k, v in enumerate(ext_roots)}
    inp = {v.id for v in inputs}
    keep = {v.id for v in keep_global}
    ins_list = list(prog.ins)
    if lds_budget is None:
        # floats per row of the 16-row block; the program itself (+ staged copies) is staged
        # into LDS too: reserve room for it (ints, generous for the input copies)
        lds_budget = max(0, (LDS_FLOATS - (len(ins_list) + 16) * INS_INTS) // 16)
    # stage read-only external inputs through LDS
    shadows = {}
    for v in ext_roots:
        if v.id not in inp:
            continue
        first = None
        for k, ins in enumerate(ins_list):
            if any(t.base is v for t in _reads(ins)):
                first = k
                break
        if first is None:
            continue
        sh = Val(v.w, v.nc, name=f"lds({v.name})")
        rest = _substitute(ins_list[first:], v, sh)
        ins_list = ins_list[:first] + [("ew", E_COPY, sh, v, None, None, 0, 1.0, False)] + rest
        shadows[sh.id] = v.id
    # barrier elision: the interpreter maps element (row, component, column f) of an
    # element-wise instruction to wave row % waves, lane f % 64 (all components in that
    # thread), so an element-wise instruction may follow another without a barrier when
    # every value it reads that was written since the last barrier was written by the same
    # threads: same root, column offsets congruent mod 64.  LINs read across rows and
    # columns: barriers around them always.
    nb = len(ins_list)
    no_bar = [False] * nb
    group = [0] * nb
    g_id, written = 0, {}

    def _w_off(ins):
        y = _writes(ins)
        return y.base.id, y.c0

    for k, ins in enumerate(ins_list):
        if k > 0:
            prev = ins_list[k - 1]
            ok = prev[0] == "ew" and ins[0] == "ew"
            if ok:
                for t in _reads(ins):
                    offs = written.get(t.base.id)
                    if offs is not None and any((o - t.c0) % 64 for o in offs):
                        ok = False
                        break
            if ok:
                no_bar[k - 1] = True
            else:
                g_id += 1
                written = {}
        group[k] = g_id
        r_, o_ = _w_off(ins)
        written.setdefault(r_, []).append(o_)
    group_start = {}
    for k in range(nb):
        group_start.setdefault(group[k], k)
    # liveness of every root (first write .. last read)
    first_w, last_r, roots = {}, {}, {}
    for k, ins in enumerate(ins_list):
        y = _writes(ins).base
        roots[y.id] = y
        first_w.setdefault(y.id, k)
        last_r.setdefault(y.id, k)
        for t in _reads(ins):
            roots[t.base.id] = t.base
            last_r[t.base.id] = max(last_r.get(t.base.id, k), k)
    # first-fit LDS allocation in instruction order (a slot is reused only after its last
    # reader finished: instructions are separated by a barrier)
    lds_off, free, top = {}, [], 0
    active = []
    for k, ins in enumerate(ins_list):
        still = []
        g0 = group_start[group[k]]  # within a barrier-free group other threads may still read
        for rid, off, size in active:
            if last_r[rid] < g0:
                free.append((off, size))
            else:
                still.append((rid, off, size))
        active = still
        y = _writes(ins).base
        if y.id in lds_off or first_w[y.id] != k:
            continue  # a value gets its LDS slot at its first write, or never
        size = y.nc * y.w + 1  # odd row stride: MFMA A-operand reads hit distinct banks
        free.sort()
        slot = None
        for q, (off, sz) in enumerate(free):
            if sz >= size:
                slot = off
                free[q] = (off + size, sz - size)
                if free[q][1] == 0:
                    free.pop(q)
                break
        if slot is None and top + size <= lds_budget:
            slot = top
            top += size
        if slot is not None:
            lds_off[y.id] = slot
            active.append((y.id, slot, size))
    bufs, where = [], {}
    prefix = [0]

    def buf(v):
        b = v.base
        if b.id in where:
            return where[b.id]
        lo = lds_off.get(b.id, -1)
        if b.id in ext:
            kind = B_PTR if lo < 0 else B_LDS_PTR
            g = n_weights + ext[b.id]
        elif lo >= 0 and b.id not in keep:
            kind, g = B_LDS, 0
        else:
            kind = B_WS if lo < 0 else B_LDS_WS
            g = prefix[0]
            prefix[0] += b.w * b.nc
        where[b.id] = len(bufs)
        bufs.append((kind, g, b.w, b.nc, lo, 0))
        return where[b.id]

    def opnd(v):
        """Operand descriptor embedded in the instruction (no table lookup on the device):
        [present, global kind (0 none, 1 workspace, 2 pointer), global index, global row
        stride, LDS offset (-1 none), LDS row stride, component stride, c0, w, nc]."""
        if v is None:
            return [0] * OPD_INTS
        kind, g, w, nc, lo, _ = bufs[buf(v)]
        gk = {B_WS: 1, B_LDS_WS: 1, B_PTR: 2, B_LDS_PTR: 2}.get(kind, 0)
        return [1, gk, g if gk else 0, nc * w, lo, nc * w + 1, w, v.c0, v.w, v.nc, 0, 0]

    rows = []
    for ins in ins_list:
        r = [0] * INS_INTS
        if ins[0] == "lin":
            _, y, xs, trans, bias, acc = ins
            assert 1 <= len(xs) <= 2, "LIN with more than two K blocks"
            W = xs[0][1]
            assert all(t[1] is W for t in xs), "K blocks of one LIN share one weight"
            r[0], r[4] = 1, int(acc)
            ops_ = [y, xs[0][0], xs[1][0] if len(xs) > 1 else None, None]
            # fast-path flag: every A operand is an LDS value (the destination may be anywhere)
            r[5] = int(all(t is None or bufs[buf(t)][4] >= 0 for t in ops_[1:3]))
            r[56], r[57] = W.pid, W.K
            r[58] = xs[0][2]
            r[59] = xs[1][2] if len(xs) > 1 else 0
            r[60] = bias if bias is not None else -1
            r[61] = int(trans)
        else:
            _, op, y, a, b, c, arg, coef, acc = ins
            r[0], r[1], r[2] = 0, op, arg
            r[3] = int(np.array([coef], dtype=np.float32).view(np.int32)[0])
            r[4] = int(acc)
            ops_ = [y, a, b, c]
            # fast-path flag: every operand (incl. the destination) is an LDS value
            r[5] = int(all(t is None or bufs[buf(t)][4] >= 0 for t in ops_))
        r[6] = int(no_bar[len(rows)])  # no barrier after this instruction
        for q, v in enumerate(ops_):
            r[8 + OPD_INTS * q: 8 + OPD_INTS * (q + 1)] = opnd(v)
        rows.append(r)
    ins = np.asarray(rows, dtype=np.int32).reshape(-1, INS_INTS)
    return ins, np.asarray(bufs, dtype=np.int32).reshape(-1, BUF_INTS), prefix[0], top, where


def wgrad_rounds(wg):
    """Group weight-gradient records into launch rounds: within a round every destination
    (weight column block) is distinct; a later record on a destination accumulates onto the
    earlier round's result.  Bias records ride with the k0 = 0 weight record of the same
    adjoint.  Returns [[(pid, k0, G, X, bias_pid | None, accumulate)]], {pid: covered}."""
    bias_of = {}
    for rec in wg:
        if rec[0] == "b":
            bias_of.setdefault(rec[2].id, []).append(rec[1])
    seen = {}
    rounds = []
    # records carrying a bias first: the bias is written (not accumulated) in its first round
    ws_ = [r for r in wg if r[0] == "w"]
    ws_ = [r for r in ws_ if r[2] == 0 and bias_of.get(r[3].id)] + \
        [r for r in ws_ if not (r[2] == 0 and bias_of.get(r[3].id))]
    for rec in ws_:
        _, pid, k0, G, X, trans = rec
        assert trans, "weight gradients of x W products are not generated"
        key = (pid, k0)
        r = seen.get(key, 0)
        seen[key] = r + 1
        bias = None
        if k0 == 0 and bias_of.get(G.id):
            bias = bias_of[G.id].pop(0)
        while len(rounds) <= r:
            rounds.append([])
        rounds[r].append((pid, k0, G, X, bias, r > 0))
    return rounds
