"""Fused multi-tensor AdamW (HIP kernel ``csrc/optim.hip``), hipGraph-capturable.

API-compatible with ``torch.optim.AdamW`` (param_groups, state_dict with
per-parameter ``step``/``exp_avg``/``exp_avg_sq``), so reference-style
checkpoints (``optimizer_state_dict``) and ``ReduceLROnPlateau`` work.  The
learning rate and step counter are device scalars: changing ``lr`` through
``param_groups`` is picked up at the next ``step()`` without recapturing.

GPU: one kernel launch for all parameters (its last block advances the step counts).  CPU: the
plain-torch update (reference math), used by the CPU tests.
"""
import struct

import torch

from .. import _native


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, adamw=True):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adamw = adamw
        self._tables = None
        self._dev_state = None
        self._host_lr = None
        # optional NaN/Inf guard: the step's loss tensor; a non-finite loss skips the update on
        # the device (captured into the step graph, no host sync) and is counted
        self.guard = None
        self._skipped_cpu = 0
        # optional per-parameter usage flags (device scalars, > 0 = used this step): set by
        # the captured training step for parameters that a step may not reach (heads of
        # branches absent from a batch), which then keep torch's skip-if-no-grad semantics
        self._flags = {}

    def set_usage_flags(self, flags):
        """``{param: 1-element device tensor view}``; rebuilds the tables at the next step."""
        self._flags = dict(flags)
        self._tables = None

    def _init_state(self):
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)

    def _build_tables(self):
        """Per param-group (ref blob, block table, device [step, lr])."""
        tables = []
        for group in self.param_groups:
            refs, blocks = [], []
            ps = [p for p in group["params"] if p.grad is not None]
            for ti, p in enumerate(ps):
                st = self.state[p]
                n = p.numel()
                assert p.is_contiguous() and p.grad.is_contiguous()
                step = st["step"]
                if not (torch.is_tensor(step) and step.is_cuda and step.dtype == torch.float32 and step.numel() == 1):
                    step = st["step"] = torch.full((), float(step), dtype=torch.float32, device=p.device)
                fl = self._flags.get(p)
                refs.append((p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), n,
                             step.data_ptr(), 0 if fl is None else fl.data_ptr()))
                for c in range((n + 2047) // 2048):
                    blocks.append((ti, c))
            if not ps:
                tables.append(None)
                continue
            # TensorRef {float* p; const float* g; float* m; float* v; int64 n; float* step;
            #            const float* used;} = 56 bytes
            blob = b"".join(struct.pack("<QQQQqQQ", *r) for r in refs)
            assert len(blob) == 56 * len(refs) and struct.unpack_from("<QQQQqQQ", blob, 56 * (len(refs) - 1)) == refs[-1]
            dev = ps[0].device
            rb = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
            bt = torch.tensor(blocks, dtype=torch.int32).view(-1).to(dev)
            state = torch.tensor([0.0, group["lr"], 0.0], dtype=torch.float32, device=dev)
            tables.append([rb, bt, state, group["lr"], tuple(p.grad.data_ptr() for p in ps), ps,
                           self._hp_key(group)])
        self._tables = tables

    def _tables_valid(self):
        if self._tables is None:
            return False
        for group, t in zip(self.param_groups, self._tables):
            ps = [p for p in group["params"] if p.grad is not None]
            if t is None:
                if ps:
                    return False
                continue
            if tuple(p.grad.data_ptr() for p in ps) != t[4]:
                return False
            # a checkpoint load / state replacement swaps the per-parameter step tensors
            if any(not torch.is_tensor(self.state[p].get("step")) or not self.state[p]["step"].is_cuda for p in ps):
                return False
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._init_state()
        gpu = any(p.is_cuda for g in self.param_groups for p in g["params"])
        from ..ops.pna import fused

        if not gpu or not fused("adamw"):
            self._cpu_step()
            return loss
        capturing = torch.cuda.is_current_stream_capturing()
        if not self._tables_valid():
            assert not capturing, "FusedAdamW tables must be built before graph capture"
            self._build_tables()
        for group, t in zip(self.param_groups, self._tables):
            if t is None:
                continue
            if t[3] != group["lr"] and not capturing:
                t[2][1].fill_(group["lr"])
                t[3] = group["lr"]
            b1, b2 = group["betas"]
            g = self.guard if (self.guard is not None and self.guard.is_cuda) else None
            _native.ops().adamw_step(t[0], t[1], t[2], b1, b2, group["eps"], group["weight_decay"], self.adamw, 1.0,
                                     None if g is None else g.reshape(1).float())
        return loss

    @staticmethod
    def _hp_key(group):
        """The hyper-parameters a captured launch bakes in as kernel arguments (not lr)."""
        return (tuple(float(b) for b in group["betas"]), float(group["eps"]), float(group["weight_decay"]))

    def sync_hparams(self):
        """Copy the host learning rates into the device scalars the captured update reads.
        A captured step never calls ``step()`` on the host, so without this a schedule
        (ReduceLROnPlateau, ``param_groups[...]["lr"] = ...``) would never reach a replayed
        step.  Called by ``TrainStep`` before every replay; a no-op unless an lr changed.
        Returns False when another hyper-parameter changed since the tables were built (those
        are kernel arguments of the captured launch: the caller must recapture)."""
        if self._tables is None:
            return True
        ok = True
        for group, t in zip(self.param_groups, self._tables):
            if t is None:
                continue
            if t[6] != self._hp_key(group):
                ok = False  # betas / eps / weight decay are captured launch arguments
            if t[3] != group["lr"]:
                t[2][1].fill_(group["lr"])
                t[3] = group["lr"]
        return ok

    def skipped_steps(self):
        """Updates skipped by the non-finite guard so far (one device read)."""
        n = self._skipped_cpu
        for t in self._tables or []:
            if t is not None:
                n += int(t[2][2].item())
                break
        return n

    def _cpu_step(self):
        if self.guard is not None and not self.guard.is_cuda and not bool(torch.isfinite(self.guard).all()):
            self._skipped_cpu += 1
            return
        for group in self.param_groups:
            b1, b2 = group["betas"]
            lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                fl = self._flags.get(p)
                if fl is not None and not float(fl.reshape(-1)[0]) > 0.0:
                    continue
                st = self.state[p]
                st["step"] += 1
                t = float(st["step"])
                g = p.grad
                if self.adamw:
                    p.mul_(1 - lr * wd)
                else:
                    g = g + wd * p
                st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
                st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
                bc1 = 1 - b1 ** t
                bc2 = 1 - b2 ** t
                denom = (st["exp_avg_sq"].sqrt() / (bc2 ** 0.5)).add_(eps)
                p.addcdiv_(st["exp_avg"], denom, value=-lr / bc1)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables = None
