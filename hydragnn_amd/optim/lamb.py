"""LAMB optimizer (replaces DeepSpeed ``FusedLamb``, reference ``optimizer.py:29-36``).

Per-tensor trust ratio ||w|| / ||adam_update + wd*w||, multi-tensor ``torch._foreach``
math (a handful of fused launches per step regardless of parameter count).
"""
import torch


class Lamb(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_trust=10.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, max_trust=max_trust))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for g in self.param_groups:
            ps = [p for p in g["params"] if p.grad is not None]
            if not ps:
                continue
            b1, b2 = g["betas"]
            for p in ps:
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
            ms = [self.state[p]["exp_avg"] for p in ps]
            vs = [self.state[p]["exp_avg_sq"] for p in ps]
            gs = [p.grad for p in ps]
            for p in ps:
                self.state[p]["step"] += 1
            t = float(self.state[ps[0]]["step"])
            torch._foreach_mul_(ms, b1)
            torch._foreach_add_(ms, gs, alpha=1 - b1)
            torch._foreach_mul_(vs, b2)
            torch._foreach_addcmul_(vs, gs, gs, value=1 - b2)
            bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
            denom = torch._foreach_sqrt(vs)
            torch._foreach_div_(denom, bc2 ** 0.5)
            torch._foreach_add_(denom, g["eps"])
            upd = torch._foreach_div(ms, denom)
            torch._foreach_div_(upd, bc1)
            if g["weight_decay"]:
                torch._foreach_add_(upd, ps, alpha=g["weight_decay"])
            wn = torch._foreach_norm(ps)
            un = torch._foreach_norm(upd)
            for p, u, w, n in zip(ps, upd, wn, un):
                ratio = torch.where((w > 0) & (n > 0), (w / n).clamp(max=g["max_trust"]), torch.ones_like(w))
                p.add_(u * (-g["lr"] * ratio))
        return loss
