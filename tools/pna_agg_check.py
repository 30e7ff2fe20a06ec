"""Debug aid (python tools/pna_agg_check.py <pytest args>): compares every fused PNA aggregation (ops.pna.pna_aggregate)
with the composite, forward and backward, and prints the largest differences (eager only)."""
import torch

from hydragnn_amd import _native
from hydragnn_amd.ops import pna


def install():
    orig = pna.pna_aggregate

    def checked(m, si, avg_deg, aggregators=("mean", "min", "max", "std"),
                scalers=("identity", "amplification", "attenuation", "linear")):
        out = orig(m, si, avg_deg, aggregators, scalers)
        if not (m.is_cuda and "PNAAggFused" in type(out.grad_fn).__name__ if out.grad_fn is not None else False):
            return out
        mr = m.detach().clone().requires_grad_(True)
        with pna.composite_mode(True):
            ref = pna.pna_aggregate_composite(mr, si, avg_deg, aggregators, scalers)
        fd = (out.detach() - ref.detach()).abs().max().item()
        print(f"[pna-check] fwd E={m.shape[0]} F={m.shape[1]} N={si.num_segments} maxdiff={fd:.3e} "
              f"scale={ref.abs().max().item():.3e} finite={bool(torch.isfinite(m).all())}", flush=True)

        def hook(g):
            (gr,) = torch.autograd.grad(ref, mr, g, retain_graph=True)
            codes = 0
            for i, s in enumerate(scalers):
                codes |= pna._SCALER_CODE[s] << (3 * i)
            _, stat, arg = _native.ops().seg_pna_agg(m.detach().contiguous(), si.rowptr, si.perm, len(scalers), codes,
                                                     float(avg_deg["log"]), float(avg_deg["lin"]), 1e-5, 1e-5 ** 0.5)
            gf = _native.ops().seg_pna_agg_bwd(g.contiguous(), m.detach().contiguous(), si.rowptr, si.perm, stat, arg,
                                               len(scalers), codes, float(avg_deg["log"]), float(avg_deg["lin"]))
            bd = (gf - gr).abs()
            i = int(bd.argmax())
            print(f"[pna-check] bwd maxdiff={bd.max().item():.3e} at {divmod(i, gf.shape[1])} "
                  f"scale={gr.abs().max().item():.3e} rowptrN={int(si.rowptr[-1])} E={m.shape[0]}", flush=True)
            return g

        if out.requires_grad:
            out.register_hook(hook)
        return out

    pna.pna_aggregate = checked
    import hydragnn_amd.models.painn as painn
    painn.pna_aggregate = checked


if __name__ == "__main__":
    # python tools/pna_agg_check.py <pytest args>: run pytest in-process with the checker installed
    import sys

    import pytest

    install()
    sys.exit(pytest.main(sys.argv[1:]))
