"""Checkpoint / resume and the NaN/Inf step guard (§5.3)."""
import os

import torch

from hydragnn_amd.optim.adamw import FusedAdamW


def test_nan_guard_skips_update_cpu():
    p = torch.nn.Parameter(torch.ones(4))
    opt = FusedAdamW([p], lr=0.1)
    p.grad = torch.ones(4)
    opt.guard = torch.tensor(float("nan"))
    opt.step()
    assert torch.equal(p.data, torch.ones(4)) and opt.skipped_steps() == 1
    opt.guard = torch.tensor(1.0)
    opt.step()
    assert not torch.equal(p.data, torch.ones(4))


def test_trainer_state_roundtrip(tmp_path, monkeypatch):
    """A run interrupted after k epochs resumes at epoch k with the scheduler, early-stopping
    and RNG state it had (the reference persists only model + optimizer)."""
    from hydragnn_amd.train.train_validate_test import _record_trainer_state, restore_trainer_state
    from hydragnn_amd.utils.model import EarlyStopping, load_trainer_state, save_trainer_state

    monkeypatch.chdir(tmp_path)
    p = torch.nn.Parameter(torch.ones(2))
    opt = torch.optim.AdamW([p], lr=1e-2)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=1, min_lr=1e-5)
    for v in (1.0, 2.0, 3.0):
        sched.step(v)
    es = EarlyStopping(patience=5)
    es(1.0)
    es(2.0)
    st = {}
    torch.manual_seed(123)
    _record_trainer_state(st, 6, sched, es, None)
    want = torch.rand(3)
    save_trainer_state("run", st)
    assert os.path.exists("logs/run/run_trainer_state.pk")
    back = load_trainer_state("run")
    assert back["epoch"] == 7 and back["early_stopping"] == es.state_dict()
    opt2 = torch.optim.AdamW([torch.nn.Parameter(torch.ones(2))], lr=1e-2)
    sched2 = torch.optim.lr_scheduler.ReduceLROnPlateau(opt2, mode="min", factor=0.5, patience=1, min_lr=1e-5)
    torch.manual_seed(999)
    restore_trainer_state(back, sched2)
    assert sched2.num_bad_epochs == sched.num_bad_epochs and sched2.best == sched.best
    assert torch.equal(torch.rand(3), want)
