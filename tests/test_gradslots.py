"""Gradient slots (parallel/gradslots.py): ops writing gradients straight into the flat
buffer of BucketedGradSync; the pack copies only the rest, in contiguous runs."""
import pytest
import torch

from hydragnn_amd.parallel import gradslots
from hydragnn_amd.parallel.ddp import BucketedGradSync


def _params(shapes, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(*s, generator=g)) for s in shapes]


def _expected(sync, grads, loss):
    out = torch.zeros_like(sync.flat)
    for p, g in grads.items():
        o = sync.offset[p]
        out[o:o + p.numel()] = g.reshape(-1)
    if loss is not None:
        out[sync.total] = loss
    return out


def test_pack_skips_provided_and_in_place_slots():
    ps = _params([(3, 4), (5,), (2, 2), (7,), (4, 3)])
    sync = BucketedGradSync(ps, bucket_cap_mb=1e9)
    g = torch.Generator().manual_seed(1)
    grads = {p: torch.randn(p.shape, generator=g) for p in ps}
    loss = torch.tensor(0.25)
    sync.release()
    sync.set_loss(loss)
    sync.begin()
    with gradslots.use(sync):
        sl = gradslots.slots([ps[1], ps[3]])
        assert sl is not None and all(s.shape == p.shape for s, p in zip(sl, [ps[1], ps[3]]))
        for s, p in zip(sl, [ps[1], ps[3]]):  # an op writes these two in place ...
            s.copy_(grads[p])
        gradslots.provide([ps[1], ps[3]])
    # ... autograd stole ps[0]'s gradient as the slot view itself (in place already) ...
    s0 = sync.slot(ps[0])
    s0.copy_(grads[ps[0]])
    ps[0].grad = s0
    # ... and handed over fresh tensors for the others
    ps[2].grad = grads[ps[2]].clone()
    ps[4].grad = grads[ps[4]].clone()
    sync.finish()
    # a lone rank without usage flags packs no guard slot (the step's guard reads the loss)
    assert not sync.guard_packed
    torch.testing.assert_close(sync.flat, _expected(sync, grads, None), rtol=0, atol=0)
    for p in ps:  # every parameter's grad is its flat view again
        assert p.grad.data_ptr() == sync.slot(p).data_ptr()
    assert not sync.provided and not sync.side_events


def test_shared_weight_second_use_adds_to_its_slot():
    """A weight used twice in one step: the first use writes its slot, the second gets no
    slot (its gradient comes back through autograd) and the pack adds it to the slot."""
    ps = _params([(3, 4), (5,)])
    sync = BucketedGradSync(ps, bucket_cap_mb=1e9)
    g1, g2, g0 = torch.randn(5), torch.randn(5), torch.randn(3, 4)
    sync.release()
    sync.set_loss(torch.tensor(1.0))
    sync.begin()
    with gradslots.use(sync):
        sl = gradslots.slots([ps[1]])
        sl[0].copy_(g1)
        gradslots.provide([ps[1]])
        assert gradslots.slots([ps[1]]) is None  # second use: autograd returns its gradient
    ps[1].grad = g2.clone()
    ps[0].grad = g0.clone()
    sync.finish()
    torch.testing.assert_close(sync.flat, _expected(sync, {ps[0]: g0, ps[1]: g1 + g2}, None), rtol=0, atol=1e-6)


def test_slots_none_outside_a_step_or_for_foreign_params():
    ps = _params([(2,), (3,)])
    other = _params([(4,)], seed=3)
    sync = BucketedGradSync(ps, bucket_cap_mb=1e9)
    assert gradslots.slots(ps) is None  # no active step
    with gradslots.use(sync):
        assert gradslots.slots(ps) is not None
        assert gradslots.slots(ps + other) is None
    assert gradslots.active() is None


def test_provided_params_count_down_their_bucket():
    """A provided parameter completes its bucket like an autograd gradient does (the
    all-reduce of a bucket whose every gradient was written in place still launches)."""
    ps = _params([(4,), (4,), (4,)])
    sync = BucketedGradSync(ps, bucket_cap_mb=16 / (1024 * 1024))  # one parameter per bucket
    assert len(sync.buckets) == 3
    launched = []
    sync._launch = lambda bi: launched.append(bi)
    sync.release()
    with gradslots.use(sync):
        gradslots.provide([ps[2]])  # during the forward, before begin()
    sync.world = 2  # the collective path (its launches are recorded, not run)
    sync.begin()
    # ps[2] is the first parameter of the reversed flat order: bucket 0 is complete
    assert launched == [0]
    sync._hook(ps[1])  # autograd's hook for a None contribution (a deferred weight gradient)
    assert launched == [0]
    ps[1].grad = torch.zeros(4)
    sync._hook(ps[1])  # the gradient itself
    assert launched == [0, 1]


@pytest.mark.gpu
def test_guard_waits_for_side_stream_loss():
    """The step guard (loss) and slot gradients written on a side stream are packed only
    after that stream's event (the pack used to read the loss unsynchronised)."""
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(torch.randn(64, 64, device=dev)) for _ in range(3)]
    sync = BucketedGradSync(ps, bucket_cap_mb=1e9, nflags=1)  # usage flags -> guard packed
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    for trial in range(3):
        sync.release()
        sync.begin()
        loss = torch.zeros((), device=dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000_000)  # the side stream lags far behind the main stream
            loss.fill_(1.5 + trial)
            sl = sync.slot(ps[2])
            sl.fill_(float(trial + 1))
        ev = torch.cuda.Event()
        ev.record(side)
        sync.set_loss(loss)
        sync.set_flags(torch.ones(1, device=dev))
        sync.provide([ps[2]], ev)
        for p in ps[:2]:
            p.grad = torch.full_like(p, 0.5)
        sync.finish()
        assert sync.guard_packed
        torch.cuda.synchronize()
        assert float(sync.guard) == 1.5 + trial
        assert torch.all(ps[2].grad == float(trial + 1))
        assert torch.all(ps[0].grad == 0.5)
