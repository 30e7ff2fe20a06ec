"""Gradient slots: ops may write a parameter's gradient straight into the training step's
flat gradient buffer instead of returning it through autograd.

The captured / padded training step keeps every gradient in one flat buffer
(:class:`~hydragnn_amd.parallel.ddp.BucketedGradSync`); gradients that autograd hands over
are copied into it by one batched pack per bucket.  While a step's forward and backward run
under :func:`use`, an op that computes the gradients of some parameters itself (the fused
graph head, ``ops/mlp.py``) can ask for their :func:`slots`, write them there — possibly
from a side stream, overlapped with the rest of backward — and :func:`provide` them: the
pack skips them, the all-reduce bucket counts them, and the step joins the side stream
before the optimizer.  The op then returns no autograd gradient for those parameters.

Reference: the reference's DDP flattens gradients into buckets after autograd produced them
(``hydragnn/utils/distributed.py:332-351``); there is no equivalent of writing in place.
"""
import contextlib

_active = None


@contextlib.contextmanager
def use(sync):
    """Make ``sync`` (a BucketedGradSync / MultiGradSync, or None) the slot provider."""
    global _active
    prev, _active = _active, sync
    try:
        yield
    finally:
        _active = prev


def active():
    return _active


def slots(params):
    """Flat-buffer views for every parameter of ``params`` (None unless all have one, or when
    one of them was already provided this step: a second use of a shared weight returns its
    gradient through autograd, and the bucket pack adds it to the slot)."""
    s = _active
    if s is None:
        return None
    done = getattr(s, "provided", None)
    if done is not None and any(id(p) in done for p in params):
        return None
    out = []
    for p in params:
        v = s.slot(p)
        if v is None:
            return None
        out.append(v)
    return out


def provide(params, event=None):
    """The gradients of ``params`` are in their slots (after ``event``, when given)."""
    _active.provide(params, event)
