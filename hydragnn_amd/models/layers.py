"""Small building blocks shared by the model stacks."""
import torch
from torch import nn


class Linear(nn.Linear):
    """``nn.Linear`` (same parameters/state-dict keys) whose backward uses the
    split-K weight-gradient HIP kernel for tall activations (``ops/linear.py``)."""

    def forward(self, x):
        from ..ops.linear import linear

        return linear(x, self.weight, self.bias)


class BatchNorm(nn.Module):
    """Node-feature batch norm with PyG ``BatchNorm`` parameter naming (``.module``).

    Reference: PyG ``torch_geometric.nn.BatchNorm`` used at ``Base.py:206,215``
    and in GPS (``gps.py:80-83``).  Optional ``mask``-free fast path; padded
    rows are excluded through ``num_valid`` when the batch is padded for graph
    capture (see ``train/step.py``).
    """

    def __init__(self, in_channels, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True):
        super().__init__()
        self.in_channels = in_channels
        self.module = nn.BatchNorm1d(in_channels, eps=eps, momentum=momentum, affine=affine,
                                     track_running_stats=track_running_stats)

    def reset_parameters(self):
        self.module.reset_parameters()

    def forward(self, x, num_valid=None):
        from ..ops.norm import batch_norm  # local import to avoid cycles

        return batch_norm(x, self.module, num_valid)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels})"


class Ctx:
    """Per-batch message-passing context handed to every conv layer."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def get(self, k, default=None):
        return self.__dict__.get(k, default)

    def copy(self, **kw):
        d = dict(self.__dict__)
        d.update(kw)
        return Ctx(**d)


def mlp(dims, act, last_act=False, bias=True):
    layers = []
    for i in range(len(dims) - 1):
        layers.append(Linear(dims[i], dims[i + 1], bias=bias))
        if i < len(dims) - 2 or last_act:
            layers.append(act)
    return nn.Sequential(*layers)
