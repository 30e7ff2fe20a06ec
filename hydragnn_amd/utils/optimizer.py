"""Optimizer selection (reference ``utils/optimizer/optimizer.py:12-113``).

Same type strings: SGD, Adam, Adadelta, Adagrad, Adamax, AdamW, RMSprop, FusedLAMB;
``use_zero_redundancy`` shards optimizer state across ranks (ZeRO-1,
``parallel/zero.py``).  AdamW / Adam on GPU use the fused multi-tensor HIP
kernel (one launch per step, hipGraph-capturable); FusedLAMB is a native LAMB.
"""
import torch

from ..optim.adamw import FusedAdamW
from ..optim.lamb import Lamb


def _make(name, params, lr):
    gpu = any(p.is_cuda for p in params)
    if name == "SGD":
        return torch.optim.SGD(params, lr=lr)
    if name == "Adam":
        return FusedAdamW(params, lr=lr, weight_decay=0.0, adamw=False) if gpu else torch.optim.Adam(params, lr=lr)
    if name == "Adadelta":
        return torch.optim.Adadelta(params, lr=lr)
    if name == "Adagrad":
        return torch.optim.Adagrad(params, lr=lr)
    if name == "Adamax":
        return torch.optim.Adamax(params, lr=lr)
    if name == "AdamW":
        return FusedAdamW(params, lr=lr) if gpu else torch.optim.AdamW(params, lr=lr)
    if name == "RMSprop":
        return torch.optim.RMSprop(params, lr=lr)
    if name == "FusedLAMB":
        return Lamb(params, lr=lr)
    raise NameError("The string used to identify the optimizer is NOT recognized")


def select_standard_optimizer(model, optimizer_config):
    params = [p for p in model.parameters() if p.requires_grad]
    return _make(optimizer_config.get("type", "AdamW"), params, optimizer_config["learning_rate"])


def select_zero_redundancy_optimizer(model, optimizer_config):
    from ..parallel.zero import ZeroRedundancyOptimizer

    params = [p for p in model.parameters() if p.requires_grad]
    name = optimizer_config.get("type", "AdamW")
    lr = optimizer_config["learning_rate"]
    return ZeroRedundancyOptimizer(params, lambda ps: _make(name, ps, lr), elementwise=name != "FusedLAMB")


def select_optimizer(model, config):
    if config.get("use_zero_redundancy", False):
        return select_zero_redundancy_optimizer(model, config)
    return select_standard_optimizer(model, config)
