"""``run_training(config | path)`` (reference ``hydragnn/run_training.py:49-182``).

Pipeline: logging -> process group -> data (raw -> serialized -> splits ->
loaders) -> ``update_config`` -> model -> DDP wrap (bucketed RCCL all-reduce) ->
optimizer + ``ReduceLROnPlateau(factor=0.5, patience=5, min_lr=1e-5)`` ->
optional resume -> ``train_validate_test`` -> ``save_model`` -> timers.

On a GPU the splits are moved into HBM (``DeviceGraphStore``) and training
batches run through the hipGraph-captured ``TrainStep`` (set
``HYDRAGNN_CAPTURE=0`` for eager, ``HYDRAGNN_DEVICE_DATA=0`` for the host
loader path).  Force training (``compute_grad_energy``) captures the double
backward too (energy + force loss masked over the padded bucket).

``train_model(config, train_loader, val_loader, test_loader)`` is the same pipeline
from loaders the caller built (the reference examples' low-level sequence
``update_config -> create_model_config -> get_distributed_model -> select_optimizer ->
train_validate_test -> save_model``, e.g. ``examples/ising_model/train_ising.py``).
"""
import json
import os
from functools import singledispatch

import torch
import torch.distributed as dist

from .data.load_data import dataset_loading_and_splitting, to_device_loaders
from .models.create import create_model_config
from .parallel.distributed import get_device, get_distributed_model, setup_ddp
from .train.step import TrainStep
from .train.train_validate_test import train_validate_test
from .utils.config_utils import get_log_name_config, save_config, update_config
from .utils.model import get_summary_writer, load_existing_model_config, save_model
from .utils.optimizer import select_optimizer
from .utils.print_utils import print_distributed, setup_log
from .utils.time_utils import print_timers


@singledispatch
def run_training(config, use_deepspeed=False):
    raise TypeError("Input must be filename string or configuration dictionary.")


@run_training.register
def _(config_file: str, use_deepspeed=False):
    with open(config_file, "r") as f:
        config = json.load(f)
    return run_training(config, use_deepspeed)


def _device_path_enabled(config):
    # HYDRAGNN_DEVICE_DATA=2 forces the store/padded-step path on CPU (tests of the padding logic)
    flag = int(os.getenv("HYDRAGNN_DEVICE_DATA", "1"))
    return flag == 2 or (torch.cuda.is_available() and flag == 1)


def make_step_engine(config, model, optimizer, loaders):
    """On a GPU: move the split loaders into HBM (``DeviceGraphStore``) and build the
    captured ``TrainStep`` for ``model`` (plain, DDP-wrapped, or task-parallel
    ``MultiTaskModelMP``: encoder synced over WORLD, the branch decoder over its branch
    group, both inside the step graph).  Returns ``(engine | None, loaders)``."""
    if not _device_path_enabled(config):
        return None, loaders
    nn_cfg = config["NeuralNetwork"]
    module = model.module if hasattr(model, "module") else model
    loaders = to_device_loaders(tuple(loaders), get_device(), module.head_type, module.head_dims,
                                attn_scope=getattr(module, "attn_scope", "batch"))
    mode = "graph" if (int(os.getenv("HYDRAGNN_CAPTURE", "1")) == 1 and getattr(module, "capturable", True)) \
        else "eager"
    world = dist.get_world_size() if dist.is_initialized() else 1
    engine = TrainStep(model, mode=mode, world=world, optimizer=optimizer,
                       compute_grad_energy=nn_cfg["Training"].get("compute_grad_energy", False))
    engine.prepare(loaders[0].store, loaders[0].batch_size)
    return engine, tuple(loaders)


@run_training.register
def _(config: dict, use_deepspeed=False):
    assert not use_deepspeed, "DeepSpeed is not part of hydragnn_amd (ZeRO-1 via Optimizer.use_zero_redundancy)"
    verbosity = config["Verbosity"]["level"]
    os.environ.setdefault("SERIALIZED_DATA_PATH", os.getcwd())
    setup_log(get_log_name_config(config))
    setup_ddp()
    train_loader, val_loader, test_loader = dataset_loading_and_splitting(config=config)
    return train_model(config, train_loader, val_loader, test_loader)


def train_model(config, train_loader, val_loader, test_loader, log_name=None):
    """Train from prebuilt host loaders (any dataset class: serialized, pickle, columnar,
    DistDataset); ``update_config`` is applied here.  ``log_name`` defaults to the
    config-derived name (configs without a Dataset section must pass one).  Returns the
    (DDP-wrapped) model."""
    verbosity = config["Verbosity"]["level"]
    setup_ddp()
    config = update_config(config, train_loader, val_loader, test_loader)
    vis = config.get("Visualization", {})
    plot_init_solution = vis.get("plot_init_solution", False)
    plot_hist_solution = vis.get("plot_hist_solution", False)
    create_plots = vis.get("create_plots", False)
    nn_cfg = config["NeuralNetwork"]
    # Training.precision (extension key): "fp32" (reference numerics) or "bf16" (MFMA bf16
    # GEMMs with fp32 accumulation / storage / master weights; geometry, segment
    # reductions and normalisation stay fp32)
    from .ops.linear import set_precision

    set_precision(nn_cfg["Training"].get("precision", "fp32"))
    model = create_model_config(config=nn_cfg, verbosity=verbosity)
    log_name = log_name or get_log_name_config(config)
    model = get_distributed_model(model, verbosity, sync_batch_norm=nn_cfg["Architecture"].get("SyncBatchNorm", False),
                                  find_unused_parameters=True)
    optimizer = select_optimizer(model, nn_cfg["Training"]["Optimizer"])
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=0.5, patience=5,
                                                           min_lr=0.00001)
    writer = get_summary_writer(log_name)
    if dist.is_initialized():
        dist.barrier()
    save_config(config, log_name)
    load_existing_model_config(model, nn_cfg["Training"], optimizer=optimizer)
    trainer_state = {}
    if nn_cfg["Training"].get("continue"):
        from .train.train_validate_test import restore_trainer_state
        from .utils.model import load_trainer_state

        trainer_state = load_trainer_state(nn_cfg["Training"]["startfrom"]) or {}
        restore_trainer_state(trainer_state, scheduler)
    compute_grad_energy = nn_cfg["Training"].get("compute_grad_energy", False)
    engine, (train_loader, val_loader, test_loader) = make_step_engine(
        config, model, optimizer, (train_loader, val_loader, test_loader))
    from .parallel.zero import ZeroRedundancyOptimizer

    if isinstance(optimizer, ZeroRedundancyOptimizer) and hasattr(model, "_sync_enabled") and \
            (engine is None or engine.sync is None):
        # eager DDP + ZeRO-1: the optimizer reduce-scatters the gradients itself (no all-reduce)
        model._sync_enabled = False
        optimizer.reduce_grads = True
    print_distributed(verbosity, f"model: {nn_cfg['Architecture']['mpnn_type']}, "
                                 f"params: {sum(p.numel() for p in model.parameters())}")
    train_validate_test(model, optimizer, train_loader, val_loader, test_loader, writer, scheduler, nn_cfg, log_name,
                        verbosity, plot_init_solution, plot_hist_solution, create_plots,
                        compute_grad_energy=compute_grad_energy, step_engine=engine, trainer_state=trainer_state)
    save_model(model, optimizer, log_name)
    print_timers(verbosity)
    return model
