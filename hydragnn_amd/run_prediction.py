"""``run_prediction(config | path)`` (reference ``hydragnn/run_prediction.py:35-107``):
rebuild data + model, load ``./logs/<name>/<name>.pk``, run ``test()``, optionally
denormalise.  Returns (error, task_errors, true_values, predicted_values)."""
import json
import os
from functools import singledispatch

import torch

from .data.load_data import dataset_loading_and_splitting, to_device_loaders
from .models.create import create_model_config
from .parallel.distributed import get_device, get_distributed_model, setup_ddp
from .postprocess.postprocess import output_denormalize
from .train.train_validate_test import test
from .utils.config_utils import get_log_name_config, update_config
from .utils.model import load_existing_model


@singledispatch
def run_prediction(config, use_deepspeed=False):
    raise TypeError("Input must be filename string or configuration dictionary.")


@run_prediction.register
def _(config_file: str, use_deepspeed=False):
    with open(config_file, "r") as f:
        config = json.load(f)
    return run_prediction(config, use_deepspeed)


@run_prediction.register
def _(config: dict, use_deepspeed=False, model=None):
    os.environ.setdefault("SERIALIZED_DATA_PATH", os.getcwd())
    setup_ddp()
    verbosity = config["Verbosity"]["level"]
    train_loader, val_loader, test_loader = dataset_loading_and_splitting(config=config)
    config = update_config(config, train_loader, val_loader, test_loader)
    nn_cfg = config["NeuralNetwork"]
    if model is None:
        model = create_model_config(config=nn_cfg, verbosity=verbosity)
        model = get_distributed_model(model, verbosity)
        load_existing_model(model, get_log_name_config(config))
    if torch.cuda.is_available() and int(os.getenv("HYDRAGNN_DEVICE_DATA", "1")) == 1:
        module = model.module if hasattr(model, "module") else model
        _, _, test_loader = to_device_loaders((train_loader, val_loader, test_loader), get_device(), module.head_type,
                                              module.head_dims, attn_scope=getattr(module, "attn_scope", "batch"))
    error, error_rmse_task, true_values, predicted_values = test(
        test_loader, model, verbosity, compute_grad_energy=nn_cfg["Training"].get("compute_grad_energy", False))
    if nn_cfg["Variables_of_interest"].get("denormalize_output"):
        true_values, predicted_values = output_denormalize(nn_cfg["Variables_of_interest"]["y_minmax"], true_values,
                                                           predicted_values)
    return error, error_rmse_task, true_values, predicted_values
