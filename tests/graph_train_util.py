"""Shared driver of the end-to-end accuracy tests (reference ``tests/test_graphs.py:26-198``):
generate the deterministic dataset (rank 0), run_training, run_prediction, check the
per-head RMSE and sample-MAE thresholds."""
import os
import warnings
import zlib

import torch

import hydragnn_amd
from hydragnn_amd.data.lsms import deterministic_graph_data
from hydragnn_amd.parallel.distributed import get_comm_size_and_rank
from hydragnn_amd.utils.config_utils import merge_config

from ci_configs import ci, thresholds


# Every model trains once from init seed 0, as the reference does (``create.py:131``).  The
# PNA / PNAPlus convolutions create and re-draw their parameters in the reference's order
# (PyG PNAConv / PNAPlusStack.py reset_parameters), which made seed 0 pass for the edge-length
# configurations that collapsed to a constant predictor with the previous draw order (CPU
# MAE 0.168 at seed 0; rounds 2-4 retried them with seeds 1, 2).  No per-model seed retries.
INIT_SEEDS = (0,)


def unittest_train_model(mpnn_type, global_attn_engine, global_attn_type, ci_input, use_lengths, workdir,
                         overwrite_config=None, num_samples_tot=500):
    err = None
    seeds = INIT_SEEDS
    if overwrite_config and "init_seed" in overwrite_config.get("NeuralNetwork", {}).get("Architecture", {}):
        seeds = (overwrite_config["NeuralNetwork"]["Architecture"]["init_seed"],)
    for i, seed in enumerate(seeds):
        try:
            return _train_once(mpnn_type, global_attn_engine, global_attn_type, ci_input, use_lengths, workdir,
                               overwrite_config, num_samples_tot, seed)
        except AssertionError as e:
            err = e
            if i + 1 < len(seeds):
                # surfaced in the pytest warnings summary (visible in -q driver logs) and in
                # RETRIES_LOG, so a pass that needed a retry is never silent
                msg = f"{mpnn_type} (lengths={use_lengths}, {ci_input}): seed {seed} missed the thresholds ({e}); " \
                      f"retraining with seed {seeds[i + 1]}"
                warnings.warn(msg)
                log = os.environ.get("HYDRAGNN_TEST_RETRIES_LOG")
                if log:
                    with open(log, "a") as f:
                        f.write(msg + "\n")
    raise err


def ci_config(mpnn_type, ci_input, workdir, overwrite_config=None, num_samples_tot=500, init_seed=0,
              use_lengths=False, global_attn_engine="", global_attn_type=""):
    """The CI config with dataset paths resolved under ``workdir``; rank 0 generates the
    deterministic BCC dataset the first time (reference ``tests/test_graphs.py:40-95``)."""
    _, rank = get_comm_size_and_rank()
    os.environ["SERIALIZED_DATA_PATH"] = workdir
    config = ci(ci_input)
    arch = config["NeuralNetwork"]["Architecture"]
    arch["global_attn_engine"] = global_attn_engine
    arch["global_attn_type"] = global_attn_type
    arch["mpnn_type"] = mpnn_type
    if overwrite_config:
        config = merge_config(config, overwrite_config)
        arch = config["NeuralNetwork"]["Architecture"]
    # reuse serialized files when present
    for split in list(config["Dataset"]["path"].keys()):
        name = config["Dataset"]["name"] + ("" if split == "total" else "_" + split) + ".pkl"
        pkl = os.path.join(workdir, "serialized_dataset", name)
        if os.path.exists(pkl):
            config["Dataset"]["path"][split] = pkl
    if mpnn_type == "MFC" and ci_input == "ci_multihead":
        arch["task_weights"][0] = 2
    if use_lengths:
        arch["edge_features"] = ["lengths"]
    arch["init_seed"] = init_seed
    if rank == 0:
        pkl_input = list(config["Dataset"]["path"].values())[0].endswith(".pkl")
        if not pkl_input:
            for split, path in config["Dataset"]["path"].items():
                full = os.path.join(workdir, path)
                config["Dataset"]["path"][split] = full
                os.makedirs(full, exist_ok=True)
                perc = config["NeuralNetwork"]["Training"]["perc_train"]
                n = {"total": num_samples_tot, "train": int(num_samples_tot * perc)}.get(
                    split, int(num_samples_tot * (1 - perc) * 0.5))
                if not os.listdir(full):
                    deterministic_graph_data(full, number_configurations=n, seed=97 + zlib.crc32(f"{split}-{n}".encode()) % 10000)
    else:
        for split, path in config["Dataset"]["path"].items():
            if not path.endswith(".pkl"):
                config["Dataset"]["path"][split] = os.path.join(workdir, path)
    return config


def run_ci(mpnn_type, ci_input, workdir, overwrite_config=None, num_samples_tot=500, init_seed=0, predict=True,
           **kw):
    """run_training (+ run_prediction) of a CI config inside ``workdir`` (logs/ land there)."""
    config = ci_config(mpnn_type, ci_input, workdir, overwrite_config, num_samples_tot, init_seed, **kw)
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        hydragnn_amd.run_training(config)
        return hydragnn_amd.run_prediction(config) if predict else None
    finally:
        os.chdir(cwd)


def _train_once(mpnn_type, global_attn_engine, global_attn_type, ci_input, use_lengths, workdir, overwrite_config,
                num_samples_tot, init_seed):
    torch.manual_seed(int(os.environ.get("HYDRAGNN_TEST_SEED", "97")))
    error, error_task, true_values, pred_values = run_ci(
        mpnn_type, ci_input, workdir, overwrite_config, num_samples_tot, init_seed, use_lengths=use_lengths,
        global_attn_engine=global_attn_engine, global_attn_type=global_attn_type)
    t = thresholds(mpnn_type, ci_input, use_lengths)
    for ih in range(len(true_values)):
        assert float(error_task[ih]) < t[0], f"head {ih} RMSE {float(error_task[ih])} >= {t[0]}"
        mae = torch.nn.functional.l1_loss(pred_values[ih], true_values[ih])
        assert float(mae) < t[1], f"head {ih} MAE {float(mae)} >= {t[1]}"
    assert float(error) < t[0], f"total error {float(error)} >= {t[0]}"
    return float(error)
