"""Model utilities: activations, losses, checkpoints, degree statistics, early
stopping (reference ``hydragnn/utils/model/model.py:29-363``).

Checkpoint layout is kept identical to the reference:
``./logs/<name>/<name>[_epoch_<E>].pk`` holding
``{"model_state_dict", "optimizer_state_dict"}`` with DDP-style ``module.``
prefixed keys; ``<name>.pk`` is a symlink to the newest epoch file.
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from .print_utils import print_master, iterate_tqdm


def activation_function_selection(name: str):
    if name == "relu":
        return torch.nn.ReLU()
    if name == "selu":
        return torch.nn.SELU()
    if name == "prelu":
        return torch.nn.PReLU()
    if name == "elu":
        return torch.nn.ELU()
    if name == "lrelu_01":
        return torch.nn.LeakyReLU(0.1)
    if name == "lrelu_025":
        return torch.nn.LeakyReLU(0.25)
    if name == "lrelu_05":
        return torch.nn.LeakyReLU(0.5)
    if name == "sigmoid":
        return torch.nn.Sigmoid()
    if name in ("silu", "swish"):
        return torch.nn.SiLU()
    if name == "tanh":
        return torch.nn.Tanh()
    raise ValueError(f"unknown activation function {name}")


def _rmse(x, y):
    return torch.sqrt(torch.nn.functional.mse_loss(x, y))


def loss_function_selection(name: str):
    """Same names as the reference; ``smooth_l1`` returns a callable instance (the
    reference returns the class — Appendix D #10) and unknown names raise."""
    if name == "mse":
        return torch.nn.functional.mse_loss
    if name == "mae":
        return torch.nn.functional.l1_loss
    if name == "smooth_l1":
        return torch.nn.SmoothL1Loss()
    if name == "rmse":
        return _rmse
    if name == "GaussianNLLLoss":
        return torch.nn.GaussianNLLLoss()
    raise ValueError(f"unknown loss function {name}")


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def _state_dict_with_prefix(model):
    sd = _unwrap(model).state_dict()
    return {("module." + k if not k.startswith("module.") else k): v for k, v in sd.items()}


def save_model(model, optimizer, name, path="./logs/", use_deepspeed=False):
    """Rank-0 save in the reference ``.pk`` layout (``model.py:63-106``).  A task-parallel
    model (``MultiTaskModelMP``) saves from rank 0 of every branch group instead, so each
    branch checkpoint is written once (reference ``model.py:70-77``)."""
    rank = dist.get_rank() if dist.is_initialized() else 0
    head_pg = getattr(model, "head_pg", None)
    if head_pg is not None and dist.is_initialized():
        rank = dist.get_rank(head_pg)
        suffix = f"_branch{model.branch_id}"
        if not name.endswith(suffix):
            name = name + suffix
    if optimizer is not None and hasattr(optimizer, "consolidate_state_dict"):
        optimizer.consolidate_state_dict()
    if rank != 0:
        return
    d = os.path.join(path, name)
    os.makedirs(d, exist_ok=True)
    state = {"model_state_dict": _state_dict_with_prefix(model)}
    if optimizer is not None:
        state["optimizer_state_dict"] = optimizer.state_dict()
    epoch = os.environ.get("HYDRAGNN_EPOCH")
    fname = os.path.join(d, name + ".pk")
    if epoch is not None:
        efile = os.path.join(d, f"{name}_epoch_{epoch}.pk")
        torch.save(state, efile)
        if os.path.lexists(fname):
            os.remove(fname)
        os.symlink(os.path.basename(efile), fname)
    else:
        if os.path.lexists(fname):
            os.remove(fname)
        torch.save(state, fname)


def load_existing_model(model, model_name, path="./logs/", optimizer=None, use_deepspeed=False):
    """Load ``<path>/<name>/<name>.pk`` (``model.py:128-149``); adds/strips ``module.`` as needed."""
    fname = os.path.join(path, model_name, model_name + ".pk")
    dev = next(_unwrap(model).parameters()).device
    ckpt = torch.load(fname, map_location=dev, weights_only=True)
    sd = ckpt["model_state_dict"]
    target = model if hasattr(model, "module") else None
    if target is None:
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
        model.load_state_dict(sd)
    else:
        sd = {("module." + k if not k.startswith("module.") else k): v for k, v in sd.items()}
        model.load_state_dict(sd)
    if optimizer is not None and "optimizer_state_dict" in ckpt:
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])


def load_existing_model_config(model, config, path="./logs/", optimizer=None, use_deepspeed=False):
    if "continue" in config and config["continue"]:
        model_name = config["startfrom"]
        load_existing_model(model, model_name, path, optimizer, use_deepspeed)


def trainer_state_path(name, path="./logs/"):
    return os.path.join(path, name, name + "_trainer_state.pk")


def save_trainer_state(name, state, path="./logs/"):
    """Sidecar next to the ``.pk`` checkpoint with what the reference does not persist
    (SURVEY §5.4): next epoch, LR-scheduler state, early-stopping counters, RNG states.
    Plain tensors/numbers only, so it loads with ``weights_only=True``."""
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    d = os.path.join(path, name)
    os.makedirs(d, exist_ok=True)
    tmp = trainer_state_path(name, path) + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, trainer_state_path(name, path))


def load_trainer_state(name, path="./logs/"):
    f = trainer_state_path(name, path)
    if not os.path.exists(f):
        return None
    return torch.load(f, map_location="cpu", weights_only=True)


def get_summary_writer(name, path="./logs/"):
    """TensorBoard is not installed: return a JSONL scalar writer with the same add_scalar API."""
    from .metrics import ScalarWriter

    rank = dist.get_rank() if dist.is_initialized() else 0
    return ScalarWriter(os.path.join(path, name)) if rank == 0 else None


def update_multibranch_heads(output_heads):
    """Wrap legacy single-branch head dicts as ``[{"type": "branch-0", "architecture": ...}]``."""
    out = dict(output_heads)
    for name, val in output_heads.items():
        if isinstance(val, list):
            for b in val:
                if not (isinstance(b, dict) and "type" in b and "architecture" in b):
                    raise ValueError(f"output_heads['{name}'] does not contain proper branch config, {val}.")
        elif isinstance(val, dict):
            out[name] = [{"type": "branch-0", "architecture": val}]
        else:
            raise ValueError("Unknown output_heads config!")
    return out


def _degree(edge_index, num_nodes):
    return torch.bincount(edge_index[1].long(), minlength=num_nodes)


def _allreduce_cpu(t, op=None):
    if dist.is_initialized():
        from ..parallel.distributed import comm_reduce

        return comm_reduce(t, op or dist.ReduceOp.SUM)
    return t


def calculate_PNA_degree(loader, max_neighbours):
    """Degree histogram over the dataset (all ranks), capped at max_neighbours."""
    deg = torch.zeros(max_neighbours + 1, dtype=torch.long)
    it = loader.dataset if hasattr(loader, "dataset") else loader
    for data in iterate_tqdm(it, 2, desc="Calculate PNA degree"):
        d = _degree(data.edge_index, data.num_nodes)
        deg += torch.bincount(d, minlength=deg.numel())[: max_neighbours + 1]
    return _allreduce_cpu(deg)


calculate_PNA_degree_dist = calculate_PNA_degree


def calculate_avg_deg(loader):
    deg = torch.zeros(1, dtype=torch.float64)
    counter = torch.zeros(1, dtype=torch.float64)
    it = loader.dataset if hasattr(loader, "dataset") else loader
    for data in iterate_tqdm(it, 2, desc="Calculate avg degree"):
        d = _degree(data.edge_index, data.num_nodes)
        deg += d.sum()
        counter += d.numel()
    deg = _allreduce_cpu(deg)
    counter = _allreduce_cpu(counter)
    return float(deg / counter)


calculate_avg_deg_dist = calculate_avg_deg


def unsorted_segment_mean(data, segment_ids, num_segments):
    from ..ops.segment import scatter_mean_index

    return scatter_mean_index(data, segment_ids, num_segments)


def print_model(model):
    num_params = 0
    for k, v in model.state_dict().items():
        print_master("%50s\t%20s\t%10d" % (k, list(v.shape), v.numel()))
        num_params += v.numel()
    print_master("-" * 50)
    print_master("%50s\t%20s\t%10d" % ("Total", "", num_params))
    print_master("All (total, MB): %d %g" % (num_params, num_params * 4 / 1024 / 1024))


def tensor_divide(x1, x2):
    return torch.from_numpy(np.divide(x1, x2, out=np.zeros_like(x1), where=x2 != 0))


class EarlyStopping:
    def __init__(self, patience=10, min_delta=0.0):
        self.patience = patience
        self.min_delta = min_delta
        self.val_loss_min = float("inf")
        self.count = 0

    def __call__(self, val_loss):
        if val_loss > self.val_loss_min + self.min_delta:
            self.count += 1
            if self.count >= self.patience:
                return True
        else:
            self.val_loss_min = val_loss
            self.count = 0
        return False

    def state_dict(self):
        return {"val_loss_min": self.val_loss_min, "count": self.count}

    def load_state_dict(self, s):
        self.val_loss_min, self.count = s["val_loss_min"], s["count"]


class Checkpoint:
    """Save when the validation metric improves after ``warmup`` epochs (``model.py:323-363``)."""

    def __init__(self, name, warmup=0, path="./logs/", use_deepspeed=False):
        self.count = 1
        self.warmup = warmup
        self.path = path
        self.name = name
        self.min_perf_metric = float("inf")
        self.min_delta = 0
        self.use_deepspeed = use_deepspeed

    def __call__(self, model, optimizer, perf_metric):
        if (perf_metric > self.min_perf_metric + self.min_delta) or (self.count < self.warmup):
            self.count += 1
            return False
        self.min_perf_metric = perf_metric
        save_model(model, optimizer, name=self.name, path=self.path)
        return True
