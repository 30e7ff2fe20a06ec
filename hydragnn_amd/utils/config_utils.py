"""JSON config processing (reference ``utils/input_config_parsing/config_utils.py:25-388``).

Same schema, same defaults and derived keys:
``input_dim``, ``output_dim``/``output_type``/``num_nodes`` (from the first sample's
``y_loc``), ``pna_deg`` + ``max_neighbours`` (PNA family), ``avg_num_neighbors``
(MACE), ``edge_dim`` (from ``edge_features``), ``equivariance`` checks, CGCNN
hidden_dim := input_dim without GPS, ``denormalize_output`` min/max, and the
multibranch ``output_heads`` wrapping.
"""
import copy
import json
import os

import numpy as np
import torch
import torch.distributed as dist

from .model import update_multibranch_heads


def _allreduce(t, op):
    """Cross-rank reduction of a dataset statistic.  ``HYDRAGNN_AGGR_BACKEND`` (reference
    ``graph_samples_checks_and_updates.py:33,436``, ``model.py:194,208``): "torch" (default,
    the process group), "mpi" (host-side reduction: the gloo host group, this framework's
    MPI replacement), anything else: rank-local value (no reduction)."""
    backend = os.getenv("HYDRAGNN_AGGR_BACKEND", "torch")
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1) or \
            backend not in ("torch", "mpi"):
        return t
    if backend == "mpi":
        from ..parallel.distributed import host_group

        h = t.detach().cpu().clone()
        dist.all_reduce(h, op=op, group=host_group())
        return h.to(t.device)
    from ..parallel.distributed import comm_reduce

    return comm_reduce(t, op)


def check_if_graph_size_variable(train_loader, val_loader, test_loader):
    sizes = set()
    for loader in (train_loader, val_loader, test_loader):
        for d in loader.dataset:
            sizes.add(int(d.num_nodes))
            if len(sizes) > 1:
                break
    var = torch.tensor([1 if len(sizes) > 1 else 0])
    return bool(_allreduce(var, dist.ReduceOp.MAX if dist.is_available() else None).item())


def gather_deg(dataset):
    """Global in-degree histogram (``graph_samples_checks_and_updates.py:433-490``)."""
    md = 0
    for d in dataset:
        if d.num_edges:
            md = max(md, int(torch.bincount(d.edge_index[1], minlength=d.num_nodes).max()))
    md = int(_allreduce(torch.tensor([md]), dist.ReduceOp.MAX if dist.is_available() else None).item())
    deg = torch.zeros(md + 1, dtype=torch.long)
    for d in dataset:
        dd = torch.bincount(d.edge_index[1], minlength=d.num_nodes)
        deg += torch.bincount(dd, minlength=md + 1)[: md + 1]
    return _allreduce(deg, dist.ReduceOp.SUM if dist.is_available() else None)


def calculate_avg_deg(dataset):
    s = torch.zeros(1, dtype=torch.float64)
    c = torch.zeros(1, dtype=torch.float64)
    for d in dataset:
        dd = torch.bincount(d.edge_index[1], minlength=d.num_nodes)
        s += dd.sum()
        c += dd.numel()
    s = _allreduce(s, dist.ReduceOp.SUM if dist.is_available() else None)
    c = _allreduce(c, dist.ReduceOp.SUM if dist.is_available() else None)
    return float(s / c)


def update_config(config, train_loader, val_loader, test_loader):
    nn_ = config["NeuralNetwork"]
    arch = nn_["Architecture"]
    env = os.getenv("HYDRAGNN_USE_VARIABLE_GRAPH_SIZE")
    graph_size_variable = bool(int(env)) if env is not None else check_if_graph_size_variable(
        train_loader, val_loader, test_loader)
    if "Dataset" in config:
        check_output_dim_consistent(train_loader.dataset[0], config)
    arch.setdefault("global_attn_engine", None)
    arch.setdefault("global_attn_type", None)
    arch.setdefault("global_attn_heads", 0)
    arch.setdefault("pe_dim", 0)
    arch["output_heads"] = update_multibranch_heads(arch["output_heads"])
    nn_["Training"].setdefault("compute_grad_energy", False)
    config["NeuralNetwork"] = update_config_NN_outputs(nn_, train_loader.dataset[0], graph_size_variable)
    config = normalize_output_config(config)
    nn_ = config["NeuralNetwork"]
    arch = nn_["Architecture"]
    arch["input_dim"] = len(nn_["Variables_of_interest"]["input_node_features"])
    if arch["mpnn_type"] in ("PNA", "PNAPlus", "PNAEq"):
        if hasattr(train_loader.dataset, "pna_deg"):
            deg = torch.as_tensor(train_loader.dataset.pna_deg)
        else:
            deg = gather_deg(train_loader.dataset)
        arch["pna_deg"] = deg.tolist()
        arch["max_neighbours"] = len(deg) - 1
    else:
        arch["pna_deg"] = None
    if arch["mpnn_type"] == "CGCNN" and not arch["global_attn_engine"]:
        arch["hidden_dim"] = arch["input_dim"]
    if arch["mpnn_type"] == "MACE":
        if hasattr(train_loader.dataset, "avg_num_neighbors"):
            arch["avg_num_neighbors"] = float(train_loader.dataset.avg_num_neighbors)
        else:
            arch["avg_num_neighbors"] = calculate_avg_deg(train_loader.dataset)
    else:
        arch["avg_num_neighbors"] = None
    for k in ("radius", "radial_type", "distance_transform", "num_gaussians", "num_filters", "envelope_exponent",
              "num_after_skip", "num_before_skip", "basis_emb_size", "int_emb_size", "out_emb_size", "num_radial",
              "num_spherical", "correlation", "max_ell", "node_max_ell"):
        arch.setdefault(k, None)
    arch = update_config_edge_dim(arch)
    arch = update_config_equivariance(arch)
    arch.setdefault("freeze_conv_layers", False)
    arch.setdefault("initial_bias", None)
    arch.setdefault("activation_function", "relu")
    arch.setdefault("SyncBatchNorm", False)
    nn_["Architecture"] = arch
    tr = nn_["Training"]
    tr.setdefault("conv_checkpointing", False)
    tr.setdefault("loss_function_type", "mse")
    tr.setdefault("Optimizer", {"type": "AdamW"})
    tr["Optimizer"].setdefault("type", "AdamW")
    return config


def update_config_equivariance(arch):
    models = ("EGNN", "SchNet", "PNAEq", "PAINN", "MACE")
    if arch.get("equivariance"):
        assert arch["mpnn_type"] in models, \
            "E(3) equivariance can only be ensured for EGNN, SchNet, PNAEq, PAINN, and MACE."
    else:
        arch["equivariance"] = False
    return arch


def update_config_edge_dim(arch):
    arch["edge_dim"] = None
    edge_models = ("GAT", "PNA", "PNAPlus", "PAINN", "PNAEq", "CGCNN", "SchNet", "EGNN", "DimeNet", "MACE")
    if arch.get("edge_features"):
        assert arch["mpnn_type"] in edge_models, \
            "Edge features can only be used with GAT, PNA, PNAPlus, PAINN, PNAEq, CGCNN, SchNet, EGNN, DimeNet, MACE."
        arch["edge_dim"] = len(arch["edge_features"])
    elif arch["mpnn_type"] == "CGCNN":
        arch["edge_dim"] = 0
    return arch


def check_output_dim_consistent(data, config):
    var = config["NeuralNetwork"]["Variables_of_interest"]
    ot, oi = var["type"], var["output_index"]
    yl = data.get("y_loc")
    if yl is None:
        return
    ds = config["Dataset"]
    for ih in range(len(ot)):
        span = int(yl[0, ih + 1] - yl[0, ih])
        if ot[ih] == "graph":
            assert span == ds["graph_features"]["dim"][oi[ih]]
        elif ot[ih] == "node":
            assert span // data.num_nodes == ds["node_features"]["dim"][oi[ih]]


def update_config_NN_outputs(nn_, data, graph_size_variable):
    var = nn_["Variables_of_interest"]
    ot = var["type"]
    yl = data.get("y_loc")
    if nn_["Training"]["compute_grad_energy"]:
        dims = var["output_dim"]
    elif yl is not None:
        dims = []
        for ih, t in enumerate(ot):
            span = int(yl[0, ih + 1] - yl[0, ih])
            if t == "graph":
                dims.append(span)
            elif t == "node":
                heads = nn_["Architecture"]["output_heads"]
                if graph_size_variable and heads["node"][0]["architecture"]["type"] == "mlp_per_node":
                    raise ValueError('"mlp_per_node" is not allowed for variable graph size, Please set '
                                     'config["NeuralNetwork"]["Architecture"]["output_heads"]["node"]["type"] to be '
                                     '"mlp" or "conv" in input file.')
                dims.append(span // data.num_nodes)
            else:
                raise ValueError("Unknown output type", t)
    else:
        for t in ot:
            if t != "graph":
                raise ValueError("y_loc is needed for outputs that are not at graph levels", t)
        dims = var["output_dim"]
    nn_["Architecture"]["output_dim"] = dims
    nn_["Architecture"]["output_type"] = ot
    nn_["Architecture"]["num_nodes"] = data.num_nodes
    return nn_


def normalize_output_config(config):
    var = config["NeuralNetwork"]["Variables_of_interest"]
    if var.get("denormalize_output"):
        if var.get("minmax_node_feature") is not None and var.get("minmax_graph_feature") is not None:
            path = None
        elif list(config["Dataset"]["path"].values())[0].endswith(".pkl"):
            path = list(config["Dataset"]["path"].values())[0]
        else:
            base = os.environ.get("SERIALIZED_DATA_PATH", os.getcwd())
            name = config["Dataset"]["name"]
            path = (f"{base}/serialized_dataset/{name}.pkl" if "total" in config["Dataset"]["path"]
                    else f"{base}/serialized_dataset/{name}_train.pkl")
        var = update_config_minmax(path, var)
    else:
        var["denormalize_output"] = False
    config["NeuralNetwork"]["Variables_of_interest"] = var
    return config


def update_config_minmax(dataset_path, var):
    if "minmax_node_feature" not in var and "minmax_graph_feature" not in var:
        from ..data.serialized import read_serialized

        node_mm, graph_mm, _ = read_serialized(dataset_path)
    else:
        node_mm = np.asarray(var["minmax_node_feature"])
        graph_mm = np.asarray(var["minmax_graph_feature"])
    var["x_minmax"] = [node_mm[:, i].tolist() for i in var["input_node_features"]]
    var["y_minmax"] = []
    for ih, t in enumerate(var["type"]):
        idx = var["output_index"][ih]
        if t == "graph":
            var["y_minmax"].append(graph_mm[:, idx].tolist())
        elif t == "node":
            var["y_minmax"].append(node_mm[:, idx].tolist())
        else:
            raise ValueError("Unknown output type", t)
    return var


def get_log_name_config(config):
    a = config["NeuralNetwork"]["Architecture"]
    t = config["NeuralNetwork"]["Training"]
    name = config["Dataset"]["name"]
    cut = name.rfind("_")
    return (a["mpnn_type"] + "-r-" + str(a.get("radius")) + "-ncl-" + str(a["num_conv_layers"]) + "-hd-"
            + str(a["hidden_dim"]) + "-ne-" + str(t["num_epoch"]) + "-lr-" + str(t["Optimizer"]["learning_rate"])
            + "-bs-" + str(t["batch_size"]) + "-data-" + name[: (cut if cut > 0 else None)] + "-node_ft-"
            + "".join(str(x) for x in config["NeuralNetwork"]["Variables_of_interest"]["input_node_features"])
            + "-task_weights-" + "".join(str(w) + "-" for w in a["task_weights"]))


def save_config(config, log_name, path="./logs/"):
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    if rank == 0:
        os.makedirs(os.path.join(path, log_name), exist_ok=True)
        with open(os.path.join(path, log_name, "config.json"), "w") as f:
            json.dump(config, f, indent=4, default=_json_default)


def _json_default(o):
    if torch.is_tensor(o):
        return o.tolist()
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    raise TypeError(type(o))


def parse_deepspeed_config(config):
    """DeepSpeed is not part of this framework; kept for config compatibility."""
    ds = dict(config["NeuralNetwork"].get("ds_config", {}))
    if "train_micro_batch_size_per_gpu" not in ds:
        ds["train_micro_batch_size_per_gpu"] = config["NeuralNetwork"]["Training"]["batch_size"]
        ds["gradient_accumulation_steps"] = 1
    ds.setdefault("steps_per_print", 1e9)
    return ds


def merge_config(a, b):
    result = copy.deepcopy(a)
    for k, v in b.items():
        av = result.get(k)
        if isinstance(av, dict) and isinstance(v, dict):
            result[k] = merge_config(av, v)
        else:
            result[k] = copy.deepcopy(v)
    return result


def merge_pna_deg(deg_list):
    """Merge per-dataset PNA in-degree histograms of different lengths into one (reference
    ``examples/multidataset/train.py:214-232``, multi-dataset setup C21): each histogram is
    resampled onto the shortest length with a cubic interpolating spline over [0, 1] and the
    resampled histograms are summed (truncated to int64)."""
    from scipy.interpolate import make_interp_spline

    degs = [np.asarray(d, dtype=np.float64) for d in deg_list if d is not None]
    assert degs, "merge_pna_deg: no histograms"
    mlen = min(len(d) for d in degs)
    out = np.zeros(mlen)
    grid = np.linspace(0, 1, num=mlen)
    for d in degs:
        k = min(3, len(d) - 1)
        out += make_interp_spline(np.linspace(0, 1, num=len(d)), d, k=k)(grid) if k > 0 else d[:mlen]
    return out.astype(np.int64).tolist()


def proportional_process_list(ndata_list, world_size):
    """Ranks per dataset in proportion to dataset sizes (ceil, then the largest share gives
    back the excess) — the reference's multidataset rank assignment (``train.py:206-212``)."""
    nd = np.asarray(ndata_list, dtype=np.float64)
    pl = np.ceil(nd / nd.sum() * world_size).astype(np.int64)
    imax = int(np.argmax(pl))
    pl[imax] -= int(pl.sum()) - world_size
    assert pl.min() >= 1, f"not enough ranks ({world_size}) for {len(nd)} datasets"
    return pl.tolist()
