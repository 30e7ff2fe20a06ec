"""Serialized dataset files and the per-sample preprocessing pipeline.

File format (our own; loadable with ``torch.load(weights_only=True)``):
``{"minmax_node_feature": Tensor[2, Fn], "minmax_graph_feature": Tensor[2, Fg],
"samples": [ {key: Tensor, ...}, ... ]}``.  File names follow the reference
(``serialized_dataset/<name>[_<split>].pkl``) so configs that point at them
keep working.

``SerializedDataLoader.load_serialized_data`` reproduces
``preprocess/serialized_dataset_loader.py:110-212``: optional rotation
normalisation -> radius graph (PBC or not, ``max_neighbours`` cap) -> edge
length (``Distance``) normalised by the max length over the split (all ranks)
-> optional spherical / point-pair descriptors -> Laplacian eigenvector PE
(``pe_dim``) and ``rel_pe`` -> target packing (``y``/``y_loc``) and input feature
column selection.
"""
import os

import numpy as np
import torch

from .graph import Graph
from . import transforms as T


def write_serialized(path, samples, minmax_node=None, minmax_graph=None):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    payload = {
        "minmax_node_feature": torch.as_tensor(np.asarray(minmax_node if minmax_node is not None else np.zeros((2, 0))),
                                               dtype=torch.float64),
        "minmax_graph_feature": torch.as_tensor(
            np.asarray(minmax_graph if minmax_graph is not None else np.zeros((2, 0))), dtype=torch.float64),
        "samples": [{k: v for k, v in s.items() if torch.is_tensor(v)} for s in samples],
    }
    torch.save(payload, path)


def read_serialized(path):
    d = torch.load(path, map_location="cpu", weights_only=True)
    samples = [Graph(**s) for s in d["samples"]]
    return d["minmax_node_feature"].numpy(), d["minmax_graph_feature"].numpy(), samples


def update_predicted_values(types, index, graph_feature_dim, node_feature_dim, data):
    """Pack the selected targets into ``data.y`` [total, 1] with offsets ``data.y_loc``
    (``graph_samples_checks_and_updates.py:493-534``)."""
    out = []
    y_loc = torch.zeros(1, len(types) + 1, dtype=torch.int64)
    for item, t in enumerate(types):
        if t == "graph":
            s = sum(graph_feature_dim[:index[item]])
            feat = data.y.reshape(-1)[s:s + graph_feature_dim[index[item]]].reshape(-1, 1)
        elif t == "node":
            s = sum(node_feature_dim[:index[item]])
            feat = data.x[:, s:s + node_feature_dim[index[item]]].reshape(-1, 1)
        else:
            raise ValueError("Unknown output type", t)
        out.append(feat)
        y_loc[0, item + 1] = y_loc[0, item] + feat.shape[0] * feat.shape[1]
    data.y = torch.cat(out, 0).to(torch.float32)
    data.y_loc = y_loc


def update_atom_features(atom_features, data):
    data.x = data.x[:, list(atom_features)]


class SerializedDataLoader:
    def __init__(self, config, dist=False):
        ds = config["Dataset"]
        arch = config["NeuralNetwork"]["Architecture"]
        var = config["NeuralNetwork"]["Variables_of_interest"]
        self.verbosity = config.get("Verbosity", {}).get("level", 0)
        self.node_feature_dim = ds["node_features"]["dim"]
        self.graph_feature_dim = ds["graph_features"]["dim"]
        self.rotational_invariance = ds.get("rotational_invariance", False)
        self.pbc = arch.get("periodic_boundary_conditions", False)
        self.radius = arch["radius"]
        self.max_neighbours = arch["max_neighbours"]
        self.variables = var
        self.types = var["type"]
        self.output_index = var["output_index"]
        self.input_node_features = var["input_node_features"]
        desc = ds.get("Descriptors", {})
        self.spherical = desc.get("SphericalCoordinates", False)
        self.ppf = desc.get("PointPairFeatures", False)
        self.pe_dim = arch.get("pe_dim", 0) or 0
        self.dist = dist

    def load_serialized_data(self, dataset_path):
        _, _, dataset = read_serialized(dataset_path)
        return self.process(dataset)

    def process(self, dataset):
        import torch.distributed as dist

        gpu_graphs = None
        if torch.cuda.is_available() and dataset and os.environ.get("HYDRAGNN_GPU_PREPROCESS", "1") == "1" and \
                (not self.pbc or all(d.get("pbc") is None or bool(torch.as_tensor(d.pbc).all()) for d in dataset)):
            if self.rotational_invariance:
                for d in dataset:
                    d.pos = T.normalize_rotation(d.pos).to(torch.float32)
            gpu_graphs = T.build_radius_graphs_gpu(dataset, self.radius, self.max_neighbours, pbc=self.pbc)
        for gi, d in enumerate(dataset):
            if gpu_graphs is not None:
                d.edge_index, sh = gpu_graphs[gi]
                if sh is not None:
                    d.edge_shifts = sh
                d.edge_attr = T.distance(d.pos, d.edge_index, shifts=sh, norm=False)
                continue
            if self.rotational_invariance:
                d.pos = T.normalize_rotation(d.pos).to(torch.float32)
            if self.pbc:
                cell = d.get("cell")
                assert cell is not None, "periodic_boundary_conditions requires data.cell"
                ei, sh, _ = T.radius_graph_pbc_robust(d.pos, cell, d.get("pbc", [True, True, True]),
                                                      self.radius, self.max_neighbours)
                d.edge_index, d.edge_shifts = ei, sh
                d.edge_attr = T.distance(d.pos, ei, shifts=sh, norm=False)
            else:
                d.edge_index = T.radius_graph(d.pos, self.radius, max_num_neighbors=self.max_neighbours)
                d.edge_attr = T.distance(d.pos, d.edge_index, norm=False)
        mx = max([float(d.edge_attr.max()) for d in dataset if d.edge_attr.numel()] + [float("-inf")])
        if self.dist and dist.is_initialized():
            from ..parallel.distributed import comm_reduce

            mx = float(comm_reduce(torch.tensor([mx], dtype=torch.float64), dist.ReduceOp.MAX)[0])
        pes = None
        if self.pe_dim:  # all Laplacians in one batched launch on the GPU (HIP Jacobi), host otherwise
            pes = T.laplacian_pe_batch(dataset, self.pe_dim, device="cuda" if torch.cuda.is_available() else None)
        for i, d in enumerate(dataset):
            d.edge_attr = (d.edge_attr / mx).to(torch.float32)
            if self.spherical:
                d.edge_attr = torch.cat([d.edge_attr, T.spherical(d.pos, d.edge_index)], -1)
            if self.ppf and d.get("normal") is not None:
                d.edge_attr = torch.cat([d.edge_attr, T.point_pair_features(d.pos, d.normal, d.edge_index)], -1)
            if self.pe_dim:
                d.pe = pes[i]
                d.rel_pe = T.relative_pe(d.pe, d.edge_index)
            update_predicted_values(self.types, self.output_index, self.graph_feature_dim, self.node_feature_dim, d)
            update_atom_features(self.input_node_features, d)
            d.sort_edges_by_dst()
        if "subsample_percentage" in self.variables:
            from .splitting import stratified_subsample

            dataset = stratified_subsample(dataset, self.variables["subsample_percentage"])
        return dataset
