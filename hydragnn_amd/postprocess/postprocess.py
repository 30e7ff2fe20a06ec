"""Output denormalisation and node-count unscaling (reference ``postprocess/postprocess.py:13-54``).
Vectorised over tensors instead of per-element Python loops."""
import torch


def output_denormalize(y_minmax, true_values, predicted_values):
    for ih in range(len(y_minmax)):
        ymin, ymax = float(y_minmax[ih][0]), float(y_minmax[ih][1])
        predicted_values[ih] = predicted_values[ih] * (ymax - ymin) + ymin
        true_values[ih] = true_values[ih] * (ymax - ymin) + ymin
    return true_values, predicted_values


def unscale_features_by_num_nodes(datasets_list, scaled_index_list, nodes_num_list):
    n = torch.as_tensor(nodes_num_list, dtype=torch.float32)
    for ds in datasets_list:
        for k in scaled_index_list:
            v = ds[k]
            ds[k] = v * n.to(v.device).view(-1, *([1] * (v.dim() - 1)))[: v.shape[0]]
    return datasets_list


def unscale_features_by_num_nodes_config(config, datasets_list, nodes_num_list):
    var = config["NeuralNetwork"]["Variables_of_interest"]
    idx = [i for i, n in enumerate(var["output_names"]) if "_scaled_num_nodes" in n]
    if idx:
        assert var["denormalize_output"], "Cannot unscale features without 'denormalize_output'"
        datasets_list = unscale_features_by_num_nodes(datasets_list, idx, nodes_num_list)
    return datasets_list
