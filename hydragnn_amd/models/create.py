"""Model factory (reference ``hydragnn/models/create.py:35-519``): same ``mpnn_type``
strings, same config keys, ``torch.manual_seed(0)`` before construction."""
import torch

from ..parallel.distributed import get_device
from ..utils.time_utils import Timer


def create_model_config(config, verbosity=0, use_gpu=True):
    a, t = config["Architecture"], config["Training"]
    return create_model(
        a["mpnn_type"], a["input_dim"], a["hidden_dim"], a["output_dim"], a.get("pe_dim", 0),
        a.get("global_attn_engine"), a.get("global_attn_type"), a.get("global_attn_heads", 0), a["output_type"],
        a["output_heads"], a.get("activation_function", "relu"), t.get("loss_function_type", "mse"),
        a["task_weights"], a["num_conv_layers"], a.get("freeze_conv_layers", False), a.get("initial_bias"),
        a.get("num_nodes"), a.get("max_neighbours"), a.get("edge_dim"), a.get("pna_deg"), a.get("num_before_skip"),
        a.get("num_after_skip"), a.get("num_radial"), a.get("radial_type"), a.get("distance_transform"),
        a.get("basis_emb_size"), a.get("int_emb_size"), a.get("out_emb_size"), a.get("envelope_exponent"),
        a.get("num_spherical"), a.get("num_gaussians"), a.get("num_filters"), a.get("radius"),
        a.get("equivariance", False), a.get("correlation"), a.get("max_ell"), a.get("node_max_ell"),
        a.get("avg_num_neighbors"), t.get("conv_checkpointing", False), verbosity, use_gpu,
        attn_scope=a.get("global_attn_scope", "batch"), dropout=a.get("dropout", 0.25),
        init_seed=a.get("init_seed", 0),
    )


def create_model(mpnn_type, input_dim, hidden_dim, output_dim, pe_dim, global_attn_engine, global_attn_type,
                 global_attn_heads, output_type, output_heads, activation_function, loss_function_type,
                 task_weights, num_conv_layers, freeze_conv=False, initial_bias=None, num_nodes=None,
                 max_neighbours=None, edge_dim=None, pna_deg=None, num_before_skip=None, num_after_skip=None,
                 num_radial=None, radial_type=None, distance_transform=None, basis_emb_size=None, int_emb_size=None,
                 out_emb_size=None, envelope_exponent=None, num_spherical=None, num_gaussians=None, num_filters=None,
                 radius=None, equivariance=False, correlation=None, max_ell=None, node_max_ell=None,
                 avg_num_neighbors=None, conv_checkpointing=False, verbosity=0, use_gpu=True, attn_scope="batch",
                 dropout=0.25, init_seed=0):
    timer = Timer("create_model")
    timer.start()
    torch.manual_seed(init_seed)  # reference seeds 0; "init_seed" is an extension key
    device = get_device(use_gpu, verbosity_level=verbosity)
    common = dict(input_dim=input_dim, hidden_dim=hidden_dim, output_dim=output_dim, pe_dim=pe_dim,
                  global_attn_engine=global_attn_engine, global_attn_type=global_attn_type,
                  global_attn_heads=global_attn_heads, output_type=output_type, config_heads=output_heads,
                  activation_function_type=activation_function, loss_function_type=loss_function_type,
                  equivariance=equivariance, loss_weights=task_weights, freeze_conv=freeze_conv,
                  initial_bias=initial_bias, num_conv_layers=num_conv_layers, num_nodes=num_nodes,
                  attn_scope=attn_scope, dropout=dropout)
    from . import stacks

    if mpnn_type == "GIN":
        model = stacks.GINStack("", "", **common)
    elif mpnn_type == "SAGE":
        model = stacks.SAGEStack("", "", **common)
    elif mpnn_type == "MFC":
        assert max_neighbours is not None, "MFC requires max_neighbours input."
        model = stacks.MFCStack("", "", max_neighbours, **common)
    elif mpnn_type == "PNA":
        assert pna_deg is not None, "PNA requires degree input."
        model = stacks.PNAStack("", "", pna_deg, edge_dim, **common)
    elif mpnn_type == "PNAPlus":
        assert pna_deg is not None, "PNAPlus requires degree input."
        assert envelope_exponent is not None, "PNAPlus requires envelope_exponent input."
        assert num_radial is not None, "PNAPlus requires num_radial input."
        assert radius is not None, "PNAPlus requires radius input."
        model = stacks.PNAPlusStack("", "", pna_deg, edge_dim, envelope_exponent, num_radial, radius, **common)
    elif mpnn_type == "GAT":
        model = stacks.GATStack("", "", heads=6, negative_slope=0.05, edge_dim=edge_dim, **common)
    elif mpnn_type == "CGCNN":
        model = stacks.CGCNNStack("", "", edge_dim, **common)
    elif mpnn_type == "SchNet":
        assert num_gaussians is not None and num_filters is not None and radius is not None, \
            "SchNet requires num_gaussians, num_filters and radius."
        model = stacks.SCFStack("", "", num_filters, edge_dim, num_gaussians, radius,
                                max_neighbours=max_neighbours, **common)
    elif mpnn_type == "DimeNet":
        for k, v in dict(basis_emb_size=basis_emb_size, envelope_exponent=envelope_exponent,
                         int_emb_size=int_emb_size, out_emb_size=out_emb_size, num_after_skip=num_after_skip,
                         num_before_skip=num_before_skip, num_radial=num_radial, num_spherical=num_spherical,
                         radius=radius).items():
            assert v is not None, f"DimeNet requires {k} input."
        model = stacks.DIMEStack("", "", basis_emb_size, envelope_exponent, int_emb_size, out_emb_size,
                                 num_after_skip, num_before_skip, num_radial, num_spherical, edge_dim, radius,
                                 max_neighbours=max_neighbours, **common)
    elif mpnn_type == "EGNN":
        model = stacks.EGCLStack("", "", edge_dim, **common)
    elif mpnn_type == "PAINN":
        assert num_radial is not None and radius is not None, "PAINN requires num_radial and radius."
        model = stacks.PAINNStack("", "", edge_dim, num_radial, radius, **common)
    elif mpnn_type == "PNAEq":
        assert pna_deg is not None and num_radial is not None and radius is not None, \
            "PNAEq requires pna_deg, num_radial and radius."
        model = stacks.PNAEqStack("", "", pna_deg, edge_dim, num_radial, radius, **common)
    elif mpnn_type == "MACE":
        for k, v in dict(radius=radius, num_radial=num_radial, max_ell=max_ell, node_max_ell=node_max_ell,
                         avg_num_neighbors=avg_num_neighbors, envelope_exponent=envelope_exponent).items():
            assert v is not None, f"MACE requires {k} input."
        model = stacks.MACEStack("", "", radius, radial_type, distance_transform, num_radial, edge_dim, max_ell,
                                 node_max_ell, avg_num_neighbors, envelope_exponent, correlation, **common)
    else:
        raise ValueError(f"Unknown mpnn_type: {mpnn_type}")
    if conv_checkpointing:
        model.enable_conv_checkpointing()
    timer.stop()
    return model.to(device)
