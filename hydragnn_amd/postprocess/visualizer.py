"""Result plots (reference ``postprocess/visualizer.py:24-742``): parity scatter plots per
head, global error analysis, error histograms, per-node vector parity, loss history and
the graph-size histogram.  matplotlib (Agg backend) only; PNG files under
``./logs/<model_name>/``."""
import os

import numpy as np


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def _np(v):
    import torch

    if torch.is_tensor(v):
        return v.detach().float().cpu().numpy()
    return np.asarray(v, dtype=np.float64)


class Visualizer:
    def __init__(self, model_with_config_name, node_feature=None, num_heads=1, head_dims=(1,), num_nodes_list=None):
        self.name = model_with_config_name
        self.dir = os.path.join("./logs", model_with_config_name)
        os.makedirs(self.dir, exist_ok=True)
        self.node_feature = np.asarray(node_feature) if node_feature is not None else None
        self.num_heads = num_heads
        self.head_dims = list(head_dims)
        self.num_nodes_list = list(num_nodes_list or [])

    @staticmethod
    def _names(output_names, n):
        return list(output_names) if output_names else [f"head{i}" for i in range(n)]

    def _parity(self, ax, t, p, title):
        ax.scatter(t, p, s=4, alpha=0.6, edgecolor="none")
        lo = float(min(t.min(), p.min())) if t.size else 0.0
        hi = float(max(t.max(), p.max())) if t.size else 1.0
        ax.plot([lo, hi], [lo, hi], "k--", lw=0.8)
        mae = float(np.mean(np.abs(t - p))) if t.size else 0.0
        ax.set_title(f"{title}  MAE={mae:.4f}")
        ax.set_xlabel("True")
        ax.set_ylabel("Predicted")

    def create_scatter_plots(self, true_values, predicted_values, output_names=None, iepoch=None):
        if not true_values or len(true_values[0]) == 0:
            return
        plt = _plt()
        names = self._names(output_names, len(true_values))
        fig, axs = plt.subplots(1, len(true_values), figsize=(4.5 * len(true_values), 4), squeeze=False)
        for ih in range(len(true_values)):
            self._parity(axs[0, ih], _np(true_values[ih]).ravel(), _np(predicted_values[ih]).ravel(), names[ih])
        suffix = "" if iepoch is None else (f"_{iepoch}" if iepoch >= 0 else "_init")
        fig.tight_layout()
        fig.savefig(os.path.join(self.dir, f"scatter{suffix}.png"), dpi=100)
        plt.close(fig)

    def create_plot_global(self, true_values, predicted_values, output_names=None):
        if not true_values or len(true_values[0]) == 0:
            return
        plt = _plt()
        names = self._names(output_names, len(true_values))
        for ih in range(len(true_values)):
            t, p = _np(true_values[ih]).ravel(), _np(predicted_values[ih]).ravel()
            fig, axs = plt.subplots(1, 3, figsize=(13, 4))
            self._parity(axs[0], t, p, names[ih])
            err = p - t
            axs[1].hist(err, bins=50)
            axs[1].set_title("error histogram")
            order = np.argsort(t)
            axs[2].plot(t[order], np.abs(err[order]), ".", ms=2)
            axs[2].set_title("|error| vs true")
            fig.tight_layout()
            fig.savefig(os.path.join(self.dir, f"global_{names[ih]}.png"), dpi=100)
            plt.close(fig)

    create_plot_global_analysis = create_plot_global

    def create_parity_plot_vector(self, varname, true_values, predicted_values, head_dim, iepoch=None):
        plt = _plt()
        t = _np(true_values).reshape(-1, head_dim)
        p = _np(predicted_values).reshape(-1, head_dim)
        fig, axs = plt.subplots(1, head_dim, figsize=(4 * head_dim, 4), squeeze=False)
        for k in range(head_dim):
            self._parity(axs[0, k], t[:, k], p[:, k], f"{varname}[{k}]")
        fig.tight_layout()
        fig.savefig(os.path.join(self.dir, f"parity_vector_{varname}.png"), dpi=100)
        plt.close(fig)

    def plot_history(self, total_loss_train, total_loss_val, total_loss_test, task_loss_train, task_loss_val,
                     task_loss_test, task_weights, task_names):
        plt = _plt()
        tl = [_np(x) for x in (total_loss_train, total_loss_val, total_loss_test)]
        ntask = _np(task_loss_train).shape[1] if _np(task_loss_train).ndim == 2 else 0
        fig, axs = plt.subplots(1, 1 + ntask, figsize=(4.5 * (1 + ntask), 4), squeeze=False)
        for v, lab in zip(tl, ("train", "validate", "test")):
            axs[0, 0].plot(v, label=lab)
        axs[0, 0].set_yscale("log")
        axs[0, 0].legend()
        axs[0, 0].set_title("total loss")
        names = self._names(task_names, ntask)
        for k in range(ntask):
            for v, lab in zip((task_loss_train, task_loss_val, task_loss_test), ("train", "validate", "test")):
                axs[0, 1 + k].plot(_np(v)[:, k], label=lab)
            axs[0, 1 + k].set_yscale("log")
            axs[0, 1 + k].set_title(f"{names[k]} (w={task_weights[k]:.3g})")
        fig.tight_layout()
        fig.savefig(os.path.join(self.dir, "history_loss.png"), dpi=100)
        plt.close(fig)
        np.savez(os.path.join(self.dir, "history_loss.npz"), *tl)

    def num_nodes_plot(self):
        if not self.num_nodes_list:
            return
        plt = _plt()
        fig, ax = plt.subplots(figsize=(4, 3))
        ax.hist(self.num_nodes_list, bins=min(50, max(5, len(set(self.num_nodes_list)))))
        ax.set_title("number of nodes per graph")
        fig.tight_layout()
        fig.savefig(os.path.join(self.dir, "num_nodes.png"), dpi=100)
        plt.close(fig)
