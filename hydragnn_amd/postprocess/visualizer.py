"""Result plots (reference ``postprocess/visualizer.py:24-742``).

Same plot families and file names as the reference, written vectorised (numpy over
the whole sample set instead of per-sample Python loops):

* ``create_scatter_plots``        - per head: parity + error PDF (scalar heads) or the
                                    per-node / per-component parity grid (ref :692-720)
* ``create_plot_global`` /
  ``create_plot_global_analysis`` - scatter / conditional-mean abs. error / error PDF;
                                    vector heads get the 3x3 length / sum / component
                                    panel (ref :134-279, :722-732)
* ``create_parity_plot_and_error_histogram_scalar`` (ref :281-385)
* ``create_error_histogram_per_node``               (ref :387-465)
* ``create_parity_plot_vector``                      (ref :467-516)
* ``create_parity_plot_per_node_vector``             (ref :519-612)
* ``plot_history`` (loss curves + ``history_loss.npz``; no pickle) (ref :629-690)
* ``num_nodes_plot``                                  (ref :734-742)

matplotlib with the Agg backend; PNGs under ``./logs/<model_name>/``.
"""
import math
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
        return v.detach().double().cpu().numpy()
    if isinstance(v, (list, tuple)) and v and all(torch.is_tensor(x) for x in v):
        return np.stack([x.detach().double().cpu().numpy() for x in v])
    return np.asarray(v, dtype=np.float64)


def _as_2d(v):
    a = _np(v)
    return a.reshape(a.shape[0], -1) if a.ndim != 2 else a


def _grid(n):
    nrow = max(1, int(math.floor(math.sqrt(n))))
    return nrow, int(math.ceil(n / nrow))


def _rng(a):
    """Histogram range that always admits finite bins (degenerate / near-constant data)."""
    lo, hi = float(np.min(a)), float(np.max(a))
    if not hi - lo > 1e-9 * max(1.0, abs(lo), abs(hi)):
        lo, hi = lo - 0.5, hi + 0.5
    return lo, hi


def hist2d_contour(x, y, bins=50):
    """Normalised 2-D histogram on bin centres (ref ``__hist2d_contour``)."""
    x, y = np.ravel(x), np.ravel(y)
    h, xe, ye = np.histogram2d(x, y, bins=bins, range=[_rng(x), _rng(y)])
    xc, yc = 0.5 * (xe[:-1] + xe[1:]), 0.5 * (ye[:-1] + ye[1:])
    gy, gx = np.meshgrid(yc, xc)
    return gx, gy, h / max(h.max(), 1e-300)


def err_condmean(true, pred, weight=1.0, bins=50):
    """Mean absolute error conditioned on the true value, from a 2-D histogram of
    (true, |err|) (ref ``__err_condmean``).  Returns (true bin centres, mean |err|)."""
    t = np.ravel(true)
    e = np.abs(t - np.ravel(pred)) * weight
    h, xe, ye = np.histogram2d(t, e, bins=bins, range=[_rng(t), _rng(e)])
    h = h / max(h.max(), 1e-300)
    yc = 0.5 * (ye[:-1] + ye[1:])
    return 0.5 * (xe[:-1] + xe[1:]), h @ yc / (h.sum(axis=1) + 1e-12)


def error_pdf(true, pred, bins=40):
    """Density histogram of pred - true on bin centres."""
    d = np.ravel(pred) - np.ravel(true)
    if d.size == 0:
        return np.zeros(0), np.zeros(0)
    h, be = np.histogram(d, bins=bins, range=_rng(d), density=True)
    return 0.5 * (be[:-1] + be[1:]), h


class Visualizer:
    def __init__(self, model_with_config_name, node_feature=None, num_heads=1, head_dims=(1,), num_nodes_list=None):
        self.model_with_config_name = model_with_config_name
        self.name = model_with_config_name
        self.dir = os.path.join("./logs", model_with_config_name)
        os.makedirs(self.dir, exist_ok=True)
        self.node_feature = None if node_feature is None else _as_2d(node_feature)
        self.num_heads = num_heads
        self.head_dims = list(head_dims)
        self.num_nodes_list = list(num_nodes_list or [])

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _names(output_names, n):
        return list(output_names) if output_names else [f"head{i}" for i in range(n)]

    def _path(self, stem, iepoch=None):
        if iepoch is None:
            return os.path.join(self.dir, f"{stem}.png")
        tag = str(iepoch).zfill(4) if iepoch >= 0 else "init"
        return os.path.join(self.dir, f"{stem}_{tag}.png")

    def _feature(self, nsamp, ncol):
        """Per-(sample, node) colour values; zeros when no node feature was given or
        its shape does not line up with the predictions."""
        f = self.node_feature
        if f is None or f.shape[0] != nsamp or f.shape[1] < ncol:
            return np.zeros((nsamp, ncol))
        return f[:, :ncol]

    @staticmethod
    def add_identity(ax, *line_args, **line_kwargs):
        """y = x over the overlap of the current axis ranges, kept in sync on zoom."""
        (line,) = ax.plot([], [], *line_args, **line_kwargs)

        def cb(a):
            lo = max(a.get_xlim()[0], a.get_ylim()[0])
            hi = min(a.get_xlim()[1], a.get_ylim()[1])
            line.set_data([lo, hi], [lo, hi])

        cb(ax)
        ax.callbacks.connect("xlim_changed", cb)
        ax.callbacks.connect("ylim_changed", cb)
        return ax

    def _scatter(self, ax, x, y, s=None, c=None, marker=None, title="", xlabel="True", ylabel="Predicted",
                 equal=True):
        x, y = np.ravel(x), np.ravel(y)
        if c is not None and np.size(c) == x.size and np.ptp(np.ravel(c)) > 0:
            ax.scatter(x, y, s=s, c=np.ravel(c), marker=marker, cmap="viridis")
        else:
            ax.scatter(x, y, s=s, edgecolor="b", marker=marker, facecolor="none")
        mae = float(np.mean(np.abs(x - y))) if x.size else 0.0
        ax.set_title(f"{title}, number of samples ={x.size}, MAE={mae:.4g}")
        ax.set_xlabel(xlabel)
        ax.set_ylabel(ylabel)
        if equal and x.size:
            ax.set_aspect("equal")
            lo = min(ax.get_xlim()[0], ax.get_ylim()[0])
            hi = max(ax.get_xlim()[1], ax.get_ylim()[1])
            ax.set_xlim(lo, hi)
            ax.set_ylim(lo, hi)
        self.add_identity(ax, color="r", ls="--")

    def _save(self, fig, path, save_plot=True):
        plt = _plt()
        if save_plot:
            fig.savefig(path, dpi=100)
            plt.close(fig)
        else:
            plt.show()

    # ------------------------------------------------------------------ global analysis
    def create_plot_global_analysis(self, varname, true_values, predicted_values, save_plot=True):
        """Scalar heads: scatter / conditional-mean |err| / error PDF.  Vector heads: the same
        three rows for the vector length, the component sum and the raw components."""
        plt = _plt()
        t, p = _as_2d(true_values), _as_2d(predicted_values)
        if t.shape[1] == 1:
            fig, axs = plt.subplots(1, 3, figsize=(15, 4.5))
            self._scatter(axs[0], t, p, title="Scalar output")
            xc, me = err_condmean(t, p)
            axs[1].plot(xc, me, "ro")
            axs[1].set_title("Conditional mean abs. error")
            axs[1].set_xlabel("True")
            axs[1].set_ylabel("abs. error")
            xc, h = error_pdf(t, p)
            axs[2].plot(xc, h, "ro")
            axs[2].set_title("Scalar output: error PDF")
            axs[2].set_xlabel("Error")
            axs[2].set_ylabel("PDF")
        else:
            k = t.shape[1]
            fig, axs = plt.subplots(3, 3, figsize=(18, 16))
            cols = [
                ("length", np.linalg.norm(t, axis=1), np.linalg.norm(p, axis=1), 1.0 / math.sqrt(k)),
                ("sum", t.sum(1), p.sum(1), 1.0 / k),
                ("components", t.ravel(), p.ravel(), 1.0),
            ]
            for j, (nm, a, b, w) in enumerate(cols):
                self._scatter(axs[0, j], a, b, title=f"Vector output: {nm}")
                xc, me = err_condmean(a, b, weight=w)
                axs[1, j].plot(xc, me, "ro")
                axs[1, j].set_ylabel("Conditional mean abs error")
                axs[1, j].set_xlabel("True")
                xc, h = error_pdf(a, b)
                axs[2, j].plot(xc, h, "ro")
                axs[2, j].set_ylabel("Error PDF")
                axs[2, j].set_xlabel("Error")
        fig.tight_layout()
        self._save(fig, os.path.join(self.dir, f"{varname}_scatter_condm_err.png"), save_plot)

    def create_plot_global(self, true_values, predicted_values, output_names=None):
        if not true_values or len(true_values[0]) == 0:
            return
        names = self._names(output_names, len(true_values))
        for ih in range(len(true_values)):
            t, p = _np(true_values[ih]), _np(predicted_values[ih])
            dim = self.head_dims[ih] if ih < len(self.head_dims) else 1
            self.create_plot_global_analysis(names[ih], t.reshape(-1, dim), p.reshape(-1, dim))

    # ------------------------------------------------------------------ parity + histograms
    def create_parity_plot_and_error_histogram_scalar(self, varname, true_values, predicted_values, iepoch=None,
                                                      save_plot=True):
        """[nsamp, 1]: parity + error PDF.  [nsamp, nnode]: one parity panel per node
        (coloured by the node feature), plus the per-sample node SUM and the per-node
        sample sum (ref SMP_Mean4sites)."""
        plt = _plt()
        t, p = _as_2d(true_values), _as_2d(predicted_values)
        ns, nn = t.shape
        if nn == 1:
            fig, axs = plt.subplots(1, 2, figsize=(12, 6))
            self._scatter(axs[0], t, p, title=varname)
            xc, h = error_pdf(t, p)
            axs[1].plot(xc, h, "ro")
            axs[1].set_title(f"{varname}: error PDF")
        else:
            f = self._feature(ns, nn)
            nrow, ncol = _grid(nn + 2)
            fig, axs = plt.subplots(nrow, ncol, figsize=(ncol * 3, nrow * 3), squeeze=False)
            axs = axs.ravel()
            for i in range(nn):
                self._scatter(axs[i], t[:, i], p[:, i], s=6, c=f[:, i], title=f"node:{i}")
            self._scatter(axs[nn], t.sum(1), p.sum(1), s=40, c=f.sum(1), title="SUM")
            self._scatter(axs[nn + 1], t.sum(0), p.sum(0), s=40, c=f.sum(0), title=f"SMP_Mean4sites:0-{nn}")
            for ax in axs[nn + 2:]:
                ax.axis("off")
        fig.tight_layout()
        self._save(fig, self._path(varname, iepoch), save_plot)

    def create_error_histogram_per_node(self, varname, true_values, predicted_values, iepoch=None, save_plot=True):
        t, p = _as_2d(true_values), _as_2d(predicted_values)
        nn = t.shape[1]
        if nn == 1:
            return
        plt = _plt()
        nrow, ncol = _grid(nn + 2)
        fig, axs = plt.subplots(nrow, ncol, figsize=(ncol * 3.5, nrow * 3.2), squeeze=False)
        axs = axs.ravel()
        panels = [(t[:, i], p[:, i], f"node:{i}") for i in range(nn)]
        panels += [(t.sum(1), p.sum(1), "SUM"), (t.sum(0), p.sum(0), f"SMP_Mean4sites:0-{nn}")]
        for ax, (a, b, title) in zip(axs, panels):
            xc, h = error_pdf(a, b)
            ax.plot(xc, h, "ro")
            ax.set_title(title)
        for ax in axs[nn + 2:]:
            ax.axis("off")
        fig.tight_layout()
        self._save(fig, self._path(f"{varname}_error_hist1d", iepoch), save_plot)

    def create_parity_plot_vector(self, varname, true_values, predicted_values, head_dim, iepoch=None,
                                  save_plot=True):
        plt = _plt()
        t = _np(true_values).reshape(-1, head_dim)
        p = _np(predicted_values).reshape(-1, head_dim)
        markers = ["o", "s", "d"]
        nrow, ncol = _grid(head_dim)
        fig, axs = plt.subplots(nrow, ncol, figsize=(ncol * 4, nrow * 4), squeeze=False)
        axs = axs.ravel()
        for k in range(head_dim):
            self._scatter(axs[k], t[:, k], p[:, k], s=6, marker=markers[k % 3], title=f"comp:{k}")
        for ax in axs[head_dim:]:
            ax.axis("off")
        fig.tight_layout()
        self._save(fig, self._path(varname, iepoch), save_plot)

    def create_parity_plot_per_node_vector(self, varname, true_values, predicted_values, iepoch=None, save_plot=True):
        """[nsamp, nnode*3] 3-vectors: per-node parity (one marker per component), the
        per-sample node sum and the per-node sample sum."""
        plt = _plt()
        t, p = _as_2d(true_values), _as_2d(predicted_values)
        ns = t.shape[0]
        t, p = t.reshape(ns, -1, 3), p.reshape(ns, -1, 3)
        nn = t.shape[1]
        f = self._feature(ns, nn)
        markers = ["o", "s", "d"]
        nrow, ncol = _grid(nn + 2)
        fig, axs = plt.subplots(nrow, ncol, figsize=(ncol * 3, nrow * 3), squeeze=False)
        axs = axs.ravel()
        for c in range(3):
            for i in range(nn):
                self._scatter(axs[i], t[:, i, c], p[:, i, c], s=6, c=f[:, i], marker=markers[c], title=f"node:{i}")
            self._scatter(axs[nn], t[:, :, c].sum(1), p[:, :, c].sum(1), s=40, c=f.sum(1), marker=markers[c],
                          title="SUM")
            self._scatter(axs[nn + 1], t[:, :, c].sum(0), p[:, :, c].sum(0), s=40, c=f.sum(0), marker=markers[c],
                          title=f"SMP_Mean4sites:0-{nn}")
        for ax in axs[nn + 2:]:
            ax.axis("off")
        fig.tight_layout()
        self._save(fig, self._path(varname, iepoch), save_plot)

    def create_scatter_plots(self, true_values, predicted_values, output_names=None, iepoch=None):
        """One file per head: scalar heads -> parity + error PDF; vector heads -> parity per
        component; node-level heads laid out [sample, node] when every sample has the
        same node count (the reference's fixed-size LSMS configurations)."""
        if not true_values or len(true_values[0]) == 0:
            return
        names = self._names(output_names, len(true_values))
        for ih in range(len(true_values)):
            t, p = _np(true_values[ih]), _np(predicted_values[ih])
            dim = self.head_dims[ih] if ih < len(self.head_dims) else 1
            if dim > 1:
                self.create_parity_plot_vector(names[ih], t, p, dim, iepoch)
            else:
                self.create_parity_plot_and_error_histogram_scalar(names[ih], t.reshape(-1, 1), p.reshape(-1, 1),
                                                                   iepoch)

    # ------------------------------------------------------------------ history / sizes
    def plot_history(self, total_loss_train, total_loss_val, total_loss_test, task_loss_train, task_loss_val,
                     task_loss_test, task_weights, task_names):
        plt = _plt()
        tl = [_np(x).ravel() for x in (total_loss_train, total_loss_val, total_loss_test)]
        tk = [_np(x) for x in (task_loss_train, task_loss_val, task_loss_test)]
        ntask = tk[0].shape[1] if tk[0].ndim == 2 else 0
        nrow = 2 if ntask > 0 else 1
        ncol = max(1, ntask)
        fig, axs = plt.subplots(nrow, ncol, figsize=(16, 6 * nrow), squeeze=False)
        for v, lab, ls in zip(tl, ("train", "validation", "test"), ("-", ":", "--")):
            axs[0, 0].plot(v, ls, label=lab)
        axs[0, 0].set_title("total loss")
        axs[0, 0].set_xlabel("Epochs")
        axs[0, 0].set_yscale("log")
        axs[0, 0].legend()
        for ax in axs[0, 1:]:
            ax.axis("off")
        names = self._names(task_names, ntask)
        for k in range(ntask):
            ax = axs[1, k]
            for v, lab, ls in zip(tk, ("train", "validation", "test"), ("-", "-", "--")):
                ax.plot(v[:, k], ls, label=lab)
            ax.set_title(f"{names[k]}, {float(task_weights[k]):.4f}")
            ax.set_xlabel("Epochs")
            ax.set_yscale("log")
            if k == 0:
                ax.legend()
        fig.tight_layout()
        fig.savefig(os.path.join(self.dir, "history_loss.png"), dpi=100)
        plt.close(fig)
        np.savez(os.path.join(self.dir, "history_loss.npz"), total_train=tl[0], total_val=tl[1], total_test=tl[2],
                 task_train=tk[0], task_val=tk[1], task_test=tk[2], task_weights=np.asarray(task_weights, dtype=float),
                 task_names=np.asarray(names))

    def num_nodes_plot(self):
        if not self.num_nodes_list:
            return
        plt = _plt()
        fig, ax = plt.subplots(figsize=(4, 3))
        ax.hist(self.num_nodes_list, bins=min(50, max(5, len(set(self.num_nodes_list)))))
        ax.set_title("number of nodes per graph")
        ax.set_xlabel("nodes")
        fig.tight_layout()
        fig.savefig(os.path.join(self.dir, "num_nodes.png"), dpi=100)
        plt.close(fig)
