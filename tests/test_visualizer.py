"""Visualizer plot families (reference postprocess/visualizer.py): every entry point
writes its PNG under ./logs/<name>/, and the histogram helpers are exact."""
import os

import numpy as np
import pytest

from hydragnn_amd.postprocess.visualizer import Visualizer, err_condmean, error_pdf


def test_err_condmean_constant_error():
    t = np.linspace(0, 1, 1000)
    xc, me = err_condmean(t, t + 0.5)
    # every bin of the true value sees |err| = 0.5 (bin centre of a degenerate histogram)
    assert xc.shape == (50,) and np.allclose(me[me > 0], me[me > 0][0])


def test_error_pdf_normalised():
    rng = np.random.default_rng(0)
    t = rng.normal(size=5000)
    xc, h = error_pdf(t, t + rng.normal(scale=0.1, size=t.size))
    assert abs(np.sum(h) * (xc[1] - xc[0]) - 1.0) < 1e-6


def test_all_plots(tmp_path, monkeypatch):
    pytest.importorskip("matplotlib")
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(1)
    ns, nn = 40, 4
    feat = rng.normal(size=(ns, nn))
    v = Visualizer("m", node_feature=feat, num_heads=2, head_dims=[1, 3], num_nodes_list=[3, 4, 4, 5])
    t_s, t_v = rng.normal(size=(ns, 1)), rng.normal(size=(ns, 3))
    v.create_plot_global([t_s, t_v], [t_s + 0.1, t_v * 0.9], output_names=["e", "f"])
    v.create_scatter_plots([t_s, t_v], [t_s, t_v], output_names=["e", "f"], iepoch=3)
    tn = rng.normal(size=(ns, nn))
    v.create_parity_plot_and_error_histogram_scalar("charge", tn, tn + 0.01)
    v.create_error_histogram_per_node("charge", tn, tn + 0.01, iepoch=2)
    v.create_parity_plot_per_node_vector("mom", rng.normal(size=(ns, nn * 3)), rng.normal(size=(ns, nn * 3)))
    hist = np.abs(rng.normal(size=6)) + 0.1
    v.plot_history(hist, hist, hist, np.abs(rng.normal(size=(6, 2))) + 0.1, np.ones((6, 2)), np.ones((6, 2)),
                   [1.0, 0.5], ["e", "f"])
    v.num_nodes_plot()
    files = set(os.listdir(tmp_path / "logs" / "m"))
    for f in ["e_scatter_condm_err.png", "f_scatter_condm_err.png", "e_0003.png", "f_0003.png", "charge.png",
              "charge_error_hist1d_0002.png", "mom.png", "history_loss.png", "history_loss.npz", "num_nodes.png"]:
        assert f in files, (f, files)
    d = np.load(tmp_path / "logs" / "m" / "history_loss.npz")  # no pickle
    assert d["task_train"].shape == (6, 2)
