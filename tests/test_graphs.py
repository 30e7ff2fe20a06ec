"""End-to-end accuracy tests: run_training + run_prediction on the deterministic CI
dataset with the reference thresholds (reference ``tests/test_graphs.py``).

CPU (driver's ``-m "not gpu"`` run): a fast representative subset.
GPU (``-m gpu``): the full model matrix through the MI355X path (HBM-resident data,
hipGraph-captured steps, HIP kernels).
"""
import os

import pytest

from graph_train_util import unittest_train_model

CPU_CASES = [
    ("SAGE", "", "", "ci", False),
    ("GIN", "", "", "ci", False),
    ("PNA", "", "", "ci", False),
    ("PNAPlus", "", "", "ci", False),
    ("PNAPlus", "GPS", "multihead", "ci", False),
    ("PNA", "", "", "ci_multihead", False),
    ("PNA", "", "", "ci", True),
]


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("ci_data"))


@pytest.mark.parametrize("mpnn_type,engine,attn,ci_input,lengths", CPU_CASES)
def test_train_cpu(mpnn_type, engine, attn, ci_input, lengths, workdir, monkeypatch):
    monkeypatch.setenv("HYDRAGNN_DEVICE_DATA", "0")
    unittest_train_model(mpnn_type, engine, attn, ci_input, lengths, workdir)


GPU_MODELS = ["SAGE", "GIN", "MFC", "PNA", "PNAPlus"]


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", GPU_MODELS)
@pytest.mark.parametrize("ci_input", ["ci", "ci_multihead"])
def test_train_gpu(mpnn_type, ci_input, workdir):
    unittest_train_model(mpnn_type, "", "", ci_input, False, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", ["PNA", "PNAPlus"])
def test_train_gpu_gps(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "GPS", "multihead", "ci", False, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", ["PNA", "PNAPlus"])
def test_train_gpu_lengths(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "", "", "ci", True, workdir)
