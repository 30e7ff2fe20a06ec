"""End-to-end accuracy tests: run_training + run_prediction on the deterministic CI
dataset with the reference thresholds (reference ``tests/test_graphs.py:200-320``,
same model matrix).

CPU (driver's ``-m "not gpu"`` run): a fast representative subset.
GPU (``-m gpu``): the full reference matrix through the MI355X path (HBM-resident
data, hipGraph-captured steps where shapes allow, HIP kernels).
"""
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
    ("EGNN", "", "", "ci", False),
    ("CGCNN", "", "", "ci", False),
]

ALL_MODELS = ["SAGE", "GIN", "GAT", "MFC", "PNA", "PNAPlus", "CGCNN", "SchNet", "DimeNet", "EGNN", "PNAEq", "PAINN",
              "MACE"]
EDGE_MODELS = ["GAT", "PNA", "PNAPlus", "CGCNN", "SchNet", "DimeNet", "EGNN", "PNAEq", "PAINN"]
EQUIVARIANT = ["EGNN", "SchNet", "PNAEq", "PAINN", "MACE"]
VECTOR_OUT = ["GAT", "PNA", "PNAPlus", "SchNet", "DimeNet", "EGNN", "PNAEq"]
CONV_HEAD = ["SAGE", "GIN", "GAT", "MFC", "PNA", "PNAPlus", "SchNet", "DimeNet", "EGNN", "PNAEq", "PAINN"]


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("ci_data"))


@pytest.mark.parametrize("mpnn_type,engine,attn,ci_input,lengths", CPU_CASES)
def test_train_cpu(mpnn_type, engine, attn, ci_input, lengths, workdir, monkeypatch):
    monkeypatch.setenv("HYDRAGNN_DEVICE_DATA", "0")
    unittest_train_model(mpnn_type, engine, attn, ci_input, lengths, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", ALL_MODELS)
@pytest.mark.parametrize("ci_input", ["ci", "ci_multihead"])
def test_train_gpu(mpnn_type, ci_input, workdir):
    unittest_train_model(mpnn_type, "", "", ci_input, False, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", EDGE_MODELS + ["MACE"])
def test_train_gpu_lengths(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "", "", "ci", True, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", EDGE_MODELS)
def test_train_gpu_lengths_gps(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "GPS", "multihead", "ci", True, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", EQUIVARIANT)
def test_train_gpu_equivariant(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "", "", "ci_equivariant", False, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", VECTOR_OUT)
def test_train_gpu_vectoroutput(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "", "", "ci_vectoroutput", True, workdir)


@pytest.mark.gpu
@pytest.mark.parametrize("mpnn_type", CONV_HEAD)
def test_train_gpu_conv_head(mpnn_type, workdir):
    unittest_train_model(mpnn_type, "", "", "ci_conv_head", False, workdir)
