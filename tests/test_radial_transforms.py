"""MACE radial bases x distance transforms (reference ``tests/test_radial_transforms.py:186-208``,
which sweeps bessel/gaussian/chebyshev x None/Agnesi/Soft; here the MACE stack is really
built with them).  Parity with ase's covalent-radius table is unpinned (ase is absent):
the table is checked at anchor values and the transforms by their analytic properties."""
import pytest
import torch

from hydragnn_amd.ops.covalent import COVALENT_RADII, AgnesiTransform, SoftTransform


def test_covalent_table_anchors():
    assert len(COVALENT_RADII) == 119
    for z, r in {1: 0.31, 6: 0.76, 8: 0.66, 14: 1.11, 26: 1.32, 29: 1.32, 78: 1.36, 92: 1.96}.items():
        assert COVALENT_RADII[z] == r


def test_agnesi_properties():
    t = AgnesiTransform()
    x = torch.linspace(1e-3, 8.0, 400).view(-1, 1)
    z = torch.full((400,), 6, dtype=torch.long)
    y = t(x, z, z).view(-1)
    assert torch.all((y > 0) & (y <= 1))
    assert torch.all(y[1:] <= y[:-1] + 1e-7)  # monotone decreasing in the distance
    # at r = r0 (sum of radii / 2 = 0.76 for C-C): y = 1 / (1 + a / 2)
    y0 = t(torch.tensor([[0.76]]), z[:1], z[:1]).item()
    assert abs(y0 - 1.0 / (1.0 + 1.0805 / 2)) < 1e-5


def test_soft_properties():
    t = SoftTransform()
    z = torch.full((3,), 8, dtype=torch.long)
    x = torch.tensor([[0.0], [0.33], [20.0]])
    y = t(x, z, z).view(-1)
    assert abs(y[0].item() - 0.5) < 1e-6  # y(0) = 1/2
    assert abs(y[2].item() - 20.0) < 1e-4  # identity far beyond r0
    # analytic derivative 1 - sech^2(s) (1 + a b u^(b-1)) / (2 r0) at an interior point
    xg = torch.tensor([[0.4]], requires_grad=True)
    t(xg, z[:1], z[:1]).sum().backward()
    r0, u = 0.33, 0.4 / 0.33
    s = -u - 0.2 * u ** 3
    want = 1 - (1 - torch.tanh(torch.tensor(s)) ** 2) * (1 + 0.2 * 3 * u ** 2) / (2 * r0)
    assert abs(xg.grad.item() - float(want)) < 1e-4


@pytest.mark.parametrize("radial_type", ["bessel", "gaussian", "chebyshev"])
@pytest.mark.parametrize("transform", [None, "Agnesi", "Soft"])
def test_mace_radial_embedding_variants(radial_type, transform):
    from hydragnn_amd.models.mace import RadialEmbeddingBlock

    blk = RadialEmbeddingBlock(5.0, 8, 5, radial_type, transform)
    d = torch.rand(50, 1) * 4.9 + 0.05
    z = torch.randint(1, 30, (50,))
    out = blk(d, z, z.flip(0))
    assert out.shape == (50, 8) and torch.isfinite(out).all()
    # the polynomial cutoff acts on the raw length: zero beyond r_max whatever the transform
    far = blk(torch.full((4, 1), 5.5), z[:4], z[:4])
    assert torch.all(far == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("radial_type", ["bessel", "gaussian", "chebyshev"])
@pytest.mark.parametrize("transform", [None, "Agnesi", "Soft"])
def test_mace_trains_with_radial_variants(radial_type, transform, tmp_path):
    from graph_train_util import unittest_train_model

    unittest_train_model("MACE", "", "", "ci", False, str(tmp_path),
                         overwrite_config={"NeuralNetwork": {"Architecture": {"radial_type": radial_type,
                                                                              "distance_transform": transform}}})
