import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# single-process run_training calls still rendezvous (world 1) on HYDRAGNN_MASTER_PORT;
# give every pytest-xdist worker its own port so parallel workers do not collide
_w = os.environ.get("PYTEST_XDIST_WORKER", "")
if _w.startswith("gw") and "HYDRAGNN_MASTER_PORT" not in os.environ:
    os.environ["HYDRAGNN_MASTER_PORT"] = str(18900 + 13 * int(_w[2:]))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running end-to-end test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
