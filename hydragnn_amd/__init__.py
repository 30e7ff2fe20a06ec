"""hydragnn_amd — an MI355X-native multi-headed graph neural network framework with the
capabilities of HydraGNN (GPS global attention, 13 message-passing families,
multi-task / multi-branch heads, energy-force training, distributed training).

Compute path: PyTorch-ROCm + hand-written gfx950 HIP kernels (``_C.so``, ops under
``torch.ops.hydra``) + RCCL over xGMI.  Public API mirrors ``hydragnn``:
``run_training``, ``run_prediction`` and the ``utils``/``models``/``data`` modules.
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401
from .run_prediction import run_prediction  # noqa: F401
from .run_training import run_training, train_model  # noqa: F401
