"""Registry of all message-passing stacks (imported lazily by ``create.py``)."""
from .basic import GINStack, MFCStack, SAGEStack  # noqa: F401
from .pnaplus import PNAPlusStack, PNAStack  # noqa: F401

_lazy = {
    "GATStack": ".gat",
    "CGCNNStack": ".cgcnn",
    "SCFStack": ".schnet",
    "DIMEStack": ".dimenet",
    "EGCLStack": ".egnn",
    "PAINNStack": ".painn",
    "PNAEqStack": ".painn",
    "MACEStack": ".mace",
}


def __getattr__(name):
    if name in _lazy:
        import importlib

        mod = importlib.import_module(_lazy[name], __package__)
        return getattr(mod, name)
    raise AttributeError(name)
