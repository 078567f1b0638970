"""MI355X-native MMSBM EM engine for the triplet-link E/M loop of
AleixMT/TrigenicInteractionPredictor (src/TrigenicInteractionPredictor.py).

`Model` is the drop-in for the reference class; `EMEngine` is the batched
device engine underneath it (HIP kernels in libmmsbm.so via ctypes).
"""
from .model import Model  # noqa: F401

__all__ = ["Model", "EMEngine", "build"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "EMEngine":
        from .engine import EMEngine
        return EMEngine
    if name == "build":
        from .build import build
        return build
    raise AttributeError(name)
