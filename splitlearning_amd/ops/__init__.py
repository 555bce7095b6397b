"""Op dispatch: HIP kernels on GPU tensors, eager torch on CPU tensors.

`impl(device)` returns the module implementing the op set for that device.
`set_backend("torch")` forces the eager path everywhere (A/B checks);
`set_backend("hip")` requires the native extension even where "auto" would
also pick it.  There is no silent fallback: a GPU device with backend
"auto"/"hip" imports `hip_ops`, which fails loudly if `_C` is missing.
"""
from __future__ import annotations

import torch

from . import torch_ops
from .rng import keep_mask, step_seed

_BACKEND = "auto"


def set_backend(name: str):
    global _BACKEND
    if name not in ("auto", "hip", "torch"):
        raise ValueError(name)
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def impl(device):
    device = torch.device(device)
    if device.type == "cuda" and _BACKEND != "torch":
        from . import hip_ops
        hip_ops.C()   # raise now if the extension is missing
        return hip_ops
    if _BACKEND == "hip" and device.type != "cuda":
        raise RuntimeError("HIP backend requested for a non-GPU device")
    return torch_ops


__all__ = ["impl", "set_backend", "get_backend", "torch_ops", "keep_mask", "step_seed"]
