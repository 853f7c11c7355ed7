"""Recursive structure helpers (torchrec/utils/data_structure.py:10-52)."""
from typing import Callable

import torch
from torch import Tensor


def map_structure(func: Callable, structure):
    if not callable(func):
        raise TypeError("func must be callable, got: %s" % func)
    if isinstance(structure, list):
        return [map_structure(func, item) for item in structure]
    if isinstance(structure, dict):
        return {key: map_structure(func, structure[key]) for key in structure}
    return func(structure)


def tensor_to_device(structure, device: torch.device, non_blocking: bool = False):
    """``.to(device)`` of every tensor in a nested batch (the H2D boundary of
    IModel.train_step, IModel.py:119).  ``non_blocking`` lets a pinned columnar
    batch overlap the copy with compute."""
    def _to(t):
        return t.to(device=device, non_blocking=non_blocking) if isinstance(t, Tensor) else t
    return map_structure(_to, structure)
