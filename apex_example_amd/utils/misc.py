"""Seeding and determinism switches (test_apex_distributed_spawn.py:60-80, R-07/R-08)."""
from __future__ import annotations

import os
import random

import torch


def set_cuda(deterministic=True):
    """cudnn flags map to MIOpen on ROCm: deterministic=True constrains MIOpen's
    solver choice (slower); False enables benchmark-mode solver search."""
    if torch.cuda.is_available():
        torch.backends.cudnn.deterministic = bool(deterministic)
        torch.backends.cudnn.benchmark = not deterministic


_DETERMINISTIC = False


def set_deterministic(on=True):
    """Framework-wide deterministic mode (the reference runs
    with cudnn.deterministic, test_apex_distributed_spawn.py:60-67,112).

    Every reduction of this framework's own kernels is already fixed-order (slab
    partials + finalize kernels, no float atomics): optimizers / norms, LayerNorm,
    BatchNorm, bias gradients, split-K weight-gradient reductions, attention, the
    embedding backward (device sort + ordered run sums).  MIOpen is constrained to
    deterministic solvers, the embedding backward takes its deterministic mode, and
    PyTorch ops are asked for their deterministic variants (warn-only).  Returns the
    mode."""
    global _DETERMINISTIC
    _DETERMINISTIC = bool(on)
    if torch.cuda.is_available():
        torch.backends.cudnn.deterministic = _DETERMINISTIC
        torch.backends.cudnn.benchmark = False if _DETERMINISTIC else torch.backends.cudnn.benchmark
    torch.use_deterministic_algorithms(_DETERMINISTIC, warn_only=True)
    from .. import _native
    if _DETERMINISTIC and _native.available():
        from ..ops import embedding
        embedding._MODE = "det"
    return _DETERMINISTIC


def deterministic():
    return _DETERMINISTIC


def set_seed(seed):
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
