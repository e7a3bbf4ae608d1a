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


def set_seed(seed):
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
