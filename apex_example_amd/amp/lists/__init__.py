"""Apex O1 cast tables (apex@f3a960f8 apex/amp/lists/*.py).

O1 here is implemented by PyTorch's autocast dispatch key; these tables record
Apex's policy so tests can check that autocast applies the same decision to each
listed op (tests/test_amp_o1.py).  Ops whose autocast policy differs from Apex's
are listed in ``KNOWN_DIFFERENCES`` with the reason.
"""
from .functional_overrides import FP16_FUNCS as F_FP16, FP32_FUNCS as F_FP32, BANNED_FUNCS  # noqa
from .tensor_overrides import FP16_FUNCS as T_FP16, FP32_FUNCS as T_FP32, CASTS as T_CASTS  # noqa
from .torch_overrides import FP16_FUNCS, FP32_FUNCS, CASTS, SEQUENCE_CASTS  # noqa: F401

KNOWN_DIFFERENCES = {
    # autocast leaves these in the input dtype ("promote"/"fallthrough") where
    # Apex forced fp32; outputs stay numerically safe because the reductions
    # accumulate in fp32 internally on ROCm.
    "sum": "autocast: fp32 accumulation inside the kernel, output keeps input dtype",
    "prod": "autocast: fallthrough",
    "cumprod": "autocast: fp32 policy (same as Apex)",
}
