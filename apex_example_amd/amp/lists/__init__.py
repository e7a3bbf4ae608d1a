"""Apex O1 cast tables (apex@f3a960f8 apex/amp/lists/*.py).

These tables ARE the O1 policy specification: ``audit.audit()`` calls every
entry under O1 and checks its output dtype against them (tests/
test_amp_o1_tables.py, fp16 and bf16, CPU via fake CUDA tensors and on the
GPU).  O1 runs on PyTorch's autocast dispatch key; the entries where autocast
decides differently are overridden with Apex's decision in
``amp.amp.APEX_POLICY_OVERRIDES``; the deliberate exceptions are listed with
their reason in ``audit.KNOWN_DIFFERENCES``.
"""
from .functional_overrides import FP16_FUNCS as F_FP16, FP32_FUNCS as F_FP32, BANNED_FUNCS  # noqa
from .tensor_overrides import FP16_FUNCS as T_FP16, FP32_FUNCS as T_FP32, CASTS as T_CASTS  # noqa
from .torch_overrides import FP16_FUNCS, FP32_FUNCS, CASTS, SEQUENCE_CASTS  # noqa: F401
