"""Fused MI355X operators used by the model zoo (BatchNorm+ReLU, ...)."""
from .batch_norm import BatchNorm2dReLU, BatchNormFunction, batch_norm_act  # noqa: F401
from .attention import fused_attention, fused_attention_qkv  # noqa: F401
