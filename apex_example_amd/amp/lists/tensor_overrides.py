# Apex O1 policy for torch.Tensor methods (names only).
from . import torch_overrides

FP16_FUNCS = ["__matmul__"]

FP32_FUNCS = ["__ipow__", "__pow__", "__rpow__", "cpu"]

CASTS = [
    "__add__", "__div__", "__eq__", "__ge__", "__gt__", "__iadd__", "__idiv__", "__imul__",
    "__isub__", "__itruediv__", "__le__", "__lt__", "__mul__", "__ne__", "__radd__", "__rdiv__",
    "__rmul__", "__rsub__", "__rtruediv__", "__sub__", "__truediv__",
]

# None of these, but here to make code cleaner.
SEQUENCE_CASTS = []

# We need to grab all the methods from torch_overrides and add them to
# the Tensor lists as well, as almost all methods are duplicated
# between `torch` and `torch.Tensor` (and check with `hasattr`,
# because a few random ones aren't defined on Tensor)
FP16_FUNCS = FP16_FUNCS + [f for f in torch_overrides.FP16_FUNCS if f not in ("conv_tbc",)]
FP32_FUNCS = FP32_FUNCS + list(torch_overrides.FP32_FUNCS)
CASTS = CASTS + list(torch_overrides.CASTS)
