# Apex O1 policy for torch.* functions (names only).
FP16_FUNCS = [
    # Low level functions wrapped by torch.nn layers.
    "conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d", "conv_transpose3d",
    "conv_tbc", "prelu",
    # BLAS
    "addmm", "addmv", "addr", "matmul", "mm", "mv",
]

FP32_FUNCS = [
    # Pointwise
    "acos", "asin", "cosh", "erfinv", "exp", "expm1", "log", "log10", "log2", "log1p",
    "reciprocal", "rsqrt", "sinh", "tan",
    # Other math
    "pow",
    # Reduction
    "cumprod", "cumsum", "dist", "norm", "prod", "std", "sum", "var",
    # Misc
    "renorm",
]

# Multi-tensor fns that may need type promotion
CASTS = [
    # Multi-tensor math
    "addcdiv", "addcmul", "atan2", "cross", "bilinear", "dot",
    # Element-wise _or_ tensor-wise math
    "add", "div", "mul",
    # Comparison
    "eq", "equal", "ge", "gt", "le", "lt", "ne",
]

# Functions that take sequence arguments. We need to inspect the whole
# sequence and cast to the widest type.
SEQUENCE_CASTS = ["cat", "stack"]
