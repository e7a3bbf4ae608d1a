"""apex.contrib counterparts: fused softmax cross entropy
(``xentropy``), fast multi-head attention (``multihead_attn``), NHWC group
BatchNorm (``groupbn``) and ZeRO-style sharded optimizers (``optimizers``),
all on this package's gfx950 kernels / RCCL."""
