from .self_multihead_attn import SelfMultiheadAttn  # noqa: F401
from .encdec_multihead_attn import EncdecMultiheadAttn  # noqa: F401
