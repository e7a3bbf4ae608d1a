"""apex.contrib.optimizers counterparts."""
from ...fp16_utils import FP16_Optimizer  # noqa: F401
from ...optimizers import FusedAdam, FusedLAMB, FusedSGD  # noqa: F401
from .distributed_fused_adam import DistributedFusedAdam  # noqa: F401
