"""Fused multi-tensor optimizers (apex.optimizers API) on gfx950 kernels."""
from .fused_adagrad import FusedAdagrad
from .fused_adam import FusedAdam
from .fused_lamb import FusedLAMB
from .fused_novograd import FusedNovoGrad
from .fused_sgd import FusedSGD

_FUSED_TYPES = (FusedSGD, FusedAdam, FusedLAMB, FusedNovoGrad, FusedAdagrad)

__all__ = ["FusedSGD", "FusedAdam", "FusedLAMB", "FusedNovoGrad", "FusedAdagrad"]
