from .fp16util import (  # noqa: F401
    BN_convert_float,
    FP16Model,
    clip_grad_norm,
    convert_module,
    convert_network,
    master_params_to_model_params,
    model_grads_to_master_grads,
    network_to_half,
    prep_param_lists,
    to_python_float,
    tofp16,
)
from .fp16_optimizer import FP16_Optimizer  # noqa: F401
from .loss_scaler import DynamicLossScaler, LossScaler  # noqa: F401
