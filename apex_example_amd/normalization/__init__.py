from .fused_layer_norm import (  # noqa: F401
    FusedLayerNorm,
    FusedRMSNorm,
    fused_add_dropout_layer_norm,
    fused_layer_norm,
    fused_layer_norm_affine,
    fused_rms_norm_affine,
)
