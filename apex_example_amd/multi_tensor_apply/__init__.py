from .multi_tensor_apply import MultiTensorApply, multi_tensor_applier  # noqa: F401
