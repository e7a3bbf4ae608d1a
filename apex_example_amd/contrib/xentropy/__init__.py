from .softmax_xentropy import SoftmaxCrossEntropyLoss  # noqa: F401
