"""Drop-in facade for Apex's ``apex_C`` extension.

``flatten(tensors)`` concatenates the tensors' flattened views into one buffer
and ``unflatten(flat, like)`` returns views of ``flat`` shaped like ``like``.
The DDP path of this framework does not use them per step (gradients live as
views in persistent bucket buffers); they are kept for API parity.
"""
from . import _native


def flatten(tensors):
    return _native.require().apex_C.flatten(list(tensors))


def unflatten(flat, like):
    return _native.require().apex_C.unflatten(flat, list(like))
