"""Bias gradient handed from a fused residual join to the dense layer that produced h.

A post-/pre-LN transformer sublayer ends in ``dense -> dropout -> (+ residual) -> LN``
(``normalization.fused_add_dropout_layer_norm``).  Its backward kernel forms
dh = dropout'(ds) row by row and already reduces dgamma / dbeta partials per block;
it also sums dh's columns in the same pass -
which is exactly the bias gradient of the dense layer whose output h was.  The dense
backward (``fused_dense._bias_grad``) then takes that result instead of re-reading
dh for its own column-sum pass (``csrc/hip/bias_grad.hip``: one full read of dh plus a
second small kernel per layer).

One slot: the join's backward offers (dh, its version, colsum); the next bias gradient
over exactly that tensor (same storage address and element count, not modified in
place since) takes it.  The slot holds a reference to dh, so its address cannot be
reused by another tensor while the offer stands; any other consumer pattern (dh summed
with another gradient, cast, sliced) simply misses and computes the sum itself.  An offer
nobody takes is dropped at the end of the backward pass that made it (an autograd final
callback), so it never pins dh into the next step.
"""
from __future__ import annotations

ENABLED = True

_SLOT = [None]


def offer(dh, colsum):
    _SLOT[0] = (dh, dh._version, colsum) if colsum is not None else None
    if colsum is not None:
        try:  # inside a backward pass (the join's backward): drop the offer when it ends
            import torch

            torch.autograd.Variable._execution_engine.queue_callback(clear)
        except RuntimeError:  # called outside a backward pass (tests)
            pass


def take(g2, dtype):
    """colsum(g2) computed by the join's backward, or None."""
    ent = _SLOT[0]
    if ent is None:
        return None
    dh, ver, cs = ent
    if (g2.data_ptr() == dh.data_ptr() and g2.numel() == dh.numel() and dh._version == ver
            and g2.dim() == 2 and g2.size(1) == cs.numel() and cs.dtype == dtype
            and g2.is_contiguous() and dh.is_contiguous() and g2.device == cs.device):
        _SLOT[0] = None
        return cs
    return None


def clear():
    _SLOT[0] = None
