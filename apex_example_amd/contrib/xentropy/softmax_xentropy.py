"""Fused softmax cross entropy with label smoothing
(apex@f3a960f8 apex/contrib/xentropy/softmax_xentropy.py).

``SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing=0.0, padding_idx=0,
half_to_float=False)`` returns the per-row losses

    loss = logsumexp(x) - (1 - smoothing) * x[label] - smoothing * mean(x)

(0 for rows whose label is ``padding_idx``), computed by one gfx950 kernel pass
over the 16-bit logits (csrc/hip/xentropy.hip) that keeps only the row's
log-sum-exp for the backward; the backward writes the logits gradient in the
logits' dtype in one more pass.  No fp32 copy of the logits and no
log-softmax tensor is materialised.  CPU tensors run the extension's ATen
reference path.
"""
from __future__ import annotations

import torch

from ... import _native


def _C():
    return _native.require().xentropy


class SoftmaxCrossEntropyLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing=0.0, padding_idx=0, half_to_float=False):
        losses, max_log_sum_exp = _C().forward(logits, labels, float(smoothing), int(padding_idx),
                                               bool(half_to_float))
        ctx.save_for_backward(logits, max_log_sum_exp, labels)
        ctx.smoothing = float(smoothing)
        ctx.padding_idx = int(padding_idx)
        return losses

    @staticmethod
    def backward(ctx, grad_loss):
        logits, max_log_sum_exp, labels = ctx.saved_tensors
        grad_logits = _C().backward(grad_loss.contiguous(), logits, max_log_sum_exp, labels,
                                    ctx.smoothing, ctx.padding_idx)
        return grad_logits, None, None, None, None


def softmax_cross_entropy(logits, labels, smoothing=0.0, padding_idx=-100, reduction="mean"):
    """Convenience wrapper: fused per-row losses reduced over non-padding rows
    (the count stays on the device: no host sync)."""
    losses = SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing, padding_idx, True)
    if reduction == "none":
        return losses
    if reduction == "sum":
        return losses.sum()
    valid = (labels != padding_idx).sum().clamp_min(1)
    return losses.sum() / valid
