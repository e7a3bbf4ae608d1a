"""Fused multi-head attention (head dim 64, bf16 / fp16) on the gfx950 MFMA
kernels of csrc/hip/attention.hip: flash-attention style forward (online
softmax, never materialises the S x S scores) and backward (dK/dV and dQ
kernels recomputing P from the saved log-sum-exp; no atomics, so gradients are
bitwise reproducible), with an optional causal mask and dropout whose keep
mask is a counter-based hash of (seed, batch*head, query, key) regenerated
exactly by the backward.

``fused_attention_qkv(qkv)`` takes the packed [B, S, 3, H, 64] output of a
fused QKV projection and returns o as [B, S, H, 64] (``.view(B, S, H*64)`` is
free); its backward writes dQ/dK/dV straight into ONE packed buffer, so the
projection's input gradient needs no concatenation.  Layout-generic views
([S, B, ...] sequence-first included) work: the kernels take strides.

Eligibility (``supported``): GPU tensor, bf16/fp16, head dim 64, q/k/v of one
sequence length, no additive mask.  Callers fall back to
``F.scaled_dot_product_attention`` otherwise.
"""
from __future__ import annotations

import math

import torch

from .. import _native


def _C():
    return _native.require().attn


def supported(t: torch.Tensor, head_dim: int) -> bool:
    return (t.is_cuda and head_dim == 64 and t.dtype in (torch.bfloat16, torch.float16)
            and _native.available())


_WARNED = set()


def effective_dropout(p: float) -> float:
    """The dropout rate the kernels apply for a requested ``p``: one hash byte per
    (query, key) is compared with round(256 p), so the rate is a multiple of 1/256
    (p = 0.1 runs at 26/256 = 0.1016), and any p > 0 drops at least 1/256."""
    if p <= 0.0:
        return 0.0
    return min(256, max(1, int(p * 256.0 + 0.5))) / 256.0


def _check_rate(p: float) -> None:
    """Warn (once per rate) where the 1/256 quantisation moves the rate by more than 2 %."""
    q = effective_dropout(p)
    if p > 0.0 and abs(q - p) > 0.02 * p and p not in _WARNED:
        import warnings

        _WARNED.add(p)
        warnings.warn("fused attention: dropout p=%g runs at %g (the kernels quantise the rate "
                      "to 1/256)" % (p, q))


def _seed(dropout_p: float) -> int:
    """Per-call dropout seed from torch's CPU generator (no device sync; follows
    torch.manual_seed)."""
    if dropout_p <= 0.0:
        return 0
    _check_rate(dropout_p)
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


class FusedAttentionFunction(torch.autograd.Function):
    """o = softmax(q k^T * scale [+ causal mask]) [dropout] v on [B, S, H, 64] views."""

    @staticmethod
    def forward(ctx, q, k, v, causal, dropout_p, scale, seed):
        o, lse = _C().fwd(q, k, v, bool(causal), float(dropout_p), int(seed), float(scale))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (bool(causal), float(dropout_p), int(seed), float(scale))
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        causal, p, seed, scale = ctx.cfg
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format)
        _C().bwd(do, q, k, v, o, lse, causal, p, seed, scale, dq, dk, dv)
        return dq, dk, dv, None, None, None, None


class FusedQKVAttentionFunction(torch.autograd.Function):
    """Packed variant: qkv [B, S, 3, H, 64] (any strides) -> o [B, S, H, 64];
    backward returns one packed dqkv of qkv's layout."""

    @staticmethod
    def forward(ctx, qkv, causal, dropout_p, scale, seed):
        q, k, v = qkv.unbind(2)
        o, lse = _C().fwd(q, k, v, bool(causal), float(dropout_p), int(seed), float(scale))
        ctx.save_for_backward(qkv, o, lse)
        ctx.cfg = (bool(causal), float(dropout_p), int(seed), float(scale))
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        causal, p, seed, scale = ctx.cfg
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv.unbind(2)
        dq, dk, dv = dqkv.unbind(2)
        _C().bwd(do, q, k, v, o, lse, causal, p, seed, scale, dq, dk, dv)
        return dqkv, None, None, None, None


def fused_attention(q, k, v, causal=False, dropout_p=0.0, scale=None):
    """q, k, v: [B, S, H, 64] -> o [B, S, H, 64]."""
    scale = 1.0 / math.sqrt(q.size(-1)) if scale is None else scale
    return FusedAttentionFunction.apply(q, k, v, causal, dropout_p, scale, _seed(dropout_p))


def fused_attention_qkv(qkv, causal=False, dropout_p=0.0, scale=None):
    """qkv: [B, S, 3, H, 64] -> o [B, S, H, 64]."""
    scale = 1.0 / math.sqrt(qkv.size(-1)) if scale is None else scale
    return FusedQKVAttentionFunction.apply(qkv, causal, dropout_p, scale, _seed(dropout_p))
