"""Shared attention core of the contrib multi-head attention modules."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ...ops import attention as fused_attn


def sdpa_masks(key_padding_mask, attn_mask, mask_additive, B, Tq, Tk, dtype, device):
    """Apex mask conventions -> one additive SDPA mask [B, 1, Tq, Tk] (or None).
    key_padding_mask [B, Tk]: True / 1 = padded key (or an additive float mask when
    ``mask_additive``); attn_mask [Tq, Tk]: True / 1 = masked (or additive)."""
    m = None
    if key_padding_mask is not None:
        kp = key_padding_mask.to(device)
        if mask_additive:
            m = kp.to(dtype).view(B, 1, 1, Tk)
        else:
            m = torch.zeros(B, 1, 1, Tk, dtype=dtype, device=device).masked_fill(
                kp.bool().view(B, 1, 1, Tk), float("-inf"))
    if attn_mask is not None:
        am = attn_mask.to(device)
        if mask_additive or am.is_floating_point():
            a = am.to(dtype).view(1, 1, Tq, Tk)
        else:
            a = torch.zeros(1, 1, Tq, Tk, dtype=dtype, device=device).masked_fill(
                am.bool().view(1, 1, Tq, Tk), float("-inf"))
        m = a if m is None else m + a
    return m


def attention_bshd(q, k, v, dropout_p, key_padding_mask=None, attn_mask=None,
                   mask_additive=False, allow_fused=True):
    """q [B, Tq, H, D], k/v [B, Tk, H, D] (any strides) -> [B, Tq, H, D].
    gfx950 fused kernels when eligible (no masks, Tq == Tk, D == 64, 16-bit),
    PyTorch SDPA otherwise."""
    B, Tq, H, D = q.shape
    Tk = k.size(1)
    if (allow_fused and key_padding_mask is None and attn_mask is None and Tq == Tk
            and fused_attn.supported(q, D)):
        return fused_attn.fused_attention(q, k, v, causal=False, dropout_p=dropout_p)
    mask = sdpa_masks(key_padding_mask, attn_mask, mask_additive, B, Tq, Tk, q.dtype, q.device)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                       attn_mask=mask, dropout_p=dropout_p,
                                       scale=1.0 / math.sqrt(D))
    return o.transpose(1, 2)
