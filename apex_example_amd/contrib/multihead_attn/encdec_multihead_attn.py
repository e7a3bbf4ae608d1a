"""EncdecMultiheadAttn (apex@f3a960f8 apex/contrib/multihead_attn/encdec_multihead_attn.py,
SURVEY.md A-24): time-first encoder-decoder attention, queries from ``query``
[Tq, B, E] (``in_proj_weight_q``), keys / values from ``key`` [Tk, B, E]
(fused ``in_proj_weight_kv``), optional fused pre-LayerNorm + residual add.
The gfx950 fused attention kernels run when Tq == Tk and no mask is given;
otherwise PyTorch SDPA.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import Parameter

from ._common import attention_bshd


class EncdecMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False,
                 impl="fast"):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim, "embed_dim must be divisible by num_heads"
        self.bias = bias
        self.include_norm_add = include_norm_add
        self.impl = impl
        self.scaling = self.head_dim ** -0.5
        self.in_proj_weight_q = Parameter(torch.empty(embed_dim, embed_dim))
        self.in_proj_weight_kv = Parameter(torch.empty(2 * embed_dim, embed_dim))
        self.out_proj_weight = Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            self.in_proj_bias_q = Parameter(torch.empty(embed_dim))
            self.in_proj_bias_kv = Parameter(torch.empty(2 * embed_dim))
            self.out_proj_bias = Parameter(torch.empty(embed_dim))
        else:
            self.register_parameter("in_proj_bias_q", None)
            self.register_parameter("in_proj_bias_kv", None)
            self.register_parameter("out_proj_bias", None)
        if include_norm_add:
            self.lyr_nrm_gamma_weights = Parameter(torch.ones(embed_dim))
            self.lyr_nrm_beta_weights = Parameter(torch.zeros(embed_dim))
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight_q)
        nn.init.xavier_uniform_(self.in_proj_weight_kv, gain=math.sqrt(1.5))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            nn.init.constant_(self.in_proj_bias_q, 0.0)
            nn.init.constant_(self.in_proj_bias_kv, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)

    def forward(self, query, key, value=None, key_padding_mask=None, need_weights=False,
                attn_mask=None, is_training=True):
        """query [Tq, B, E], key [Tk, B, E] (value = key) -> (out [Tq, B, E], None)."""
        Tq, B, E = query.shape
        Tk = key.size(0)
        x = query
        if self.include_norm_add:
            x = F.layer_norm(x, (E,), self.lyr_nrm_gamma_weights.to(x.dtype),
                             self.lyr_nrm_beta_weights.to(x.dtype))
        q = F.linear(x, self.in_proj_weight_q, self.in_proj_bias_q)
        kv = F.linear(key, self.in_proj_weight_kv, self.in_proj_bias_kv)
        q = q.view(Tq, B, self.num_heads, self.head_dim).transpose(0, 1)
        k, v = kv.view(Tk, B, 2, self.num_heads, self.head_dim).permute(1, 0, 2, 3, 4).unbind(2)
        p = self.dropout if (is_training and self.training) else 0.0
        o = attention_bshd(q, k, v, p, key_padding_mask, attn_mask, False,
                           allow_fused=(self.impl == "fast"))
        out = F.linear(o.transpose(0, 1).reshape(Tq, B, E), self.out_proj_weight,
                       self.out_proj_bias)
        if self.include_norm_add:
            out = query + F.dropout(out, p=self.dropout, training=is_training and self.training)
        return out, None
