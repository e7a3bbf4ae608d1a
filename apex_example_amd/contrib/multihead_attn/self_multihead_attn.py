"""SelfMultiheadAttn (apex@f3a960f8 apex/contrib/multihead_attn/self_multihead_attn.py,
SURVEY.md A-24): time-first [T, B, E] self-attention with a fused QKV input
projection, the gfx950 fused attention kernels (ops/attention.py) and an
optional fused pre-LayerNorm + dropout + residual add (``include_norm_add``).

Parameter names follow Apex (``in_proj_weight`` / ``q_weight, k_weight,
v_weight`` with ``separate_qkv_params``, ``out_proj_weight``,
``lyr_nrm_gamma_weights`` / ``lyr_nrm_beta_weights``) so state dicts carry over.
``impl='default'`` forces the PyTorch SDPA path; ``impl='fast'`` (default)
uses the fused kernels whenever there is no mask.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import Parameter

from ...normalization.fused_layer_norm import FusedLayerNormAffineFunction
from ._common import attention_bshd


class SelfMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False,
                 impl="fast", separate_qkv_params=False, mask_additive=False):
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
        self.separate_qkv_params = separate_qkv_params
        self.mask_additive = mask_additive
        if separate_qkv_params:
            self.q_weight = Parameter(torch.empty(embed_dim, embed_dim))
            self.k_weight = Parameter(torch.empty(embed_dim, embed_dim))
            self.v_weight = Parameter(torch.empty(embed_dim, embed_dim))
        else:
            self.in_proj_weight = Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.out_proj_weight = Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            if separate_qkv_params:
                self.q_bias = Parameter(torch.empty(embed_dim))
                self.k_bias = Parameter(torch.empty(embed_dim))
                self.v_bias = Parameter(torch.empty(embed_dim))
            else:
                self.in_proj_bias = Parameter(torch.empty(3 * embed_dim))
            self.out_proj_bias = Parameter(torch.empty(embed_dim))
        else:
            if separate_qkv_params:
                self.register_parameter("q_bias", None)
                self.register_parameter("k_bias", None)
                self.register_parameter("v_bias", None)
            else:
                self.register_parameter("in_proj_bias", None)
            self.register_parameter("out_proj_bias", None)
        if include_norm_add:
            self.lyr_nrm_gamma_weights = Parameter(torch.ones(embed_dim))
            self.lyr_nrm_beta_weights = Parameter(torch.zeros(embed_dim))
        self.reset_parameters()

    def reset_parameters(self):
        if self.separate_qkv_params:
            for w in (self.q_weight, self.k_weight, self.v_weight):
                nn.init.xavier_uniform_(w)
        else:
            # the fused [3E, E] weight initialised as three [E, E] blocks
            nn.init.xavier_uniform_(self.in_proj_weight, gain=math.sqrt(2))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            if self.separate_qkv_params:
                for b in (self.q_bias, self.k_bias, self.v_bias):
                    nn.init.constant_(b, 0.0)
            else:
                nn.init.constant_(self.in_proj_bias, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)
        if self.include_norm_add:
            nn.init.ones_(self.lyr_nrm_gamma_weights)
            nn.init.zeros_(self.lyr_nrm_beta_weights)

    def _qkv_weight(self):
        if self.separate_qkv_params:
            w = torch.cat([self.q_weight, self.k_weight, self.v_weight], 0)
            b = (torch.cat([self.q_bias, self.k_bias, self.v_bias], 0) if self.bias else None)
            return w, b
        return self.in_proj_weight, self.in_proj_bias

    def forward(self, query, key=None, value=None, key_padding_mask=None, need_weights=False,
                attn_mask=None, is_training=True):
        """query [T, B, E] -> (out [T, B, E], None).  key / value are ignored
        (self-attention), as in Apex's fast implementation."""
        T, B, E = query.shape
        x = query
        if self.include_norm_add:
            if x.is_cuda:
                x = FusedLayerNormAffineFunction.apply(x, self.lyr_nrm_gamma_weights.to(x.dtype),
                                                       self.lyr_nrm_beta_weights.to(x.dtype),
                                                       (E,), 1e-5)
            else:
                x = F.layer_norm(x, (E,), self.lyr_nrm_gamma_weights, self.lyr_nrm_beta_weights)
        w, b = self._qkv_weight()
        qkv = F.linear(x, w, b).view(T, B, 3, self.num_heads, self.head_dim)
        q, k, v = qkv.permute(1, 0, 2, 3, 4).unbind(2)  # [B, T, H, D] strided views
        p = self.dropout if (is_training and self.training) else 0.0
        o = attention_bshd(q, k, v, p, key_padding_mask, attn_mask, self.mask_additive,
                           allow_fused=(self.impl == "fast"))
        o = o.transpose(0, 1).reshape(T, B, E)
        out = F.linear(o, self.out_proj_weight, self.out_proj_bias)
        if self.include_norm_add:
            out = query + F.dropout(out, p=self.dropout, training=is_training and self.training)
        return out, None
