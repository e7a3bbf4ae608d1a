"""GPT-2 (Radford et al. 2019) language model defined in-repo: pre-LN decoder
blocks with FusedLayerNorm, causal attention on the gfx950 fused attention
kernels (ops/attention.py; PyTorch SDPA off-GPU / fp32),
tanh-GELU MLP and an LM head tied to the token embedding.

gpt2_medium(): 24 layers, d_model 1024, 16 heads, vocab 50257, 1024 positions
= 354,823,168 parameters in 292 tensors.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.embedding import Embedding
from .. import _native
from ..normalization import FusedLayerNorm, fused_add_dropout_layer_norm
from ..fused_dense import cast_params_once, fused_dense_function, fused_dense_gelu_dense_function
from ..ops import attention as fused_attn


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 1024
    n_layer: int = 24
    n_head: int = 16
    resid_pdrop: float = 0.1
    embd_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    fused_layer_norm: bool = True
    fused_attention: bool = True
    fused_dense: bool = True  # fused bias-grad / GELU-backward dense layers (fused_dense)
    # residual add + dropout + the next LayerNorm as one kernel per sublayer join
    # (fp32 residual stream, 16-bit sublayer output under O1)
    fused_residual_ln: bool = True


def _ln(cfg, n):
    if cfg.fused_layer_norm:
        return FusedLayerNorm(n, eps=cfg.layer_norm_epsilon)
    return nn.LayerNorm(n, eps=cfg.layer_norm_epsilon)


class GPT2Attention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.h = cfg.n_head
        self.d = cfg.n_embd // cfg.n_head
        self.c_attn = nn.Linear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = nn.Linear(cfg.n_embd, cfg.n_embd)
        self.p = cfg.attn_pdrop
        self.resid_dropout = nn.Dropout(cfg.resid_pdrop)
        self.fused = cfg.fused_attention
        self.fused_dense = cfg.fused_dense

    def _lin(self, m, x):
        return fused_dense_function(x, m.weight, m.bias) if self.fused_dense else m(x)

    def forward(self, x, resid_dropout=True):
        b, s, e = x.shape
        drop = self.resid_dropout if resid_dropout else (lambda t: t)
        qkv = self._lin(self.c_attn, x).view(b, s, 3, self.h, self.d)
        p = self.p if self.training else 0.0
        if self.fused and fused_attn.supported(qkv, self.d):
            o = fused_attn.fused_attention_qkv(qkv, causal=True, dropout_p=p).view(b, s, e)
            return drop(self._lin(self.c_proj, o))
        qkv = qkv.permute(2, 0, 3, 1, 4)
        o = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], is_causal=True, dropout_p=p)
        o = o.transpose(1, 2).reshape(b, s, e)
        return drop(self._lin(self.c_proj, o))


class GPT2MLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.c_fc = nn.Linear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = nn.Linear(4 * cfg.n_embd, cfg.n_embd)
        self.dropout = nn.Dropout(cfg.resid_pdrop)
        self.fused_dense = cfg.fused_dense

    def forward(self, x, dropout=True):
        drop = self.dropout if dropout else (lambda t: t)
        if self.fused_dense:
            return drop(fused_dense_gelu_dense_function(
                x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias,
                "tanh"))
        return drop(self.c_proj(F.gelu(self.c_fc(x), approximate="tanh")))


class GPT2Block(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.ln_1 = _ln(cfg, cfg.n_embd)
        self.attn = GPT2Attention(cfg)
        self.ln_2 = _ln(cfg, cfg.n_embd)
        self.mlp = GPT2MLP(cfg)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))

    def forward_joined(self, x, y, next_ln):
        """Same block with the sublayer joins fused: ``y`` = ln_1(x) is given,
        returns (next_ln(x'), x') for the block output x'.  Each join (dropout,
        residual add, the following LayerNorm) is one kernel each way."""
        # y only feeds autocast GEMMs (c_attn / c_fc / the tied LM head): under O1 it
        # leaves the join in the GEMM dtype instead of fp32 + a cast kernel
        y16 = torch.is_autocast_enabled("cuda")
        y, x = fused_add_dropout_layer_norm(x, self.attn(y, resid_dropout=False), self.ln_2,
                                            self.attn.resid_dropout.p, self.training, y16)
        return fused_add_dropout_layer_norm(x, self.mlp(y, dropout=False), next_ln,
                                            self.mlp.dropout.p, self.training, y16)


class GPT2LMHeadModel(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.config = cfg
        self.wte = Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = Embedding(cfg.n_positions, cfg.n_embd)
        self.drop = nn.Dropout(cfg.embd_pdrop)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = _ln(cfg, cfg.n_embd)
        self.apply(self._init)
        # GPT-2: scale the residual projections by 1/sqrt(2 * n_layer)
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):
                nn.init.normal_(p, std=cfg.initializer_range / (2 * cfg.n_layer) ** 0.5)

    def _init(self, m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=self.config.initializer_range)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=self.config.initializer_range)

    def forward(self, input_ids):
        s = input_ids.size(1)
        pos = torch.arange(s, device=input_ids.device).unsqueeze(0)
        x = self.drop(self.wte(input_ids) + self.wpe(pos))
        if self.config.fused_dense and x.is_cuda and torch.is_autocast_enabled("cuda"):
            # O1: every dense weight / bias cast to the GEMM dtype in one launch
            dense = [p for blk in self.h for m in (blk.attn.c_attn, blk.attn.c_proj,
                                                   blk.mlp.c_fc, blk.mlp.c_proj)
                     for p in (m.weight, m.bias)]
            with cast_params_once(dense, torch.get_autocast_dtype("cuda")):
                return self._blocks(x)
        return self._blocks(x)

    def _blocks(self, x):
        if self.config.fused_residual_ln:
            y = self.h[0].ln_1(x)
            for i, block in enumerate(self.h):
                nxt = self.h[i + 1].ln_1 if i + 1 < len(self.h) else self.ln_f
                y, x = block.forward_joined(x, y, nxt)
            return F.linear(y, self.wte.weight)  # tied LM head
        for block in self.h:
            x = block(x)
        x = self.ln_f(x)
        return F.linear(x, self.wte.weight)  # tied LM head


def lm_loss(logits, input_ids, fused=True):
    """Next-token cross entropy with an fp32 softmax.  ``fused``: the gfx950
    softmax-cross-entropy kernel (contrib.xentropy) reads the 16-bit logits
    directly (the last position's label is padding) instead of materialising a
    sliced fp32 copy of the [B*S, vocab] logits."""
    if fused and logits.is_cuda and _native.available():
        from ..contrib.xentropy import SoftmaxCrossEntropyLoss

        b, s, v = logits.shape
        labels = torch.cat([input_ids[:, 1:], input_ids.new_full((b, 1), -1)], 1).reshape(-1)
        losses = SoftmaxCrossEntropyLoss.apply(logits.reshape(b * s, v), labels, 0.0, -1, True)
        return losses.sum() / (b * (s - 1))
    return F.cross_entropy(logits[:, :-1].reshape(-1, logits.size(-1)).float(),
                           input_ids[:, 1:].reshape(-1))


def gpt2_medium(**kw):
    return GPT2LMHeadModel(GPT2Config(**kw))


def gpt2_small(**kw):
    kw.setdefault("n_embd", 768)
    kw.setdefault("n_layer", 12)
    kw.setdefault("n_head", 12)
    return GPT2LMHeadModel(GPT2Config(**kw))
