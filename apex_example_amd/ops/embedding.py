"""Embedding lookup whose backward never synchronises the host.

PyTorch's CUDA embedding backward sorts the indices and, for more than 3,072 of
them, reads the number of unique segments back to the host (``.item()``) before it
can size the segment reduction.  That read sits at the very end of a transformer's
backward (the embedding is the first layer), so every step the GPU queue drains
there and the host-side launch work of the optimizer step and the next forward
then runs against an idle GPU: BERT-large showed 4.6 ms of idle GPU time per 51 ms
step in its kernel trace, clustered around the optimizer (``tools/rocprof_summary.py
--gaps``, docs/PERF.md).

Here the weight gradient is deterministic AND host-sync-free
(``csrc/hip/embedding.hip``): a stable device sort of the ids, then one launch with
a wave per sorted position; the wave that starts a run of equal ids sums that run's
output-gradient rows in sorted order (fp32) and writes the weight row in the weight
dtype.  The grid is sized by the token count (known on the host), so nothing is
read back, and the fixed summation order makes it bitwise reproducible (the float-
atomic ``index_add_`` scatter of round 2 was not; it stays selectable as ``_MODE =
"atomic"``, ``"stock"`` is the PyTorch op).  Forward is the regular gather.
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

# backward: "det" (default) | "atomic" | "stock"
_MODE = "det"
_ENABLED = _MODE != "stock"


# dtypes the deterministic kernel reads / writes (anything else: the scatter below)
_DET_DTYPES = (torch.float32, torch.float16, torch.bfloat16)


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, weight, padding_idx):
        ctx.save_for_backward(idx)
        ctx.shape = weight.shape
        ctx.wdtype = weight.dtype
        ctx.padding_idx = padding_idx
        return F.embedding(idx, weight, padding_idx)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        V, H = ctx.shape
        if _MODE == "det" and dy.dtype in _DET_DTYPES and ctx.wdtype in _DET_DTYPES:
            pad = -1 if ctx.padding_idx is None else int(ctx.padding_idx) % V
            return None, _native.require().emb.wgrad(idx, dy, V, pad, ctx.wdtype), None
        flat = idx.reshape(-1)
        acc = torch.promote_types(dy.dtype, torch.float32)  # fp64 stays fp64
        g = torch.zeros((V, H), dtype=acc, device=dy.device)
        g.index_add_(0, flat, dy.reshape(-1, H).to(acc))
        if ctx.padding_idx is not None:
            g[ctx.padding_idx].zero_()
        return None, g.to(ctx.wdtype), None


class Embedding(nn.Embedding):
    """``nn.Embedding`` with a host-sync-free backward on the GPU (dense gradients,
    no ``max_norm`` / ``scale_grad_by_freq`` / sparse: those fall back to the stock
    op)."""

    def forward(self, idx):
        if (_ENABLED and idx.is_cuda and not self.sparse and self.max_norm is None
                and not self.scale_grad_by_freq and torch.is_grad_enabled()
                and self.weight.requires_grad):
            return _EmbeddingFn.apply(idx, self.weight, self.padding_idx)
        return super().forward(idx)
