"""Channels-last max pooling on the gfx950 kernels (csrc/hip/pool.hip).

The forward keeps a one-byte tap index per output element; the backward is a
gather over the windows covering each input pixel (no atomics, every dx
element written once), replacing ATen's NHWC max_pool2d kernels, which cost
~0.9 ms per ResNet-50 step at bs 256 on MI355X (profiles/).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native


class MaxPool2dNHWCFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = _native.require().pool.max_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geom = (x.size(2), x.size(3), k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.geom
        return _native.require().pool.max_bwd(dy, idx, H, W, k, s, p), None, None, None


class MaxPool2dNHWC(nn.MaxPool2d):
    """nn.MaxPool2d whose channels-last GPU path runs the gfx950 kernels."""

    def forward(self, x):
        k, s, p = self.kernel_size, self.stride, self.padding
        if (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
                and isinstance(k, int) and isinstance(s, int) and isinstance(p, int)
                and self.dilation == 1 and not self.ceil_mode and not self.return_indices
                and p <= k // 2 and k <= 15):
            return MaxPool2dNHWCFunction.apply(x, k, s, p)
        return F.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.dilation,
                            self.ceil_mode, self.return_indices)
