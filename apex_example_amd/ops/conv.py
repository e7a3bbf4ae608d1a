"""1x1 convolution as a plain GEMM on channels-last activations.

A stride-1 1x1 convolution over an NHWC tensor is exactly
``y[M, Cout] = x[M, Cin] @ W[Cout, Cin]^T`` with M = N*H*W, and the activation is
already that matrix in memory (channels_last), so forward and data-gradient are
library GEMMs (hipBLASLt via ``torch.mm``) with no layout change.  Measured on
MI355X at ResNet-50 bs256 shapes (tools/microbench.py conv1x1, docs/PERF.md),
hipBLASLt beats MIOpen's 1x1 forward/dgrad kernels by 1.2-4x; MIOpen's weight
gradient (long-K reduction over M) stays faster than the GEMM library's choice,
so the weight gradient keeps the MIOpen path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _as_rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


class Conv1x1GemmFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        n, ci, h, w = x.shape
        co = weight.shape[0]
        w2 = weight.reshape(co, ci)
        y2 = torch.mm(_as_rows(x), w2.t())
        ctx.save_for_backward(x, weight)
        return y2.view(n, h, w, co).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        n, ci, h, w = x.shape
        co = weight.shape[0]
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx2 = torch.mm(_as_rows(dy), weight.reshape(co, ci))
            dx = dx2.view(n, h, w, ci).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            dw = torch.ops.aten.convolution_backward(
                dy, x, weight, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
                (False, True, False))[1]
        return dx, dw


class Conv1x1SkipFunction(torch.autograd.Function):
    """(y, skip) = (conv1x1(x), x): the 1x1 GEMM convolution that also hands its
    input on as the residual branch of a bottleneck block.  Backward receives
    both gradients and forms dx = dskip + dy @ W as ONE GEMM with beta = 1
    (hipBLASLt accumulates into C), replacing conv-dgrad + a separate
    elementwise add over the block input (the residual-gradient sum autograd
    would otherwise launch)."""

    @staticmethod
    def forward(ctx, x, weight):
        n, ci, h, w = x.shape
        co = weight.shape[0]
        y2 = torch.mm(_as_rows(x), weight.reshape(co, ci).t())
        ctx.save_for_backward(x, weight)
        return y2.view(n, h, w, co).permute(0, 3, 1, 2), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        x, weight = ctx.saved_tensors
        n, ci, h, w = x.shape
        co = weight.shape[0]
        dx = dw = None
        if dy is not None:
            dy = dy.contiguous(memory_format=torch.channels_last)
        if ctx.needs_input_grad[0]:
            if dy is None:
                dx = dskip
            else:
                w2 = weight.reshape(co, ci)
                if dskip is not None:
                    # accumulate in place into the residual gradient (a fresh buffer
                    # from the BN backward): C += dy @ W, no copy of C first
                    dskip = dskip.contiguous(memory_format=torch.channels_last)
                    dx2 = _as_rows(dskip).addmm_(_as_rows(dy), w2)
                else:
                    dx2 = torch.mm(_as_rows(dy), w2)
                dx = dx2.view(n, h, w, ci).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] and dy is not None:
            dw = torch.ops.aten.convolution_backward(
                dy, x, weight, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
                (False, True, False))[1]
        return dx, dw


class Conv2d1x1(nn.Conv2d):
    """nn.Conv2d(kernel_size=1) whose stride-1 channels-last GPU path runs as a
    GEMM; every other case falls back to the regular convolution."""

    def __init__(self, in_planes, out_planes, stride=1, bias=False):
        super().__init__(in_planes, out_planes, kernel_size=1, stride=stride, bias=bias)

    def forward(self, x):
        if self._gemm_ok(x):
            return Conv1x1GemmFunction.apply(x, self.weight)
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation,
                        self.groups)

    def forward_with_skip(self, x):
        """(conv(x), x) with the residual-gradient add fused into the dgrad GEMM."""
        if self._gemm_ok(x):
            return Conv1x1SkipFunction.apply(x, self.weight)
        return self.forward(x), x

    def _gemm_ok(self, x):
        return (self.stride == (1, 1) and self.bias is None and x.is_cuda and x.dim() == 4
                and x.is_contiguous(memory_format=torch.channels_last)
                and x.dtype == self.weight.dtype and self.groups == 1)
