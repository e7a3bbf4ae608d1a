"""Fused multi-layer perceptron (apex.mlp.MLP).

``MLP(mlp_sizes, bias=True, activation='relu')`` = a chain of
Linear(+bias)(+activation) layers run as ONE autograd function: the forward
keeps only each layer's output (Apex's reserved-space scheme), the backward
walks the chain with one dgrad GEMM, one wgrad GEMM and one bias reduction per
layer and no autograd graph per op.

MI355X mapping: the forward GEMM + bias + ReLU is a single hipBLASLt call with
the RELU_BIAS epilogue (``torch._addmm_activation``), so the activation never
makes its own pass over HBM; sigmoid / none use the BIAS epilogue (addmm) plus
one elementwise pass.  Backward per layer: ONE pass of the gfx950 column-sum
kernel (csrc/hip/bias_grad.hip, ``dense.act_bwd_bias_grad``) forms the
pre-activation gradient from the saved output (relu: out > 0; sigmoid:
out * (1 - out)) AND its column sums (the bias gradient) - the mask multiply
and the bias reduction never make separate passes - then the dgrad and wgrad
GEMMs (hipBLASLt; wgrad written in the weight dtype by the GEMM).
Weights are [out, in] like nn.Linear, initialised as Apex's MLP
(normal(0, sqrt(2/(fan_in+fan_out))), bias normal(0, sqrt(1/fan_out))).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _native

_ACTS = {"none": 0, "relu": 1, "sigmoid": 2}


def _fwd_layer(x, w, b, act, last):
    a = 0 if last and act == 0 else act
    if b is not None and a == 1 and x.is_cuda:
        return torch._addmm_activation(b, x, w.t(), use_gelu=False)
    y = torch.addmm(b, x, w.t()) if b is not None else x.mm(w.t())
    if a == 1:
        y = torch.relu_(y)
    elif a == 2:
        y = torch.sigmoid_(y)
    return y


class MlpFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bias, activation, x, *params):
        n = len(params) // (2 if bias else 1)
        ws = params[:n]
        bs = params[n:] if bias else [None] * n
        outs = [x]
        h = x
        for i in range(n):
            h = _fwd_layer(h, ws[i], bs[i], activation, last=False)
            outs.append(h)
        ctx.bias = bias
        ctx.activation = activation
        ctx.n = n
        ctx.save_for_backward(*outs, *params)
        return h

    @staticmethod
    def backward(ctx, grad):
        saved = ctx.saved_tensors
        n = ctx.n
        outs = saved[: n + 1]
        params = saved[n + 1:]
        ws = params[:n]
        act = ctx.activation
        gw = [None] * n
        gb = [None] * n
        bs = params[n:] if ctx.bias else [None] * n
        g = grad.contiguous()
        native = g.is_cuda and _native.available()
        for i in reversed(range(n)):
            y = outs[i + 1]
            bdt = bs[i].dtype if bs[i] is not None else g.dtype
            if act in (1, 2) and native:
                g, db = _native.require().dense.act_bwd_bias_grad(g, y, act, bdt)
            else:
                if act == 1:
                    g = g * (y > 0).to(g.dtype)
                elif act == 2:
                    g = g * y * (1 - y)
                db = None
                if ctx.bias:
                    db = (_native.require().dense.bias_grad(g, bdt) if native
                          else g.sum(0, dtype=torch.promote_types(g.dtype, torch.float32))
                          .to(bdt))
            if ctx.bias:
                gb[i] = db
            gw[i] = g.t().mm(outs[i])
            g = g.mm(ws[i]) if (i > 0 or ctx.needs_input_grad[2]) else None
        grads = gw + (gb if ctx.bias else [])
        return (None, None, g, *grads)


class MLP(nn.Module):
    def __init__(self, mlp_sizes, bias=True, activation="relu"):
        super().__init__()
        if activation not in _ACTS:
            raise TypeError("activation must be one of %s" % sorted(_ACTS))
        self.num_layers = len(mlp_sizes) - 1
        self.mlp_sizes = list(mlp_sizes)
        self.bias = 1 if bias else 0
        self.activation = _ACTS[activation]
        self.weights = nn.ParameterList()
        self.biases = nn.ParameterList()
        for i in range(self.num_layers):
            self.weights.append(nn.Parameter(torch.empty(mlp_sizes[i + 1], mlp_sizes[i])))
            if bias:
                self.biases.append(nn.Parameter(torch.empty(mlp_sizes[i + 1])))
        self.reset_parameters()

    def reset_parameters(self):
        for w in self.weights:
            fan_out, fan_in = w.shape
            nn.init.normal_(w, 0.0, math.sqrt(2.0 / (fan_in + fan_out)))
        for b in self.biases:
            nn.init.normal_(b, 0.0, math.sqrt(1.0 / b.numel()))

    def forward(self, x):
        return MlpFunction.apply(bool(self.bias), self.activation, x, *self.weights,
                                 *self.biases)

    def extra_repr(self):
        act = {v: k for k, v in _ACTS.items()}[self.activation]
        return "MLP sizes: %s, Bias=%s, activation=%s" % (self.mlp_sizes, bool(self.bias), act)
