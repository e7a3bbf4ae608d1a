"""FusedLayerNorm / FusedRMSNorm (apex@f3a960f8 apex/normalization/fused_layer_norm.py,
SURVEY.md A-13 / N-13) on the wave64 row kernels of csrc/hip/layer_norm.hip.

Inputs may be fp32 / fp16 / bf16; gamma/beta may be fp32 with 16-bit inputs
("mixed" - amp O2 keeps LayerNorm params... in the model dtype by default;
either works).  CPU tensors run the C++ CPU path of the same extension.
"""
from __future__ import annotations

import numbers

import torch
from torch.nn import init
from torch.nn.parameter import Parameter

from .. import _native
from ..ops import _bias_handoff


def _n2(normalized_shape):
    n = 1
    for s in normalized_shape:
        n *= s
    return n


class FusedLayerNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps):
        C = _native.require().layer_norm
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        input_ = input.contiguous()
        weight_ = weight.contiguous()
        bias_ = bias.contiguous()
        output, mean, invvar = C.forward(input_, _n2(normalized_shape), weight_, bias_, eps, False)
        ctx.save_for_backward(input_, weight_, bias_, mean, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        C = _native.require().layer_norm
        input_, weight_, bias_, mean, invvar = ctx.saved_tensors
        grad_input, grad_weight, grad_bias = C.backward(
            grad_output.contiguous(), input_, mean, invvar, _n2(ctx.normalized_shape), weight_,
            ctx.needs_input_grad[1], ctx.needs_input_grad[2], False)
        return grad_input, grad_weight, grad_bias, None, None


class FusedLayerNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, normalized_shape, eps):
        C = _native.require().layer_norm
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        input_ = input.contiguous()
        output, mean, invvar = C.forward(input_, _n2(normalized_shape), None, None, eps, False)
        ctx.save_for_backward(input_, mean, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        C = _native.require().layer_norm
        input_, mean, invvar = ctx.saved_tensors
        grad_input, _, _ = C.backward(grad_output.contiguous(), input_, mean, invvar,
                                      _n2(ctx.normalized_shape), None, False, False, False)
        return grad_input, None, None


class FusedRMSNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, normalized_shape, eps):
        C = _native.require().layer_norm
        ctx.normalized_shape = normalized_shape
        input_ = input.contiguous()
        weight_ = weight.contiguous()
        output, mean, invvar = C.forward(input_, _n2(normalized_shape), weight_, None, eps, True)
        ctx.save_for_backward(input_, weight_, mean, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        C = _native.require().layer_norm
        input_, weight_, mean, invvar = ctx.saved_tensors
        grad_input, grad_weight, _ = C.backward(grad_output.contiguous(), input_, mean, invvar,
                                                _n2(ctx.normalized_shape), weight_,
                                                ctx.needs_input_grad[1], False, True)
        return grad_input, grad_weight, None, None


def _dropout_seed() -> int:
    # per-call seed from torch's CPU generator: no device sync, follows torch.manual_seed
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


class AddDropoutLayerNormFunction(torch.autograd.Function):
    """(y, s) = (LN(s), s) with s = x + dropout_p(h), one gfx950 kernel each way.

    Forward reads h and x once and writes s and y (the unfused chain - dropout,
    residual add, LayerNorm - reads/writes ~7.5 activations; this 4).  The keep
    mask is a counter hash of (seed, element) regenerated in the backward, which
    returns ds = LN'(dy) + ds_ext (the residual-stream gradient) and dh = dropout'(ds)
    in the same pass as dgamma/dbeta partials.
    """

    @staticmethod
    def forward(ctx, x, h, weight, bias, normalized_shape, eps, p, y_as_h=False):
        C = _native.require().layer_norm
        n2 = _n2(normalized_shape)
        seed = _dropout_seed() if p > 0.0 else 0
        y, s, mean, invvar = C.add_dropout_forward(x, h, n2, weight, bias, eps, p, seed,
                                                   bool(y_as_h))
        # an unused output (post-LN callers drop s) gets grad None, not a zero fill + read
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(s, weight, mean, invvar)
        ctx.cfg = (n2, float(p), seed, h.dtype if h.dtype != x.dtype else None)
        return y, s

    @staticmethod
    def backward(ctx, dy, ds_ext):
        C = _native.require().layer_norm
        s, weight, mean, invvar = ctx.saved_tensors
        n2, p, seed, h_dtype = ctx.cfg
        if dy is None:
            dy = torch.zeros_like(s)
        # the column sums of dh (the producing dense layer's bias gradient) ride on the
        # dgamma / dbeta partials: ops/_bias_handoff.py
        want_hs = (_bias_handoff.ENABLED and ctx.needs_input_grad[1] and weight is not None
                   and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3]))
        ds, dh, dw, db, dhs = C.add_dropout_backward(dy, s, mean, invvar, n2, weight, ds_ext, p,
                                                     seed, ctx.needs_input_grad[2],
                                                     ctx.needs_input_grad[3], h_dtype,
                                                     bool(want_hs))
        if want_hs:
            _bias_handoff.offer(dh, dhs)
        return ds, dh, dw, db, None, None, None, None


_FUSED_ADD_LN = True  # (tests turn it off to compare with the unfused sublayer join)


def _fused_add_ok(x, h, ln):
    n2 = _n2(ln.normalized_shape)
    # h may be 16-bit under an fp32 residual stream (amp O1): read / written as is
    mixed = x.dtype == torch.float32 and h.dtype in (torch.float16, torch.bfloat16)
    return (_FUSED_ADD_LN and isinstance(ln, FusedLayerNorm) and x.is_cuda and h.is_cuda
            and (x.dtype == h.dtype or mixed) and x.shape == h.shape
            and x.dtype in (torch.float16, torch.bfloat16, torch.float32)
            and n2 % 8 == 0 and n2 <= 2048 and x.shape[-1] == n2 and ln.elementwise_affine
            and ln.weight.dtype == ln.bias.dtype and _native.available())


def fused_add_dropout_layer_norm(x, h, ln, p=0.0, training=True, y_as_h=False):
    """(LN(s), s) for s = x + dropout(h, p): the residual join of a transformer
    sublayer (post-LN BERT uses y, pre-LN GPT-2 keeps s as the residual stream).
    ``ln`` is a FusedLayerNorm / nn.LayerNorm module (its weight, bias, eps).
    Falls back to the unfused PyTorch chain on CPU or unsupported shapes/dtypes.
    ``y_as_h``: with an fp32 residual and a 16-bit ``h`` (amp O1) return y in h's
    dtype - for a consumer that is an autocast GEMM, which would cast it anyway."""
    p = float(p) if training else 0.0
    if _fused_add_ok(x, h, ln):
        return AddDropoutLayerNormFunction.apply(x, h, ln.weight, ln.bias, ln.normalized_shape,
                                                 ln.eps, p, y_as_h and h.dtype != x.dtype)
    s = x + torch.nn.functional.dropout(h, p, training=p > 0.0)
    return ln(s), s


def fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6):
    return FusedLayerNormAffineFunction.apply(input, weight, bias, normalized_shape, eps)


def fused_layer_norm(input, normalized_shape, eps=1e-6):
    return FusedLayerNormFunction.apply(input, normalized_shape, eps)


def fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6):
    return FusedRMSNormAffineFunction.apply(input, weight, normalized_shape, eps)


class FusedLayerNorm(torch.nn.Module):
    r"""Applies Layer Normalization over a mini-batch of inputs (apex.normalization.FusedLayerNorm).

    .. math::
        y = \frac{x - \mathrm{E}[x]}{ \sqrt{\mathrm{Var}[x] + \epsilon}} * \gamma + \beta

    Same constructor and semantics as ``torch.nn.LayerNorm``; CPU input without
    the extension falls back to ``F.layer_norm`` (apex behaviour).
    """

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True):
        super(FusedLayerNorm, self).__init__()
        if isinstance(normalized_shape, numbers.Integral):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = torch.Size(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        if self.elementwise_affine:
            self.weight = Parameter(torch.Tensor(*normalized_shape))
            self.bias = Parameter(torch.Tensor(*normalized_shape))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)
            init.zeros_(self.bias)

    def forward(self, input):
        if not input.is_cuda and not _native.available():
            return torch.nn.functional.layer_norm(input, self.normalized_shape, self.weight,
                                                  self.bias, self.eps)
        if self.elementwise_affine:
            return FusedLayerNormAffineFunction.apply(input, self.weight, self.bias,
                                                      self.normalized_shape, self.eps)
        return FusedLayerNormFunction.apply(input, self.normalized_shape, self.eps)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(
            **self.__dict__)


class FusedRMSNorm(torch.nn.Module):
    r"""RMS normalization: y = x / sqrt(mean(x^2) + eps) * gamma."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True):
        super().__init__()
        if isinstance(normalized_shape, numbers.Integral):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = torch.Size(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        if elementwise_affine:
            self.weight = Parameter(torch.ones(*normalized_shape))
        else:
            self.register_parameter("weight", None)

    def forward(self, input):
        if self.elementwise_affine:
            return FusedRMSNormAffineFunction.apply(input, self.weight, self.normalized_shape,
                                                    self.eps)
        w = torch.ones(self.normalized_shape, dtype=input.dtype, device=input.device)
        return FusedRMSNormAffineFunction.apply(input, w, self.normalized_shape, self.eps)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(
            **self.__dict__)
