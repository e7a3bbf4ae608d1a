// Dense-layer helper operators (bias gradients, fused GELU backward).
#pragma once
#include <torch/extension.h>

#include <tuple>

namespace amd {

// sum over rows of a [M, N] tensor (any leading dims) -> [N] in out_dtype
at::Tensor bias_grad_op(at::Tensor g, at::ScalarType out_dtype);
// (dpre = dh * gelu'(pre), sum over rows of dpre); approximate: "none" | "tanh"
std::tuple<at::Tensor, at::Tensor> gelu_bwd_bias_grad_op(at::Tensor dh, at::Tensor pre,
                                                         bool tanh_approx,
                                                         at::ScalarType out_dtype);
// h = gelu(pre) (erf, or tanh when tanh_approx) on the streaming kernel
at::Tensor gelu_fwd_op(at::Tensor x, bool tanh_approx);
// (dpre = dh * act'(y), sum over rows of dpre) from the layer OUTPUT y;
// act: 1 = ReLU (y > 0), 2 = sigmoid (y (1 - y))  [apex.mlp backward]
std::tuple<at::Tensor, at::Tensor> act_bwd_bias_grad_op(at::Tensor dh, at::Tensor y, int64_t act,
                                                        at::ScalarType out_dtype);

}  // namespace amd
