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

// The own 256 x 256 one-wave-per-SIMD MFMA GEMM (csrc/hip/gemm4w.hip): C = A . B^T for
// bf16 / fp16 A [M, K] and B [N, K] (row-major), with the FFN epilogues.  epi 0: [C];
// epi 1: bias + GELU -> [h, pre (when want_pre)]; epi 2: dGELU from aux = pre -> [dpre,
// bias grad (when bias_grad_dtype is given)].  gemm4w_ok: the shape / dtype / layout qualifies.
bool gemm4w_ok(const at::Tensor& a, const at::Tensor& b);
bool wgrad4w_ok(const at::Tensor& dy, const at::Tensor& x, int64_t splits);
std::tuple<at::Tensor, at::Tensor> wgrad4w_bias_op(at::Tensor dy, at::Tensor x, int64_t splits,
                                                   at::ScalarType out_dtype,
                                                   c10::optional<at::Tensor> out, bool accumulate,
                                                   at::ScalarType bias_dtype);
at::Tensor wgrad4w_op(at::Tensor dy, at::Tensor x, int64_t splits, at::ScalarType out_dtype,
                      c10::optional<at::Tensor> out, bool accumulate);
std::vector<at::Tensor> gemm4w_op(at::Tensor a, at::Tensor b, int64_t epi,
                                  c10::optional<at::Tensor> bias, c10::optional<at::Tensor> aux,
                                  bool want_pre, bool tanh_approx,
                                  c10::optional<at::ScalarType> bias_grad_dtype);

}  // namespace amd
