// hipBLASLt fused-epilogue GEMMs for the FFN (see lt_ops.cpp).
#pragma once
#include <torch/extension.h>

#include <vector>

namespace amd {

// (h = gelu_tanh(x2 @ w^T + b), pre = x2 @ w^T + b); empty list = no algorithm
std::vector<at::Tensor> dense_gelu_fwd_op(at::Tensor x2, at::Tensor w, at::Tensor b);
// (dpre = (dy2 @ w2) * gelu_tanh'(pre), db = column sums of dpre); empty = no algorithm
std::vector<at::Tensor> dense_dgelu_bgrad_op(at::Tensor dy2, at::Tensor w2, at::Tensor pre,
                                             at::ScalarType bias_dtype);
void lt_algo_cache_clear();

}  // namespace amd
