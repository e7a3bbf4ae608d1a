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
// (dW = dy2^T x2 in w_dtype, db = column sums of dy2) from one BGRADB GEMM
std::vector<at::Tensor> dense_wgrad_bgrad_op(at::Tensor dy2, at::Tensor x2,
                                             at::ScalarType w_dtype, at::ScalarType bias_dtype);
void lt_algo_cache_clear();
int64_t lt_probe_op(int64_t m, int64_t n, int64_t k, int64_t epilogue, int64_t ta, int64_t tb,
                    at::ScalarType dtype, int64_t aux_type, int64_t bias_type);

}  // namespace amd
