#pragma once
#include <ATen/ATen.h>

#include <tuple>

namespace amd {

// q, k, v: [B, S, H, 64] bf16/fp16 views (head dim contiguous, any other strides).
// Returns o [B, S, H, 64] and the softmax log-sum-exp [B, H, S] (log2 units).
std::tuple<at::Tensor, at::Tensor> attn_fwd_op(at::Tensor q, at::Tensor k, at::Tensor v,
                                               bool causal, double dropout, int64_t seed,
                                               double scale);

}  // namespace amd
