// Torch bindings for the fused softmax cross entropy (csrc/hip/xentropy.hip).
#pragma once
#include <ATen/ATen.h>

#include <tuple>

namespace amd {

// logits [N, V], labels [N] int64 -> (losses [N] (fp32 if half_to_float else
// logits dtype), max_log_sum_exp [N] fp32)
std::tuple<at::Tensor, at::Tensor> xentropy_fwd_op(at::Tensor logits, at::Tensor labels,
                                                   double smoothing, int64_t padding_idx,
                                                   bool half_to_float);
at::Tensor xentropy_bwd_op(at::Tensor grad_loss, at::Tensor logits, at::Tensor lse,
                           at::Tensor labels, double smoothing, int64_t padding_idx);

}  // namespace amd
