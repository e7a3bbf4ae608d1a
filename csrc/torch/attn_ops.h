// Torch bindings for the fused attention kernels (csrc/hip/attention.hip).
#pragma once
#include <ATen/ATen.h>

#include <tuple>

namespace amd {

// q, k, v: [B, S, H, 64] bf16/fp16 views (head dim contiguous, 16-B aligned rows).
// Returns (o [B, S, H, 64] contiguous, lse [B, H, S] fp32 log2 units; a view of a
// row-padded [B, H, round_up(S, 64)] buffer).
std::tuple<at::Tensor, at::Tensor> attn_fwd_op(at::Tensor q, at::Tensor k, at::Tensor v,
                                               bool causal, double dropout, int64_t seed,
                                               double scale);

// Writes dq, dk, dv (caller-allocated [B, S, H, 64] views, e.g. slices of one
// packed dqkv buffer) from dout, the forward inputs, o and lse.
void attn_bwd_op(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o,
                 at::Tensor lse, bool causal, double dropout, int64_t seed, double scale,
                 at::Tensor dq, at::Tensor dk, at::Tensor dv);

}  // namespace amd
