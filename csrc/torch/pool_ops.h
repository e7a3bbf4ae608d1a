#pragma once
#include <ATen/ATen.h>
#include <c10/util/Optional.h>

#include <tuple>

namespace amd {

// NHWC (channels_last) max pooling: forward returns (y, tap index per element).
std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_fwd_op(at::Tensor x, int64_t k, int64_t s,
                                                         int64_t p);
// the same with a BatchNorm affine + ReLU applied to x on load (ResNet stem)
std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_bn_fwd_op(
    at::Tensor x, c10::optional<at::Tensor> mean, c10::optional<at::Tensor> invstd,
    c10::optional<at::Tensor> w, c10::optional<at::Tensor> b, int64_t k, int64_t s, int64_t p);
at::Tensor maxpool2d_nhwc_bwd_op(at::Tensor dy, at::Tensor idx, int64_t H, int64_t W, int64_t k,
                                 int64_t s, int64_t p);
at::Tensor gap_nhwc_bwd_op(at::Tensor dy, int64_t H, int64_t W);

// 3x3 / 1x1 convs (stride 1 or 2), NHWC bf16, implicit GEMM on MFMA (conv_igemm.hip)
at::Tensor conv_nhwc_fwd_op(at::Tensor x, at::Tensor w, int64_t stride);
// forward conv that also writes the consuming BatchNorm's per-tile statistics:
// returns (y, slab [S][2][Cout] fp32); shift: that BN's running mean (or None)
std::tuple<at::Tensor, at::Tensor> conv_nhwc_fwd_stats_op(at::Tensor x, at::Tensor w,
                                                          int64_t stride,
                                                          c10::optional<at::Tensor> shift);
std::tuple<at::Tensor, at::Tensor> conv_nhwc_fwd_bnbwd_op(
    at::Tensor dy, at::Tensor w, c10::optional<at::Tensor> add, at::Tensor xbn,
    c10::optional<at::Tensor> rmask, at::Tensor mean, at::Tensor invstd,
    c10::optional<at::Tensor> bn_w, c10::optional<at::Tensor> bn_b, int64_t relu_mode,
    bool add_stride2 = false);
at::Tensor conv_nhwc_dgrad_s2_op(at::Tensor dy, at::Tensor wt, int64_t H, int64_t W);
at::Tensor conv_nhwc_wgrad_op(at::Tensor dy, at::Tensor x, at::ScalarType out_dtype, int64_t algo,
                              int64_t stride, int64_t ksize, c10::optional<at::Tensor> out, bool accumulate = true);
at::Tensor splitk_reduce_op(at::Tensor part, at::ScalarType out_dtype,
                            c10::optional<at::Tensor> out_acc, bool accumulate = true);
at::Tensor stem_pad_op(at::Tensor x);
at::Tensor stem_fwd_op(at::Tensor xp, at::Tensor wk);
std::tuple<at::Tensor, at::Tensor> conv_nhwc_dgrad_s2_bnbwd_op(
    at::Tensor dy, at::Tensor wt, int64_t H, int64_t W, at::Tensor xbn,
    c10::optional<at::Tensor> rmask, at::Tensor mean, at::Tensor invstd,
    c10::optional<at::Tensor> bn_w, c10::optional<at::Tensor> bn_b, int64_t relu_mode);
std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_bwd_bn_op(at::Tensor dy, at::Tensor idx,
                                                            int64_t H, int64_t W, at::Tensor x,
                                                            at::Tensor mean, at::Tensor invstd,
                                                            c10::optional<at::Tensor> weight,
                                                            c10::optional<at::Tensor> bias);
std::tuple<at::Tensor, at::Tensor> stem_fwd_stats_op(at::Tensor xp, at::Tensor wk,
                                                     c10::optional<at::Tensor> shift);
at::Tensor stem_wgrad_op(at::Tensor xp, at::Tensor dy);
at::Tensor conv3x3_rot_weight_op(at::Tensor w);
at::Tensor conv1x1_transpose_weight_op(at::Tensor w);
std::vector<at::Tensor> conv_prep_weights_op(std::vector<at::Tensor> ws);

}  // namespace amd
