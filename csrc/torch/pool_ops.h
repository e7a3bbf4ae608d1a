#pragma once
#include <ATen/ATen.h>

#include <tuple>

namespace amd {

// NHWC (channels_last) max pooling: forward returns (y, tap index per element).
std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_fwd_op(at::Tensor x, int64_t k, int64_t s,
                                                         int64_t p);
at::Tensor maxpool2d_nhwc_bwd_op(at::Tensor dy, at::Tensor idx, int64_t H, int64_t W, int64_t k,
                                 int64_t s, int64_t p);

// 3x3 stride-1 pad-1 conv, NHWC bf16, implicit GEMM on MFMA (conv_igemm.hip)
at::Tensor conv3x3_nhwc_fwd_op(at::Tensor x, at::Tensor w);
// its weight gradient (split-K MFMA + reduce), returned as [Cout, Cin, 3, 3] channels_last
at::Tensor conv3x3_nhwc_wgrad_op(at::Tensor dy, at::Tensor x, at::ScalarType out_dtype,
                                 int64_t algo);

at::Tensor splitk_reduce_op(at::Tensor part, at::ScalarType out_dtype);
at::Tensor conv3x3_rot_weight_op(at::Tensor w);

}  // namespace amd
