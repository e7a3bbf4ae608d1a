#pragma once
#include <ATen/ATen.h>
#include <c10/util/Optional.h>

#include <tuple>

namespace amd {

using OptT = c10::optional<at::Tensor>;

// LayerNorm / RMSNorm over the trailing `n2` elements of x.
std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_forward_op(at::Tensor x, int64_t n2,
                                                                     OptT gamma, OptT beta,
                                                                     double eps, bool rms);
std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_backward_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invvar, int64_t n2, OptT gamma,
    bool need_wgrad, bool need_bgrad, bool rms);

// Residual + dropout + LayerNorm (GPU): s = x + dropout_p(h) with counter-hash keep
// bits from `seed`, y = LN(s).  Returns (y, s, mean, invvar).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> add_dropout_layer_norm_forward_op(
    at::Tensor x, at::Tensor h, int64_t n2, OptT gamma, OptT beta, double eps, double p,
    int64_t seed, bool y_as_h);
// -> (ds = LN'(dy) + dres, dh = dropout'(ds), dgamma, dbeta, colsum(dh) if need_hsum)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
add_dropout_layer_norm_backward_op(at::Tensor dy, at::Tensor s, at::Tensor mean, at::Tensor invvar,
                                   int64_t n2, OptT gamma, OptT dres, double p, int64_t seed,
                                   bool need_wgrad, bool need_bgrad,
                                   c10::optional<at::ScalarType> h_dtype, bool need_hsum);

// BatchNorm building blocks (local / synchronized).
std::tuple<at::Tensor, at::Tensor> bn_local_stats_op(at::Tensor x);
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_combine_stats_op(at::Tensor means,
                                                                   at::Tensor vars,
                                                                   at::Tensor counts, double eps,
                                                                   double momentum,
                                                                   OptT running_mean,
                                                                   OptT running_var);
// Local (per-GPU statistics) training forward: stats + running-stat update +
// num_batches_tracked += 1 + normalize(+z)(+ReLU).  Returns (y, mean, invstd).
// want_mask: also return the ReLU bitmask [M, C/8] uint8 (channels-last GPU input
// with C % 8 == 0 and relu; otherwise the 4th result is undefined / None).
// SyncBN: packed local stats [mean | var | count] and the combine of the gathered
// [world, 2C+1] stats -> (mean, invstd, 1/global count)
at::Tensor bn_local_stats_packed_op(at::Tensor x, OptT out = c10::nullopt);
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_combine_stats_sync_op(
    at::Tensor gathered, double eps, double momentum, OptT running_mean, OptT running_var,
    OptT nbt);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_forward_local_op(
    at::Tensor x, OptT weight, OptT bias, OptT running_mean, OptT running_var, OptT nbt,
    double eps, double momentum, OptT z, bool relu, bool want_mask);
at::Tensor bn_apply_op(at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
                       OptT z, bool relu);
// (mean, invstd) of a training batch; running stats / counter updated on the device
std::tuple<at::Tensor, at::Tensor> bn_train_stats_op(at::Tensor x, OptT running_mean,
                                                      OptT running_var, OptT nbt, double eps,
                                                      double momentum);
std::tuple<at::Tensor, at::Tensor> bn_apply_mask_op(at::Tensor x, at::Tensor mean,
                                                    at::Tensor invstd, OptT weight, OptT bias,
                                                    OptT z, bool relu);
// mask: the forward's ReLU bitmask; when given, z is not read.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_reduce_grad_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
    OptT z, bool relu, bool need_wgrad, OptT mask,
    OptT sum_scale, OptT grad_weight = c10::nullopt, OptT grad_bias = c10::nullopt,
    bool accumulate = true);
std::tuple<at::Tensor, at::Tensor> bn_backward_elemt_op(at::Tensor dy, at::Tensor x,
                                                        at::Tensor mean, at::Tensor invstd,
                                                        OptT weight, OptT bias, at::Tensor sum_dy,
                                                        at::Tensor sum_dy_xmu, double count,
                                                        OptT z, bool relu, bool want_dz,
                                                        OptT mask);

bool bn_backward_x2_ok(at::Tensor dy, at::Tensor x, at::Tensor x2);
std::tuple<at::Tensor, at::Tensor> bn_apply2_mask_op(at::Tensor x, at::Tensor mean,
                                                     at::Tensor invstd, OptT weight, OptT bias,
                                                     at::Tensor xz, at::Tensor meanz,
                                                     at::Tensor invstdz, OptT weightz,
                                                     OptT biasz);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_backward_elemt_x2_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
    at::Tensor sum_dy, at::Tensor sum_dy_xmu, double count, at::Tensor x2, at::Tensor mean2,
    at::Tensor invstd2, OptT weight2, bool need_wgrad2);

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_backward_local_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
    OptT z, bool relu, bool need_wgrad, bool want_dz, OptT mask);

// BatchNorm statistics from a producer's channel-major stats slab [2][C][S]
// (conv.conv_fwd_stats): local training mode -> (mean, invstd) with the running-stat
// and num_batches_tracked updates; packed mode -> [mean | biased var | count] (SyncBN)
std::tuple<at::Tensor, at::Tensor> bn_slab_train_stats_op(at::Tensor slab, int64_t count,
                                                          OptT shift, OptT running_mean,
                                                          OptT running_var, OptT nbt,
                                                          double eps, double momentum);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_slab_reduce_grad_op(
    at::Tensor slab, at::Tensor invstd, OptT weight, bool need_wgrad, OptT sum_scale,
    OptT grad_weight = c10::nullopt, OptT grad_bias = c10::nullopt, bool accumulate = true);
at::Tensor bn_slab_packed_stats_op(at::Tensor slab, int64_t count, OptT shift,
                                   OptT out = c10::nullopt);

}  // namespace amd
