// Torch bindings for the NHWC max-pooling kernels (csrc/hip/pool.hip).
#include <cstdlib>
#include "pool_ops.h"

#include "common.h"

namespace amd {

namespace {
int64_t out_size(int64_t in, int64_t k, int64_t s, int64_t p) { return (in + 2 * p - k) / s + 1; }
}  // namespace

std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_fwd_op(at::Tensor x, int64_t k, int64_t s,
                                                         int64_t p) {
  return maxpool2d_nhwc_bn_fwd_op(x, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, k, s,
                                  p);
}

std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_bn_fwd_op(
    at::Tensor x, c10::optional<at::Tensor> mean, c10::optional<at::Tensor> invstd,
    c10::optional<at::Tensor> w, c10::optional<at::Tensor> b, int64_t k, int64_t s, int64_t p) {
  c10::NoGradGuard no_grad_;
  auto f32 = [&](const c10::optional<at::Tensor>& t) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->is_cuda() &&
                    t->numel() == x.size(1),
                "maxpool BN operands: contiguous fp32 [C] GPU tensors");
    return t->data_ptr<float>();
  };
  const float* mp = f32(mean);
  const float* ip = f32(invstd);
  TORCH_CHECK((mp == nullptr) == (ip == nullptr), "maxpool BN: mean and invstd go together");
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, "maxpool2d_nhwc: 4-D GPU tensor expected");
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && p >= 0 && p <= k / 2, "unsupported pool geometry");
  x = x.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = out_size(H, k, s, p), OW = out_size(W, k, s, p);
  TORCH_CHECK(OH > 0 && OW > 0, "pool output is empty");
  auto opt = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  at::Tensor y = at::empty({N, C, OH, OW}, opt);
  at::Tensor idx = at::empty({N, C, OH, OW}, opt.dtype(at::kByte));
  maxpool2d_nhwc_fwd(x.data_ptr(), dtype_of(x), y.data_ptr(), idx.data_ptr<uint8_t>(), (int)N,
                     (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p,
                     cur_stream(), mp, ip, f32(w), f32(b));
  return {y, idx};
}

at::Tensor maxpool2d_nhwc_bwd_op(at::Tensor dy, at::Tensor idx, int64_t H, int64_t W, int64_t k,
                                 int64_t s, int64_t p) {
  c10::NoGradGuard no_grad_;
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  idx = idx.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == at::kByte, "bad pool index");
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  maxpool2d_nhwc_bwd(dy.data_ptr(), idx.data_ptr<uint8_t>(), dtype_of(dy), dx.data_ptr(), (int)N,
                     (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p,
                     cur_stream());
  return dx;
}

// the fused stem's max-pool backward with the BatchNorm + ReLU backward sums (slab [2][64][S]
// for bn.slab_reduce_grad); null when the shape is not the stem's (the caller falls back)
std::tuple<at::Tensor, at::Tensor> maxpool2d_nhwc_bwd_bn_op(at::Tensor dy, at::Tensor idx,
                                                            int64_t H, int64_t W, at::Tensor x,
                                                            at::Tensor mean, at::Tensor invstd,
                                                            c10::optional<at::Tensor> weight,
                                                            c10::optional<at::Tensor> bias) {
  c10::NoGradGuard no_grad_;
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  idx = idx.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  TORCH_CHECK(idx.sizes() == dy.sizes() && idx.scalar_type() == at::kByte, "bad pool index");
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(0) == N && x.size(1) == C && x.size(2) == H &&
                  x.size(3) == W && x.scalar_type() == dy.scalar_type() &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "max_bwd_bn: x must be the pooled BN input [N, C, H, W], channels-last, dy's dtype");
  TORCH_CHECK(dy.element_size() == 2 &&
                  maxpool2d_nhwc_bwd_bn_ok((int)H, (int)W, (int)C, (int)OH, (int)OW, 3, 2, 1),
              "max_bwd_bn: 3x3 / stride-2 / pad-1 pooling of 64 16-bit channels only");
  auto f32c = [&](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.numel() == C && t.is_contiguous(),
                "max_bwd_bn: ", what, " must be fp32 [C]");
    return t.data_ptr<float>();
  };
  const float* mp = f32c(mean, "mean");
  const float* ip = f32c(invstd, "invstd");
  const float* wp = weight.has_value() && weight->defined() ? f32c(*weight, "weight") : nullptr;
  const float* bp = bias.has_value() && bias->defined() ? f32c(*bias, "bias") : nullptr;
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor slab = at::empty({2, C, (int64_t)maxpool_bwd_bn_grid((int)N, (int)H, (int)W)},
                              dy.options().dtype(at::kFloat));
  TORCH_CHECK((uintptr_t)dy.data_ptr() % 16 == 0 && (uintptr_t)dx.data_ptr() % 16 == 0 &&
                  (uintptr_t)x.data_ptr() % 16 == 0 && (uintptr_t)idx.data_ptr() % 8 == 0,
              "max_bwd_bn: 16-byte aligned tensors expected");
  maxpool2d_nhwc_bwd_bn(dy.data_ptr(), idx.data_ptr<uint8_t>(), dtype_of(dy), dx.data_ptr(),
                        (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW, x.data_ptr(), mp, ip,
                        wp, bp, slab.data_ptr<float>(), cur_stream());
  return {dx, slab};
}

at::Tensor gap_nhwc_bwd_op(at::Tensor dy, int64_t H, int64_t W) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dy.is_cuda() && (dy.dim() == 2 || dy.dim() == 4), "gap_bwd: dy [N, C(, 1, 1)]");
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(dy.numel() == N * C, "gap_bwd: dy must hold one value per (n, c)");
  dy = dy.reshape({N, C}).contiguous();
  at::Tensor dx =
      at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  gap_nhwc_bwd(dy.data_ptr(), dtype_of(dy), dx.data_ptr(), N, H * W, (int)C, cur_stream());
  return dx;
}

}  // namespace amd

namespace amd {

at::Tensor conv_nhwc_fwd_op(at::Tensor x, at::Tensor w, int64_t stride) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && w.dim() == 4, "conv: 4-D GPU tensors expected");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "conv: bf16 only");
  TORCH_CHECK(stride == 1 || stride == 2, "conv: stride 1 or 2");
  const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = w.size(0), k = w.size(2);
  TORCH_CHECK((k == 3 || k == 1) && w.size(3) == k && w.size(1) == Cin, "conv: weight shape");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(conv3x3_nhwc_supported((int)Cin, (int)Cout), "conv: channels must be x64");
  TORCH_CHECK(N * H * W < (int64_t)1 << 31, "conv: too many pixels");
  x = x.contiguous(at::MemoryFormat::ChannelsLast);
  w = w.contiguous(at::MemoryFormat::ChannelsLast);  // [Cout][k][k][Cin] in memory
  at::Tensor y = at::empty({N, Cout, Ho, Wo},
                           x.options().memory_format(at::MemoryFormat::ChannelsLast));
  conv_nhwc_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, (int)Cin,
                (int)Cout, (int)k, (int)stride, cur_stream());
  return y;
}

std::tuple<at::Tensor, at::Tensor> conv_nhwc_fwd_stats_op(at::Tensor x, at::Tensor w,
                                                          int64_t stride,
                                                          c10::optional<at::Tensor> shift) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && w.dim() == 4, "conv: 4-D GPU tensors expected");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "conv: bf16 only");
  TORCH_CHECK(stride == 1 || stride == 2, "conv: stride 1 or 2");
  const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = w.size(0), k = w.size(2);
  TORCH_CHECK((k == 3 || k == 1) && w.size(3) == k && w.size(1) == Cin, "conv: weight shape");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(conv3x3_nhwc_supported((int)Cin, (int)Cout), "conv: channels must be x64");
  TORCH_CHECK(N * H * W < (int64_t)1 << 31, "conv: too many pixels");
  const float* sp = nullptr;
  if (shift.has_value() && shift->defined()) {
    TORCH_CHECK(shift->scalar_type() == at::kFloat && shift->is_contiguous() &&
                    shift->numel() == Cout && shift->is_cuda(),
                "conv stats: shift must be a contiguous fp32 [Cout] GPU tensor");
    sp = shift->data_ptr<float>();
  }
  x = x.contiguous(at::MemoryFormat::ChannelsLast);
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  at::Tensor y = at::empty({N, Cout, Ho, Wo},
                           x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int S = conv_fwd_mtiles((int)N, (int)H, (int)W, (int)Cout, (int)stride, (int)k, (int)Cin);
  at::Tensor slab = at::empty({2, Cout, S}, x.options().dtype(at::kFloat));
  conv_nhwc_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, (int)Cin,
                (int)Cout, (int)k, (int)stride, cur_stream(), slab.data_ptr<float>(), sp);
  return {y, slab};
}

// Stride-1 data-gradient conv (dy with the rotated 3x3 / transposed 1x1 filter) whose
// output is the gradient of a BN(+ReLU) output: stores g = relu_mask * (conv + add) and
// returns it with that BN's per-M-tile backward sums [2][C][S] (ConvBnEpi).
std::tuple<at::Tensor, at::Tensor> conv_nhwc_fwd_bnbwd_op(
    at::Tensor dy, at::Tensor w, c10::optional<at::Tensor> add, at::Tensor xbn,
    c10::optional<at::Tensor> rmask, at::Tensor mean, at::Tensor invstd,
    c10::optional<at::Tensor> bn_w, c10::optional<at::Tensor> bn_b, int64_t relu_mode,
    bool add_stride2) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && w.dim() == 4, "conv_bnbwd: 4-D GPU tensors");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  xbn.scalar_type() == at::kBFloat16,
              "conv_bnbwd: bf16 only");
  const int64_t N = dy.size(0), Cin = dy.size(1), H = dy.size(2), W = dy.size(3);
  const int64_t Cout = w.size(0), k = w.size(2);
  TORCH_CHECK((k == 3 || k == 1) && w.size(3) == k && w.size(1) == Cin, "conv_bnbwd: weight");
  TORCH_CHECK(conv3x3_nhwc_supported((int)Cin, (int)Cout), "conv_bnbwd: channels must be x64");
  TORCH_CHECK(N * H * W < (int64_t)1 << 31, "conv_bnbwd: too many pixels");
  TORCH_CHECK(relu_mode >= 0 && relu_mode <= 2, "conv_bnbwd: relu_mode 0 | 1 | 2");
  const auto cl = at::MemoryFormat::ChannelsLast;
  auto same_out = [&](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.size(0) == N && t.size(1) == Cout &&
                    t.size(2) == H && t.size(3) == W && t.scalar_type() == at::kBFloat16 &&
                    t.is_contiguous(cl),
                "conv_bnbwd: ", what, " must be a channels-last bf16 tensor shaped like the output");
  };
  same_out(xbn, "x");
  ConvBnEpi ep{};
  if (add.has_value() && add->defined()) {
    if (add_stride2) {
      // the compact gradient of a stride-2 1x1 conv over this output (even pixels only)
      TORCH_CHECK(k == 1 && H % 2 == 0 && W % 2 == 0 && add->is_cuda() && add->dim() == 4 &&
                      add->size(0) == N && add->size(1) == Cout && add->size(2) == H / 2 &&
                      add->size(3) == W / 2 && add->scalar_type() == at::kBFloat16 &&
                      add->is_contiguous(cl),
                  "conv_bnbwd: a stride-2 add must be channels-last bf16 [N, C, H/2, W/2] "
                  "(1x1 conv, even H and W)");
      ep.add_s2 = 1;
    } else {
      same_out(*add, "add");
    }
    ep.add = add->data_ptr();
  }
  ep.xbn = xbn.data_ptr();
  auto vecf = [&](const c10::optional<at::Tensor>& t, const char* what) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() == Cout,
                "conv_bnbwd: ", what, " must be a contiguous fp32 [C] GPU tensor");
    return t->data_ptr<float>();
  };
  ep.mean = vecf(mean, "mean");
  ep.invstd = vecf(invstd, "invstd");
  ep.w = vecf(bn_w, "weight");
  ep.b = vecf(bn_b, "bias");
  TORCH_CHECK(ep.mean && ep.invstd, "conv_bnbwd: mean / invstd required");
  ep.relu_mode = (int)relu_mode;
  if (relu_mode == 1) {
    TORCH_CHECK(rmask.has_value() && rmask->defined() && rmask->is_cuda() &&
                    rmask->scalar_type() == at::kByte && rmask->is_contiguous() &&
                    rmask->numel() == N * H * W * (Cout / 8),
                "conv_bnbwd: relu_mode 1 needs the forward's [M][C/8] uint8 bitmask");
    ep.rmask = rmask->data_ptr<uint8_t>();
  }
  dy = dy.contiguous(cl);
  w = w.contiguous(cl);
  at::Tensor g = at::empty({N, Cout, H, W}, dy.options().memory_format(cl));
  const int S = conv_bnbwd_mtiles((int)N, (int)H, (int)W, (int)Cout, (int)k, (int)Cin);
  at::Tensor slab = at::empty({2, Cout, S}, dy.options().dtype(at::kFloat));
  conv_nhwc_fwd_bnbwd(dy.data_ptr(), w.data_ptr(), g.data_ptr(), (int)N, (int)H, (int)W,
                      (int)Cin, (int)Cout, (int)k, 1, ep, slab.data_ptr<float>(), cur_stream());
  return {g, slab};
}

at::Tensor conv_nhwc_dgrad_s2_op(at::Tensor dy, at::Tensor wt, int64_t H, int64_t W) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && wt.dim() == 4, "conv_dgrad_s2: 4-D GPU tensors");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && wt.scalar_type() == at::kBFloat16,
              "conv_dgrad_s2: bf16 only");
  const int64_t N = dy.size(0), Cout = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  const int64_t Cin = wt.size(0), k = wt.size(2);
  TORCH_CHECK(wt.size(1) == Cout && (k == 3 || k == 1) && wt.size(3) == k,
              "conv_dgrad_s2: transposed / rotated weight [Cin, Cout, k, k] expected");
  TORCH_CHECK(H == 2 * Ho && W == 2 * Wo, "conv_dgrad_s2: even input sizes only");
  TORCH_CHECK(conv3x3_nhwc_supported((int)Cout, (int)Cin), "conv_dgrad_s2: channels x64");
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  wt = wt.contiguous(at::MemoryFormat::ChannelsLast);
  at::Tensor dx = at::empty({N, Cin, H, W},
                            dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  conv_nhwc_dgrad_s2(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), (int)N, (int)H, (int)W,
                     (int)Cin, (int)Cout, (int)k, cur_stream());
  return dx;
}

// conv_dgrad_s2 (3x3) whose output is the gradient of a BN(+ReLU) output: g = relu_mask *
// dX and that BN's backward sums [2][C][S] (as conv_fwd_bnbwd, no residual add)
std::tuple<at::Tensor, at::Tensor> conv_nhwc_dgrad_s2_bnbwd_op(
    at::Tensor dy, at::Tensor wt, int64_t H, int64_t W, at::Tensor xbn,
    c10::optional<at::Tensor> rmask, at::Tensor mean, at::Tensor invstd,
    c10::optional<at::Tensor> bn_w, c10::optional<at::Tensor> bn_b, int64_t relu_mode) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && wt.dim() == 4, "dgrad_s2_bnbwd: 4-D GPU tensors");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && wt.scalar_type() == at::kBFloat16 &&
                  xbn.scalar_type() == at::kBFloat16, "dgrad_s2_bnbwd: bf16 only");
  const int64_t N = dy.size(0), Cout = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  const int64_t Cin = wt.size(0);
  TORCH_CHECK(wt.size(1) == Cout && wt.size(2) == 3 && wt.size(3) == 3,
              "dgrad_s2_bnbwd: rotated 3x3 weight [Cin, Cout, 3, 3] expected");
  TORCH_CHECK(H == 2 * Ho && W == 2 * Wo, "dgrad_s2_bnbwd: even input sizes only");
  TORCH_CHECK(conv3x3_nhwc_supported((int)Cout, (int)Cin), "dgrad_s2_bnbwd: channels x64");
  TORCH_CHECK(N * H * W < (int64_t)1 << 31, "dgrad_s2_bnbwd: too many pixels");
  TORCH_CHECK(relu_mode >= 0 && relu_mode <= 2, "dgrad_s2_bnbwd: relu_mode 0 | 1 | 2");
  const auto cl = at::MemoryFormat::ChannelsLast;
  TORCH_CHECK(xbn.is_cuda() && xbn.dim() == 4 && xbn.size(0) == N && xbn.size(1) == Cin &&
                  xbn.size(2) == H && xbn.size(3) == W && xbn.is_contiguous(cl),
              "dgrad_s2_bnbwd: x must be the BN input, channels-last bf16 [N, Cin, H, W]");
  ConvBnEpi ep{};
  ep.xbn = xbn.data_ptr();
  auto vecf = [&](const c10::optional<at::Tensor>& t, const char* what) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() == Cin,
                "dgrad_s2_bnbwd: ", what, " must be a contiguous fp32 [C] GPU tensor");
    return t->data_ptr<float>();
  };
  ep.mean = vecf(mean, "mean");
  ep.invstd = vecf(invstd, "invstd");
  ep.w = vecf(bn_w, "weight");
  ep.b = vecf(bn_b, "bias");
  TORCH_CHECK(ep.mean && ep.invstd, "dgrad_s2_bnbwd: mean / invstd required");
  ep.relu_mode = (int)relu_mode;
  if (relu_mode == 1) {
    TORCH_CHECK(rmask.has_value() && rmask->defined() && rmask->is_cuda() &&
                    rmask->scalar_type() == at::kByte && rmask->is_contiguous() &&
                    rmask->numel() == N * H * W * (Cin / 8),
                "dgrad_s2_bnbwd: relu_mode 1 needs the forward's [M][C/8] uint8 bitmask");
    ep.rmask = rmask->data_ptr<uint8_t>();
  }
  dy = dy.contiguous(cl);
  wt = wt.contiguous(cl);
  at::Tensor g = at::empty({N, Cin, H, W}, dy.options().memory_format(cl));
  at::Tensor slab = at::empty({2, Cin, (int64_t)conv_dgrad_s2_bnbwd_mtiles((int)N, (int)H, (int)W)},
                              dy.options().dtype(at::kFloat));
  conv_nhwc_dgrad_s2_bnbwd(dy.data_ptr(), wt.data_ptr(), g.data_ptr(), (int)N, (int)H, (int)W,
                           (int)Cin, (int)Cout, ep, slab.data_ptr<float>(), cur_stream());
  return {g, slab};
}

at::Tensor conv_nhwc_wgrad_op(at::Tensor dy, at::Tensor x, at::ScalarType out_dtype, int64_t algo,
                              int64_t stride, int64_t ksize, c10::optional<at::Tensor> out,
                              bool accumulate) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && dy.dim() == 4, "conv_wgrad: 4-D GPU tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16,
              "conv_wgrad: bf16 only");
  TORCH_CHECK(ksize == 3 || (ksize == 1 && algo != 1), "conv_wgrad: kernel size");
  const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = dy.size(1);
  TORCH_CHECK(stride == 1 || (stride == 2 && algo != 1), "conv_wgrad: stride");
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == (H - 1) / stride + 1 &&
                  dy.size(3) == (W - 1) / stride + 1, "conv_wgrad: shapes");
  TORCH_CHECK(conv3x3_nhwc_supported((int)Cin, (int)Cout), "conv_wgrad: channels must be x64");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "conv_wgrad: out dtype");
  TORCH_CHECK(conv3x3_wgrad_supported((int)W, (int)algo), "conv_wgrad: width > 56 unsupported for algo 1");
  TORCH_CHECK(algo != 4 || conv3x3_wgrad_c64_ok((int)W, (int)Cin, (int)Cout, (int)ksize, (int)stride),
              "conv_wgrad: algo 4 is the 3x3 stride-1 strip-ring kernel (channels % 64, W <= 56)");
  TORCH_CHECK(algo != 1 || (Cin % 64 == 0 && Cout % 64 == 0), "conv_wgrad: algo 1 channels");
  // the kernels split pixel indices with a float reciprocal (exact below 2^22)
  TORCH_CHECK(N * H * W < ((int64_t)1 << 22), "conv_wgrad: too many pixels");
  x = x.contiguous(at::MemoryFormat::ChannelsLast);
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  const int S = conv_wgrad_splits((int)N, (int)H, (int)W, (int)Cin, (int)Cout, (int)ksize,
                                  (int)stride, (int)algo);
  at::Tensor part = at::empty({conv_wgrad_workspace(S, (int)Cin, (int)Cout, (int)ksize)},
                              x.options().dtype(at::kFloat));
  // out: accumulate into an existing gradient (a DDP bucket view) instead of a new tensor,
  // or (accumulate = false: a lazily zeroed bucket view) overwrite it
  const bool given = out.has_value() && out->defined();
  const bool accum = given && accumulate;
  at::Tensor dw;
  if (given) {
    dw = *out;
    TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == out_dtype && dw.dim() == 4 &&
                    dw.size(0) == Cout && dw.size(1) == Cin && dw.size(2) == ksize &&
                    dw.size(3) == ksize && dw.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_wgrad: out must be a channels-last [Cout, Cin, k, k] tensor of out_dtype");
  } else {
    dw = at::empty({Cout, Cin, ksize, ksize},
                   x.options().dtype(out_dtype).memory_format(at::MemoryFormat::ChannelsLast));
  }
  conv_nhwc_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), dw.data_ptr(),
                  out_dtype == at::kFloat, (int)N, (int)H, (int)W, (int)Cin, (int)Cout, (int)ksize,
                  (int)stride, S, (int)algo, cur_stream(), accum);
  return dw;
}

at::Tensor stem_pad_op(at::Tensor x) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) == 3 && x.scalar_type() == at::kBFloat16,
              "stem_pad: bf16 [N, 3, H, W] expected");
  x = x.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(stem_conv_supported((int)N, (int)H, (int)W), "stem_pad: unsupported size");
  at::Tensor xp = at::empty({N, H + 6, W + 6, 4}, x.options());
  stem_pad(x.data_ptr(), xp.data_ptr(), (int)N, (int)H, (int)W, cur_stream());
  return xp;
}

at::Tensor stem_fwd_op(at::Tensor xp, at::Tensor wk) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(xp.is_cuda() && xp.dim() == 4 && xp.size(3) == 4 && xp.is_contiguous() &&
                  xp.scalar_type() == at::kBFloat16, "stem_fwd: padded input [N, H+6, W+6, 4]");
  TORCH_CHECK(wk.is_cuda() && wk.numel() == 64 * 224 && wk.is_contiguous() &&
                  wk.scalar_type() == at::kBFloat16, "stem_fwd: packed filter [64, 7, 32]");
  const int64_t N = xp.size(0), H = xp.size(1) - 6, W = xp.size(2) - 6;
  TORCH_CHECK(stem_conv_supported((int)N, (int)H, (int)W), "stem_fwd: unsupported size");
  at::Tensor y = at::empty({N, 64, H / 2, W / 2},
                           xp.options().memory_format(at::MemoryFormat::ChannelsLast));
  stem_fwd(xp.data_ptr(), wk.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, cur_stream());
  return y;
}

// stem_fwd_op plus the stem BatchNorm's statistics slab [2][64][S] from the kernel's
// epilogue (shift: the BN's running mean, or none)
std::tuple<at::Tensor, at::Tensor> stem_fwd_stats_op(at::Tensor xp, at::Tensor wk,
                                                     c10::optional<at::Tensor> shift) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(xp.is_cuda() && xp.dim() == 4 && xp.size(3) == 4 && xp.is_contiguous() &&
                  xp.scalar_type() == at::kBFloat16, "stem_fwd: padded input [N, H+6, W+6, 4]");
  TORCH_CHECK(wk.is_cuda() && wk.numel() == 64 * 224 && wk.is_contiguous() &&
                  wk.scalar_type() == at::kBFloat16, "stem_fwd: packed filter [64, 7, 32]");
  const int64_t N = xp.size(0), H = xp.size(1) - 6, W = xp.size(2) - 6;
  TORCH_CHECK(stem_conv_supported((int)N, (int)H, (int)W), "stem_fwd: unsupported size");
  const float* sp = nullptr;
  if (shift.has_value() && shift->defined()) {
    TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->numel() == 64 &&
                    shift->is_contiguous(), "stem_fwd_stats: shift must be fp32 [64]");
    sp = shift->data_ptr<float>();
  }
  at::Tensor y = at::empty({N, 64, H / 2, W / 2},
                           xp.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor slab = at::empty({2, 64, (int64_t)stem_fwd_slab_width((int)N, (int)H)},
                              xp.options().dtype(at::kFloat));
  stem_fwd(xp.data_ptr(), wk.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, cur_stream(),
           slab.data_ptr<float>(), sp);
  return {y, slab};
}

at::Tensor stem_wgrad_op(at::Tensor xp, at::Tensor dy) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(xp.is_cuda() && xp.dim() == 4 && xp.size(3) == 4 && xp.is_contiguous() &&
                  xp.scalar_type() == at::kBFloat16, "stem_wgrad: padded input [N, H+6, W+6, 4]");
  const int64_t N = xp.size(0), H = xp.size(1) - 6, W = xp.size(2) - 6;
  TORCH_CHECK(stem_conv_supported((int)N, (int)H, (int)W), "stem_wgrad: unsupported size");
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.size(0) == N && dy.size(1) == 64 &&
                  dy.size(2) == H / 2 && dy.size(3) == W / 2 && dy.scalar_type() == at::kBFloat16,
              "stem_wgrad: dy [N, 64, H/2, W/2] bf16");
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  const int S = stem_wgrad_splits((int)N, (int)H);
  at::Tensor part = at::empty({(int64_t)S * 64 * 256 + splitk_reduce_workspace(S, 64 * 256)},
                              xp.options().dtype(at::kFloat));
  stem_wgrad(xp.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), S, (int)N, (int)H, (int)W,
             cur_stream());
  at::Tensor out = at::empty({64, 256}, xp.options().dtype(at::kFloat));
  splitk_reduce(part.data_ptr<float>(), S, 64, 256, part.data_ptr<float>() + (int64_t)S * 64 * 256,
                out.data_ptr(), true, cur_stream());
  return out;
}

at::Tensor splitk_reduce_op(at::Tensor part, at::ScalarType out_dtype,
                            c10::optional<at::Tensor> out_acc, bool accumulate) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(part.is_cuda() && part.dim() == 3 && part.scalar_type() == at::kFloat &&
                  part.is_contiguous(), "splitk_reduce: contiguous fp32 [S, M, N] expected");
  const int64_t S = part.size(0), M = part.size(1), N = part.size(2);
  TORCH_CHECK((M * N) % 4 == 0, "splitk_reduce: M*N must be a multiple of 4");
  at::Tensor stage = at::empty({splitk_reduce_workspace((int)S, M * N)}, part.options());
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "splitk_reduce: out dtype");
  // out_acc: accumulate into an existing [M, N]-contiguous tensor (a DDP bucket view)
  const bool given = out_acc.has_value() && out_acc->defined();
  const bool accum = given && accumulate;  // false: overwrite the given tensor
  at::Tensor out;
  if (given) {
    out = *out_acc;
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == out_dtype && out.numel() == M * N &&
                    out.is_contiguous(),
                "splitk_reduce: accumulation target must be a contiguous tensor of M*N elements");
  } else {
    out = at::empty({M, N}, part.options().dtype(out_dtype));
  }
  splitk_reduce(part.data_ptr<float>(), (int)S, (int)M, (int)N, stage.data_ptr<float>(),
                out.data_ptr(), out_dtype == at::kFloat, cur_stream(), accum);
  return out;
}

at::Tensor conv3x3_rot_weight_op(at::Tensor w) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.element_size() == 2, "rot_weight: 16-bit [Cout, Cin, 3, 3] expected");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t Cout = w.size(0), Cin = w.size(1);
  at::Tensor out = at::empty({Cin, Cout, 3, 3}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  conv3x3_rot_weight(w.data_ptr(), out.data_ptr(), (int)Cout, (int)Cin, cur_stream());
  return out;
}

at::Tensor conv1x1_transpose_weight_op(at::Tensor w) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.size(2) == 1 && w.size(3) == 1 &&
                  w.element_size() == 2, "transpose_weight: 16-bit [Cout, Cin, 1, 1] expected");
  w = w.contiguous();
  const int64_t Cout = w.size(0), Cin = w.size(1);
  at::Tensor out = at::empty({Cin, Cout, 1, 1}, w.options());
  conv1x1_transpose_weight(w.data_ptr(), out.data_ptr(), (int)Cout, (int)Cin, cur_stream());
  return out;
}

std::vector<at::Tensor> conv_prep_weights_op(std::vector<at::Tensor> ws) {
  c10::NoGradGuard no_grad_;
  std::vector<at::Tensor> outs;
  std::vector<const void*> in;
  std::vector<void*> out;
  std::vector<int> co, ci, taps;
  std::vector<at::Tensor> keep;
  for (auto& w : ws) {
    TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.element_size() == 2 &&
                    ((w.size(2) == 3 && w.size(3) == 3) || (w.size(2) == 1 && w.size(3) == 1)),
                "prep_weights: 16-bit [Cout, Cin, 3|1, 3|1] filters expected");
    at::Tensor wc = w.contiguous(at::MemoryFormat::ChannelsLast);
    const int64_t Cout = w.size(0), Cin = w.size(1), k = w.size(2);
    at::Tensor o = at::empty({Cin, Cout, k, k}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
    in.push_back(wc.data_ptr());
    out.push_back(o.data_ptr());
    co.push_back((int)Cout);
    ci.push_back((int)Cin);
    taps.push_back((int)(k * k));
    keep.push_back(wc);
    outs.push_back(o);
  }
  if (!outs.empty())
    prep_weights(in.data(), out.data(), co.data(), ci.data(), taps.data(), (int)outs.size(),
                 cur_stream());
  return outs;
}

}  // namespace amd
