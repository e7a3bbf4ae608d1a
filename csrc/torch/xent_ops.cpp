// Fused softmax cross entropy operators: validation, CPU reference path, GPU launch.
#include "xent_ops.h"

#include "common.h"

namespace amd {

namespace {
at::Tensor ignored_rows(const at::Tensor& labels, int64_t padding_idx, int64_t V) {
  return (labels == padding_idx) | (labels < 0) | (labels >= V);
}
}  // namespace

std::tuple<at::Tensor, at::Tensor> xentropy_fwd_op(at::Tensor logits, at::Tensor labels,
                                                   double smoothing, int64_t padding_idx,
                                                   bool half_to_float) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(logits.dim() == 2, "xentropy: logits must be [N, V]");
  TORCH_CHECK(labels.dim() == 1 && labels.size(0) == logits.size(0), "xentropy: labels must be [N]");
  logits = logits.contiguous();
  labels = labels.to(at::kLong).contiguous();
  const int64_t N = logits.size(0), V = logits.size(1);
  const auto lossT = half_to_float ? at::kFloat : logits.scalar_type();
  if (!logits.is_cuda()) {
    at::Tensor xf = logits.to(at::kFloat);
    at::Tensor lse = at::logsumexp(xf, 1);
    at::Tensor ign = ignored_rows(labels, padding_idx, V);
    at::Tensor safe = at::where(ign, at::zeros_like(labels), labels);
    at::Tensor xl = xf.gather(1, safe.unsqueeze(1)).squeeze(1);
    at::Tensor loss = lse - (1.0 - smoothing) * xl - smoothing * xf.mean(1);
    loss = at::where(ign, at::zeros_like(loss), loss);
    return {loss.to(lossT), lse};
  }
  TORCH_CHECK(labels.is_cuda(), "xentropy: labels must be on the logits' device");
  TORCH_CHECK(V < (int64_t)1 << 31, "xentropy: vocabulary too large");
  at::Tensor loss = at::empty({N}, logits.options().dtype(lossT));
  at::Tensor lse = at::empty({N}, logits.options().dtype(at::kFloat));
  xentropy_fwd(logits.data_ptr(), dtype_of(logits), labels.data_ptr<int64_t>(), N, (int)V,
               (float)smoothing, padding_idx, loss.data_ptr(), dtype_of(loss),
               lse.data_ptr<float>(), cur_stream());
  return {loss, lse};
}

at::Tensor xentropy_bwd_op(at::Tensor grad_loss, at::Tensor logits, at::Tensor lse,
                           at::Tensor labels, double smoothing, int64_t padding_idx) {
  c10::NoGradGuard no_grad_;
  logits = logits.contiguous();
  labels = labels.to(at::kLong).contiguous();
  grad_loss = grad_loss.contiguous();
  lse = lse.to(at::kFloat).contiguous();
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(grad_loss.numel() == N && lse.numel() == N, "xentropy bwd: shape mismatch");
  if (!logits.is_cuda()) {
    at::Tensor xf = logits.to(at::kFloat);
    at::Tensor p = at::exp(xf - lse.unsqueeze(1));
    at::Tensor ign = ignored_rows(labels, padding_idx, V);
    at::Tensor safe = at::where(ign, at::zeros_like(labels), labels);
    at::Tensor onehot = at::zeros_like(xf).scatter_(1, safe.unsqueeze(1), 1.0);
    at::Tensor g = at::where(ign, at::zeros_like(lse), grad_loss.to(at::kFloat));
    at::Tensor dx = g.unsqueeze(1) * (p - (1.0 - smoothing) * onehot - smoothing / (double)V);
    return dx.to(logits.scalar_type());
  }
  at::Tensor dx = at::empty_like(logits);
  xentropy_bwd(grad_loss.data_ptr(), dtype_of(grad_loss), logits.data_ptr(), dtype_of(logits),
               lse.data_ptr<float>(), labels.data_ptr<int64_t>(), N, (int)V, (float)smoothing,
               padding_idx, dx.data_ptr(), cur_stream());
  return dx;
}

}  // namespace amd
