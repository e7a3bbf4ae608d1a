// Deterministic embedding weight gradient: device sort + run-sum launches (GPU), or a
// sequential scatter in token order (CPU reference path).
#include "emb_ops.h"

#include "common.h"

namespace amd {

at::Tensor embedding_wgrad_op(at::Tensor idx, at::Tensor dy, int64_t V, int64_t padding_idx,
                              c10::ScalarType out_dtype) {
  c10::NoGradGuard no_grad_;
  at::Tensor flat = idx.reshape({-1}).to(at::kLong);
  const int64_t T = flat.numel();
  TORCH_CHECK(dy.numel() % (T > 0 ? T : 1) == 0, "embedding_wgrad: dy / idx size mismatch");
  const int64_t H = T > 0 ? dy.numel() / T : 0;
  at::Tensor dy2 = dy.reshape({T, H}).contiguous();
  at::Tensor out = at::zeros({V, H}, dy.options().dtype(out_dtype));
  if (!dy.is_cuda()) {
    // token order, fp32 accumulation: the same sums the GPU kernel forms
    at::Tensor acc = at::zeros({V, H}, dy.options().dtype(at::kFloat));
    acc.index_add_(0, flat, dy2.to(at::kFloat));
    if (padding_idx >= 0 && padding_idx < V) acc[padding_idx].zero_();
    return out.copy_(acc);
  }
  TORCH_CHECK(flat.is_cuda(), "embedding_wgrad: ids must be on the gradient's device");
  auto kdt = [](c10::ScalarType t) {
    return t == at::kFloat || t == at::kHalf || t == at::kBFloat16;
  };
  TORCH_CHECK(kdt(dy.scalar_type()) && kdt(out_dtype),
              "embedding_wgrad: fp32 / fp16 / bf16 gradients only (got ", dy.scalar_type(),
              " -> ", out_dtype, ")");
  TORCH_CHECK(H < ((int64_t)1 << 31), "embedding_wgrad: hidden size too large");
  if (T == 0) return out;
  at::Tensor sorted, perm;
  std::tie(sorted, perm) = at::sort(flat, /*stable=*/true, /*dim=*/0, /*descending=*/false);
  sorted = sorted.contiguous();
  perm = perm.contiguous();
  // 8-column vectors: every row start is then 16-byte aligned for 16-bit and fp32 data
  const bool vec = H % 8 == 0 && reinterpret_cast<uintptr_t>(dy2.data_ptr()) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0;
  at::Tensor slots = at::empty({embedding_wgrad_slots(T, (int)H)}, dy.options().dtype(at::kFloat));
  embedding_wgrad(sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dy2.data_ptr(),
                  dtype_of(dy2), T, (int)H, padding_idx, out.data_ptr(), dtype_of(out),
                  vec, slots.data_ptr<float>(), cur_stream());
  return out;
}

}  // namespace amd
