// Torch bindings for the fused attention kernels (csrc/hip/attention.hip).
#include "attn_ops.h"

#include "common.h"

namespace amd {

namespace {
AttnLaunch make_launch(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                       bool causal, double dropout, int64_t seed, double scale) {
  TORCH_CHECK(q.is_cuda() && q.dim() == 4 && q.size(3) == 64, "attn: q must be [B,S,H,64] on GPU");
  TORCH_CHECK(k.sizes() == q.sizes() && v.sizes() == q.sizes(), "attn: q/k/v shapes differ");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type() &&
                  (q.scalar_type() == at::kBFloat16 || q.scalar_type() == at::kHalf),
              "attn: bf16/fp16 q,k,v of one dtype");
  for (const at::Tensor* t : {&q, &k, &v}) {
    TORCH_CHECK(t->stride(3) == 1, "attn: head dim must be contiguous");
    TORCH_CHECK(((uintptr_t)t->data_ptr() % 16) == 0 && t->stride(0) % 8 == 0 &&
                    t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0,
                "attn: 16-byte aligned rows required");
  }
  AttnLaunch L;
  L.q = q.data_ptr(); L.k = k.data_ptr(); L.v = v.data_ptr();
  L.qsb = q.stride(0); L.qss = q.stride(1); L.qsh = q.stride(2);
  L.ksb = k.stride(0); L.kss = k.stride(1); L.ksh = k.stride(2);
  L.vsb = v.stride(0); L.vss = v.stride(1); L.vsh = v.stride(2);
  L.B = (int)q.size(0); L.S = (int)q.size(1); L.H = (int)q.size(2);
  L.scale = (float)scale; L.dropout = (float)dropout; L.seed = (uint32_t)seed;
  L.causal = causal; L.dtype = dtype_of(q);
  L.o = nullptr; L.lse = nullptr;
  return L;
}
}  // namespace

std::tuple<at::Tensor, at::Tensor> attn_fwd_op(at::Tensor q, at::Tensor k, at::Tensor v,
                                               bool causal, double dropout, int64_t seed,
                                               double scale) {
  c10::NoGradGuard no_grad_;
  AttnLaunch L = make_launch(q, k, v, causal, dropout, seed, scale);
  at::Tensor o = at::empty({L.B, L.S, L.H, 64}, q.options());
  at::Tensor lse = at::empty({L.B, L.H, L.S}, q.options().dtype(at::kFloat));
  L.o = o.data_ptr();
  L.lse = lse.data_ptr<float>();
  attn_fwd(L, cur_stream());
  return {o, lse};
}

}  // namespace amd
