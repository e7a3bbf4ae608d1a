// Torch bindings for the fused attention kernels (csrc/hip/attention.hip).
#include "attn_ops.h"

#include "common.h"

namespace amd {

namespace {
void check_view(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.size(3) == 64, "attn: ", what,
              " must be a [B,S,H,64] GPU tensor");
  TORCH_CHECK(t.stride(3) == 1, "attn: ", what, ": head dim must be contiguous");
  TORCH_CHECK(((uintptr_t)t.data_ptr() % 16) == 0 && t.stride(0) % 8 == 0 &&
                  t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              "attn: ", what, ": 16-byte aligned rows required");
  // the kernels' tile DMA uses 32-bit per-lane row offsets (csrc/hip/attention.hip)
  TORCH_CHECK(t.stride(1) >= 0 && t.stride(1) < (int64_t{1} << 24), "attn: ", what,
              ": sequence stride must be below 2^24 elements");
}

bool view_ok(const at::Tensor& t) {
  return t.stride(3) == 1 && ((uintptr_t)t.data_ptr() % 16) == 0 && t.stride(0) % 8 == 0 &&
         t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0;
}

AttnLaunch make_launch(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                       bool causal, double dropout, int64_t seed, double scale) {
  check_view(q, "q");
  check_view(k, "k");
  check_view(v, "v");
  TORCH_CHECK(k.sizes() == q.sizes() && v.sizes() == q.sizes(), "attn: q/k/v shapes differ");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type() &&
                  (q.scalar_type() == at::kBFloat16 || q.scalar_type() == at::kHalf),
              "attn: bf16/fp16 q,k,v of one dtype");
  TORCH_CHECK(dropout >= 0.0 && dropout < 1.0, "attn: dropout must be in [0, 1)");
  AttnLaunch L;
  L.q = q.data_ptr(); L.k = k.data_ptr(); L.v = v.data_ptr();
  L.qsb = q.stride(0); L.qss = q.stride(1); L.qsh = q.stride(2);
  L.ksb = k.stride(0); L.kss = k.stride(1); L.ksh = k.stride(2);
  L.vsb = v.stride(0); L.vss = v.stride(1); L.vsh = v.stride(2);
  L.B = (int)q.size(0); L.S = (int)q.size(1); L.H = (int)q.size(2);
  L.scale = (float)scale; L.dropout = (float)dropout; L.seed = (uint32_t)seed;
  L.causal = causal; L.dtype = dtype_of(q);
  L.lse_stride = attn_lse_stride(L.S);
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
  at::Tensor lse = at::empty({L.B, L.H, L.lse_stride}, q.options().dtype(at::kFloat));
  L.o = o.data_ptr();
  L.lse = lse.data_ptr<float>();
  if (L.S > 0 && L.B * L.H > 0) attn_fwd(L, cur_stream());
  return {o, L.lse_stride == L.S ? lse : lse.narrow(2, 0, L.S)};
}

void attn_bwd_op(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o,
                 at::Tensor lse, bool causal, double dropout, int64_t seed, double scale,
                 at::Tensor dq, at::Tensor dk, at::Tensor dv) {
  c10::NoGradGuard no_grad_;
  AttnLaunch F = make_launch(q, k, v, causal, dropout, seed, scale);
  if (!(dout.dim() == 4 && view_ok(dout))) dout = dout.contiguous();
  if (!(o.dim() == 4 && view_ok(o))) o = o.contiguous();
  check_view(dout, "dout");
  check_view(o, "o");
  check_view(dq, "dq");
  check_view(dk, "dk");
  check_view(dv, "dv");
  for (const at::Tensor* t : {&dout, &o, &dq, &dk, &dv}) {
    TORCH_CHECK(t->sizes() == q.sizes(), "attn bwd: shape mismatch");
    TORCH_CHECK(t->scalar_type() == q.scalar_type(), "attn bwd: dtype mismatch");
  }
  const int B = F.B, H = F.H, S = F.S, Sp = F.lse_stride;
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.dim() == 3 && lse.size(0) == B &&
                  lse.size(1) == H && lse.size(2) == S,
              "attn bwd: lse must be fp32 [B, H, S]");
  if (!(lse.stride(2) == 1 && lse.stride(1) == Sp && lse.stride(0) == (int64_t)H * Sp &&
        ((uintptr_t)lse.data_ptr() % 16) == 0)) {
    at::Tensor padded = at::empty({B, H, Sp}, lse.options());
    padded.narrow(2, 0, S).copy_(lse);
    lse = padded;
  }
  at::Tensor D = at::empty({B, H, Sp}, lse.options());
  if (S == 0 || B * H == 0) return;
  AttnBwdLaunch L;
  L.q = F.q; L.k = F.k; L.v = F.v; L.o = o.data_ptr(); L.dout = dout.data_ptr();
  L.qsb = F.qsb; L.qss = F.qss; L.qsh = F.qsh;
  L.ksb = F.ksb; L.kss = F.kss; L.ksh = F.ksh;
  L.vsb = F.vsb; L.vss = F.vss; L.vsh = F.vsh;
  L.osb = o.stride(0); L.oss = o.stride(1); L.osh = o.stride(2);
  L.dsb = dout.stride(0); L.dss = dout.stride(1); L.dsh = dout.stride(2);
  L.dq = dq.data_ptr(); L.dk = dk.data_ptr(); L.dv = dv.data_ptr();
  L.dqsb = dq.stride(0); L.dqss = dq.stride(1); L.dqsh = dq.stride(2);
  L.dksb = dk.stride(0); L.dkss = dk.stride(1); L.dksh = dk.stride(2);
  L.dvsb = dv.stride(0); L.dvss = dv.stride(1); L.dvsh = dv.stride(2);
  L.lse = lse.data_ptr<float>(); L.D = D.data_ptr<float>(); L.lse_stride = Sp;
  L.B = B; L.H = H; L.S = S;
  L.scale = F.scale; L.dropout = F.dropout; L.seed = F.seed;
  L.causal = causal; L.dtype = F.dtype;
  attn_bwd(L, cur_stream());
}

}  // namespace amd
