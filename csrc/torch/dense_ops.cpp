// Dense-layer bias gradients on the column-sum kernels (csrc/hip/bias_grad.hip);
// CPU / unsupported layouts use the ATen reference.
#include "dense_ops.h"

#include "common.h"
#include "pool_ops.h"

namespace amd {

namespace {

bool colsum_ok(const at::Tensor& t) {
  return t.is_cuda() && t.is_contiguous() && t.dim() >= 1 &&
         (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf ||
          t.scalar_type() == at::kFloat) &&
         t.size(-1) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 &&
         t.numel() > 0;
}

at::Tensor gelu_grad_ref(const at::Tensor& pre, bool tanh_approx) {
  at::Tensor x = pre.to(at::kFloat);
  if (tanh_approx) {
    const double k0 = 0.7978845608028654, k1 = 0.044715;
    at::Tensor t = at::tanh(k0 * (x + k1 * x * x * x));
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x);
  }
  return 0.5 * (1 + at::erf(x * 0.7071067811865476)) +
         x * at::exp(-0.5 * x * x) * 0.3989422804014327;
}

}  // namespace

at::Tensor bias_grad_op(at::Tensor g, at::ScalarType out_dtype) {
  c10::NoGradGuard no_grad_;
  const int64_t N = g.size(-1);
  if (!colsum_ok(g)) return g.reshape({-1, N}).to(at::kFloat).sum(0).to(out_dtype);
  const int64_t M = g.numel() / N;
  const int S = colsum_splits(M, (int)N);
  at::Tensor part = at::empty({(int64_t)S * N}, g.options().dtype(at::kFloat));
  at::Tensor out = at::empty({N}, g.options().dtype(out_dtype));
  colsum(g.data_ptr(), nullptr, nullptr, dtype_of(g), M, (int)N, 0, part.data_ptr<float>(), S,
         out.data_ptr(), dtype_of(out), cur_stream());
  return out;
}

std::tuple<at::Tensor, at::Tensor> gelu_bwd_bias_grad_op(at::Tensor dh, at::Tensor pre,
                                                         bool tanh_approx,
                                                         at::ScalarType out_dtype) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dh.sizes() == pre.sizes(), "gelu_bwd_bias_grad: shape mismatch");
  const int64_t N = dh.size(-1);
  dh = dh.contiguous();
  pre = pre.contiguous();
  if (!colsum_ok(dh) || !colsum_ok(pre) || dh.scalar_type() != pre.scalar_type()) {
    at::Tensor dpre = (dh.to(at::kFloat) * gelu_grad_ref(pre, tanh_approx)).to(dh.scalar_type());
    return {dpre, dpre.reshape({-1, N}).to(at::kFloat).sum(0).to(out_dtype)};
  }
  const int64_t M = dh.numel() / N;
  const int S = colsum_splits(M, (int)N);
  at::Tensor part = at::empty({(int64_t)S * N}, dh.options().dtype(at::kFloat));
  at::Tensor dpre = at::empty_like(dh);
  at::Tensor out = at::empty({N}, dh.options().dtype(out_dtype));
  colsum(dh.data_ptr(), pre.data_ptr(), dpre.data_ptr(), dtype_of(dh), M, (int)N,
         tanh_approx ? 2 : 1, part.data_ptr<float>(), S, out.data_ptr(), dtype_of(out),
         cur_stream());
  return {dpre, out};
}

at::Tensor gelu_fwd_op(at::Tensor x, bool tanh_approx) {
  c10::NoGradGuard no_grad_;
  x = x.contiguous();
  if (!colsum_ok(x) || x.numel() % 8 != 0)
    return at::gelu(x, tanh_approx ? "tanh" : "none");
  at::Tensor y = at::empty_like(x);
  gelu_fwd(x.data_ptr(), y.data_ptr(), dtype_of(x), x.numel(), tanh_approx, cur_stream());
  return y;
}

std::tuple<at::Tensor, at::Tensor> act_bwd_bias_grad_op(at::Tensor dh, at::Tensor y, int64_t act,
                                                        at::ScalarType out_dtype) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dh.sizes() == y.sizes(), "act_bwd_bias_grad: shape mismatch");
  TORCH_CHECK(act == 1 || act == 2, "act_bwd_bias_grad: act must be 1 (relu) or 2 (sigmoid)");
  const int64_t N = dh.size(-1);
  dh = dh.contiguous();
  y = y.contiguous();
  if (!colsum_ok(dh) || !colsum_ok(y) || dh.scalar_type() != y.scalar_type()) {
    at::Tensor yf = y.to(at::kFloat);
    at::Tensor d = act == 1 ? (yf > 0).to(at::kFloat) : yf * (1 - yf);
    at::Tensor dpre = (dh.to(at::kFloat) * d).to(dh.scalar_type());
    return {dpre, dpre.reshape({-1, N}).to(at::kFloat).sum(0).to(out_dtype)};
  }
  const int64_t M = dh.numel() / N;
  const int S = colsum_splits(M, (int)N);
  at::Tensor part = at::empty({(int64_t)S * N}, dh.options().dtype(at::kFloat));
  at::Tensor dpre = at::empty_like(dh);
  at::Tensor out = at::empty({N}, dh.options().dtype(out_dtype));
  colsum(dh.data_ptr(), y.data_ptr(), dpre.data_ptr(), dtype_of(dh), M, (int)N,
         act == 1 ? 3 : 4, part.data_ptr<float>(), S, out.data_ptr(), dtype_of(out),
         cur_stream());
  return {dpre, out};
}

static bool gemm_layout_ok(const at::Tensor& a, const at::Tensor& b) {
  return a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2 &&
         (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf) &&
         b.scalar_type() == a.scalar_type() &&
         a.stride(1) == 1 && b.stride(1) == 1 && a.size(1) == b.size(1) &&
         a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 &&
         reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
         reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 && a.size(0) < (1 << 30) &&
         // the 4-wave kernel's 32-bit DMA offsets: 256 rows of either operand
         256 * std::max(a.stride(0), b.stride(0)) * a.element_size() < (int64_t(1) << 32);
}

bool gemm4w_ok(const at::Tensor& a, const at::Tensor& b) {
  return gemm_layout_ok(a, b) &&
         gemm4w_supported((int)a.size(0), (int)b.size(0), (int)a.size(1));
}

bool wgrad4w_ok(const at::Tensor& dy, const at::Tensor& x, int64_t splits) {
  return dy.is_cuda() && x.is_cuda() && dy.dim() == 2 && x.dim() == 2 &&
         (dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf) &&
         x.scalar_type() == dy.scalar_type() && dy.size(0) == x.size(0) &&
         dy.stride(1) == 1 && x.stride(1) == 1 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0 &&
         reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 &&
         reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && splits >= 1 &&
         dy.size(1) < (1 << 30) && x.size(1) < (1 << 30) &&
         // 32-bit DMA offsets: a split's rows of either operand
         (dy.size(0) / splits) * std::max(dy.stride(0), x.stride(0)) * dy.element_size() <
             (int64_t(1) << 32) &&
         wgrad4w_supported(dy.size(0), (int)dy.size(1), (int)x.size(1), (int)splits);
}

// dW [M, N] = dy^T x in out_dtype (fp32 / bf16): fp32 partials per split of the rows, then
// the slab reduction (which also accumulates into / overwrites `out`, a DDP bucket view)
at::Tensor wgrad4w_op(at::Tensor dy, at::Tensor x, int64_t splits, at::ScalarType out_dtype,
                      c10::optional<at::Tensor> out, bool accumulate) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(wgrad4w_ok(dy, x, splits),
              "wgrad4w: bf16 / fp16 dy [T, M], x [T, N] with unit column stride, M % 256 == 0, "
              "N % 256 == 0, (T / splits) % 64 == 0");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "wgrad4w: out dtype");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  const bool given = out.has_value() && out->defined();
  if (given)
    TORCH_CHECK(out->is_cuda() && out->scalar_type() == out_dtype && out->numel() == M * N &&
                    out->is_contiguous(),
                "wgrad4w: out must be a contiguous tensor of M*N elements of out_dtype");
  WgradArgs g{};
  g.A = dy.data_ptr();
  g.B = x.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.lda = (int)dy.stride(0);
  g.ldb = (int)x.stride(0);
  g.rows = (int)(T / splits);
  g.S = (int)splits;
  g.fp16 = dy.scalar_type() == at::kHalf ? 1 : 0;
  // one split written straight into an fp32 result (no reduction pass)
  if (splits == 1 && out_dtype == at::kFloat && !(given && accumulate)) {
    at::Tensor r = given ? *out : at::empty({M, N}, dy.options().dtype(at::kFloat));
    g.P = r.data_ptr<float>();
    wgrad4w(g, cur_stream());
    return r;
  }
  at::Tensor part = at::empty({splits, M, N}, dy.options().dtype(at::kFloat));
  g.P = part.data_ptr<float>();
  wgrad4w(g, cur_stream());
  return splitk_reduce_op(part, out_dtype, out, accumulate);
}

// wgrad4w_op plus the bias gradient db [M] = column sums of dy in bias_dtype, formed from
// the kernel's dY fragments (fp32 per split, then the bias-gradient final kernel): the
// dense layer's separate column-sum pass over dy disappears
std::tuple<at::Tensor, at::Tensor> wgrad4w_bias_op(at::Tensor dy, at::Tensor x, int64_t splits,
                                                   at::ScalarType out_dtype,
                                                   c10::optional<at::Tensor> out, bool accumulate,
                                                   at::ScalarType bias_dtype) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(wgrad4w_ok(dy, x, splits), "wgrad4w_bias: see wgrad4w");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "wgrad4w: out dtype");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  const bool given = out.has_value() && out->defined();
  if (given)
    TORCH_CHECK(out->is_cuda() && out->scalar_type() == out_dtype && out->numel() == M * N &&
                    out->is_contiguous(),
                "wgrad4w: out must be a contiguous tensor of M*N elements of out_dtype");
  at::Tensor cs = at::empty({splits, M}, dy.options().dtype(at::kFloat));
  WgradArgs g{};
  g.A = dy.data_ptr();
  g.B = x.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.lda = (int)dy.stride(0);
  g.ldb = (int)x.stride(0);
  g.rows = (int)(T / splits);
  g.S = (int)splits;
  g.fp16 = dy.scalar_type() == at::kHalf ? 1 : 0;
  g.colsum = cs.data_ptr<float>();
  at::Tensor db = at::empty({M}, dy.options().dtype(bias_dtype));
  at::Tensor w;
  if (splits == 1 && out_dtype == at::kFloat && !(given && accumulate)) {
    w = given ? *out : at::empty({M, N}, dy.options().dtype(at::kFloat));
    g.P = w.data_ptr<float>();
    wgrad4w(g, cur_stream());
  } else {
    at::Tensor part = at::empty({splits, M, N}, dy.options().dtype(at::kFloat));
    g.P = part.data_ptr<float>();
    wgrad4w(g, cur_stream());
    w = splitk_reduce_op(part, out_dtype, out, accumulate);
  }
  colsum_finalize(cs.data_ptr<float>(), (int)splits, (int)M, db.data_ptr(), dtype_of(db),
                  cur_stream());
  return {w, db};
}

std::vector<at::Tensor> gemm4w_op(at::Tensor a, at::Tensor b, int64_t epi,
                                  c10::optional<at::Tensor> bias, c10::optional<at::Tensor> aux,
                                  bool want_pre, bool tanh_approx,
                                  c10::optional<at::ScalarType> bias_grad_dtype) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(gemm4w_ok(a, b),
              "gemm4w: bf16 / fp16 [M, K] x [N, K] with N % 256 == 0, K % 64 == 0, unit column "
              "stride, 16-byte aligned rows");
  TORCH_CHECK(epi >= 0 && epi <= 2, "gemm4w: epi 0 | 1 | 2");
  const int64_t M = a.size(0), N = b.size(0), K = a.size(1);
  at::Tensor c = at::empty({M, N}, a.options());
  GemmArgs g{};
  g.A = a.data_ptr();
  g.B = b.data_ptr();
  g.C = c.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = (int)a.stride(0);
  g.ldb = (int)b.stride(0);
  g.ldc = (int)N;
  g.tanh = tanh_approx ? 1 : 0;
  g.fp16 = a.scalar_type() == at::kHalf ? 1 : 0;
  std::vector<at::Tensor> out{c};
  if (epi == 1) {
    if (bias.has_value() && bias->defined()) {
      TORCH_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->numel() == N &&
                      (bias->scalar_type() == a.scalar_type() || bias->scalar_type() == at::kFloat),
                  "gemm4w: bias must be a contiguous [N] GPU tensor of the operand dtype or fp32");
      g.bias = bias->data_ptr();
      g.bias_f32 = bias->scalar_type() == at::kFloat ? 1 : 0;
    }
    if (want_pre) {
      at::Tensor pre = at::empty({M, N}, a.options());
      g.aux = pre.data_ptr();
      out.push_back(pre);
    }
  } else if (epi == 2) {
    TORCH_CHECK(aux.has_value() && aux->defined() && aux->is_cuda() &&
                    aux->scalar_type() == a.scalar_type() && aux->is_contiguous() &&
                    aux->numel() == M * N,
                "gemm4w: epi 2 needs the contiguous bf16 [M, N] pre-activation");
    g.aux = aux->data_ptr();
  }
  at::Tensor part;
  if (epi == 2 && bias_grad_dtype.has_value()) {
    part = at::empty({(M + 255) / 256, N}, a.options().dtype(at::kFloat));
    g.colsum = part.data_ptr<float>();
  }
  gemm4w(g, (int)epi, cur_stream());
  if (part.defined()) {
    at::Tensor db = at::empty({N}, a.options().dtype(*bias_grad_dtype));
    colsum_finalize(part.data_ptr<float>(), (int)part.size(0), (int)N, db.data_ptr(),
                    dtype_of(db), cur_stream());
    out.push_back(db);
  }
  return out;
}

}  // namespace amd
