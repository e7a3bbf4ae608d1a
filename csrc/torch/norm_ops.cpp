// LayerNorm and BatchNorm operators: geometry, allocation, CPU/GPU dispatch.
#include "norm_ops.h"

#include "common.h"

namespace amd {

namespace {
const void* optp(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }
bool has(const OptT& t) { return t.has_value() && t->defined(); }
}  // namespace

// ============================================================================ LayerNorm
std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_forward_op(at::Tensor x, int64_t n2,
                                                                     OptT gamma, OptT beta,
                                                                     double eps, bool rms) {
  x = x.contiguous();
  TORCH_CHECK(n2 > 0 && x.numel() % n2 == 0, "layer_norm: bad normalized size");
  const int64_t n1 = x.numel() / n2;
  auto fopt = x.options().dtype(at::kFloat);
  if (!x.is_cuda()) {
    at::Tensor xf = x.to(at::kFloat).view({n1, n2});
    at::Tensor mean = rms ? at::zeros({n1}, fopt) : xf.mean(1);
    at::Tensor xc = rms ? xf : xf - mean.unsqueeze(1);
    at::Tensor var = xc.pow(2).mean(1);
    at::Tensor invvar = (var + eps).rsqrt();
    at::Tensor y = xc * invvar.unsqueeze(1);
    if (has(gamma)) y = y * gamma->to(at::kFloat).view({1, n2});
    if (has(beta)) y = y + beta->to(at::kFloat).view({1, n2});
    return {y.to(x.scalar_type()).view(x.sizes()), mean, invvar};
  }
  at::Tensor g = has(gamma) ? gamma->contiguous() : at::Tensor();
  at::Tensor b = has(beta) ? beta->contiguous() : at::Tensor();
  if (g.defined() && b.defined())
    TORCH_CHECK(g.scalar_type() == b.scalar_type(), "gamma/beta dtype mismatch");
  at::Tensor y = at::empty_like(x);
  at::Tensor mean = at::empty({n1}, fopt);
  at::Tensor invvar = at::empty({n1}, fopt);
  DType tw = g.defined() ? dtype_of(g) : (b.defined() ? dtype_of(b) : DType::F32);
  layer_norm_fwd(x.data_ptr(), dtype_of(x), g.defined() ? g.data_ptr() : nullptr,
                 b.defined() ? b.data_ptr() : nullptr, tw, y.data_ptr(), mean.data_ptr<float>(),
                 invvar.data_ptr<float>(), n1, n2, (float)eps, rms ? 1 : 0, cur_stream());
  return {y, mean, invvar};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_backward_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invvar, int64_t n2, OptT gamma,
    bool need_wgrad, bool need_bgrad, bool rms) {
  x = x.contiguous();
  dy = dy.contiguous();
  const int64_t n1 = x.numel() / n2;
  if (!x.is_cuda()) {
    at::Tensor xf = x.to(at::kFloat).view({n1, n2});
    at::Tensor df = dy.to(at::kFloat).view({n1, n2});
    at::Tensor xh = (rms ? xf : xf - mean.unsqueeze(1)) * invvar.unsqueeze(1);
    at::Tensor dg = has(gamma) ? df * gamma->to(at::kFloat).view({1, n2}) : df;
    at::Tensor s2 = (dg * xh).mean(1, true);
    at::Tensor t = rms ? dg - xh * s2 : dg - dg.mean(1, true) - xh * s2;
    at::Tensor dx = (t * invvar.unsqueeze(1)).to(x.scalar_type()).view(x.sizes());
    at::Tensor dgam, dbet;
    if (need_wgrad && has(gamma)) dgam = (df * xh).sum(0).to(gamma->scalar_type());
    if (need_bgrad && has(gamma)) dbet = df.sum(0).to(gamma->scalar_type());
    return {dx, dgam, dbet};
  }
  at::Tensor g = has(gamma) ? gamma->contiguous() : at::Tensor();
  at::Tensor dx = at::empty_like(x);
  at::Tensor dgam, dbet, part;
  DType tw = g.defined() ? dtype_of(g) : DType::F32;
  if (need_wgrad && g.defined()) dgam = at::empty_like(g);
  if (need_bgrad && g.defined()) dbet = at::empty_like(g);
  if (dgam.defined() || dbet.defined())
    part = at::empty({layer_norm_bwd_workspace(n1, n2)}, x.options().dtype(at::kFloat));
  layer_norm_bwd(dy.data_ptr(), x.data_ptr(), dtype_of(x), g.defined() ? g.data_ptr() : nullptr,
                 tw, mean.data_ptr<float>(), invvar.data_ptr<float>(), dx.data_ptr(),
                 dgam.defined() ? dgam.data_ptr() : nullptr,
                 dbet.defined() ? dbet.data_ptr() : nullptr,
                 part.defined() ? part.data_ptr<float>() : nullptr, n1, n2, rms ? 1 : 0,
                 cur_stream());
  return {dx, dgam, dbet};
}

// ----------------------------------------------- residual + dropout + LayerNorm (GPU)
namespace {
LnFuse make_fuse(double p, int64_t seed) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  LnFuse f;
  f.seed = (uint32_t)(seed & 0xFFFFFFFF) ^ (uint32_t)((uint64_t)seed >> 32);
  const double t = p * 4294967296.0;
  f.thresh = (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t);
  f.scale = (float)(1.0 / (1.0 - p));
  return f;
}
}  // namespace

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> add_dropout_layer_norm_forward_op(
    at::Tensor x, at::Tensor h, int64_t n2, OptT gamma, OptT beta, double eps, double p,
    int64_t seed, bool y_as_h) {
  TORCH_CHECK(x.is_cuda() && h.is_cuda(), "add_dropout_layer_norm: GPU tensors only");
  // h is x's type, or 16-bit under an fp32 residual stream (amp O1)
  const bool mixed = x.scalar_type() == at::kFloat &&
                     (h.scalar_type() == at::kHalf || h.scalar_type() == at::kBFloat16);
  TORCH_CHECK(x.sizes() == h.sizes() && (x.scalar_type() == h.scalar_type() || mixed),
              "add_dropout_layer_norm: residual / sublayer output mismatch");
  x = x.contiguous();
  h = h.contiguous();
  const int64_t n1 = x.numel() / n2;
  at::Tensor g = has(gamma) ? gamma->contiguous() : at::Tensor();
  at::Tensor b = has(beta) ? beta->contiguous() : at::Tensor();
  // y_as_h (mixed only): emit y in h's 16-bit type for an autocast GEMM consumer
  const bool y16 = mixed && y_as_h;
  at::Tensor y = y16 ? at::empty_like(x, x.options().dtype(h.scalar_type())) : at::empty_like(x);
  at::Tensor s = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({n1}, fopt), invvar = at::empty({n1}, fopt);
  TORCH_CHECK(layer_norm_fused_ok(x.data_ptr(), h.data_ptr(), s.data_ptr(),
                                  g.defined() ? g.data_ptr() : nullptr,
                                  b.defined() ? b.data_ptr() : nullptr, y.data_ptr(), n2),
              "add_dropout_layer_norm: needs n2 % 8 == 0, n2 <= 2048 and 16-byte aligned rows");
  LnFuse f = make_fuse(p, seed);
  f.h = h.data_ptr();
  f.s = s.data_ptr();
  if (mixed) f.th = (int)dtype_of(h);
  if (y16) f.ty = f.th;
  DType tw = g.defined() ? dtype_of(g) : (b.defined() ? dtype_of(b) : DType::F32);
  layer_norm_fwd(x.data_ptr(), dtype_of(x), g.defined() ? g.data_ptr() : nullptr,
                 b.defined() ? b.data_ptr() : nullptr, tw, y.data_ptr(), mean.data_ptr<float>(),
                 invvar.data_ptr<float>(), n1, n2, (float)eps, 0, cur_stream(), &f);
  return {y, s, mean, invvar};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
add_dropout_layer_norm_backward_op(at::Tensor dy, at::Tensor s, at::Tensor mean, at::Tensor invvar,
                                   int64_t n2, OptT gamma, OptT dres, double p, int64_t seed,
                                   bool need_wgrad, bool need_bgrad,
                                   c10::optional<at::ScalarType> h_dtype, bool need_hsum) {
  TORCH_CHECK(s.is_cuda(), "add_dropout_layer_norm: GPU tensors only");
  s = s.contiguous();
  dy = dy.contiguous();
  at::Tensor e = has(dres) ? dres->contiguous() : at::Tensor();
  const int64_t n1 = s.numel() / n2;
  at::Tensor g = has(gamma) ? gamma->contiguous() : at::Tensor();
  const bool mixed = h_dtype.has_value() && *h_dtype != s.scalar_type();
  TORCH_CHECK(!mixed || (s.scalar_type() == at::kFloat &&
                         (*h_dtype == at::kHalf || *h_dtype == at::kBFloat16)),
              "add_dropout_layer_norm: 16-bit sublayer output needs an fp32 residual");
  at::Tensor ds = at::empty_like(s);
  at::Tensor dh = mixed ? at::empty_like(s, s.options().dtype(*h_dtype)) : at::empty_like(s);
  auto al = [](const at::Tensor& t) { return !t.defined() || ((uintptr_t)t.data_ptr() % 16) == 0; };
  TORCH_CHECK(layer_norm_fused_ok(s.data_ptr(), dh.data_ptr(), ds.data_ptr(),
                                  g.defined() ? g.data_ptr() : nullptr, nullptr, dy.data_ptr(),
                                  n2) && al(e),
              "add_dropout_layer_norm: needs n2 % 8 == 0, n2 <= 2048 and 16-byte aligned rows");
  at::Tensor dgam, dbet, part;
  DType tw = g.defined() ? dtype_of(g) : DType::F32;
  if (need_wgrad && g.defined()) dgam = at::empty_like(g);
  if (need_bgrad && g.defined()) dbet = at::empty_like(g);
  // column sums of dh (in gamma's dtype) with the dgamma / dbeta partials: the bias
  // gradient of the dense layer whose output h is (fused_dense picks it up)
  at::Tensor dhs;
  if (need_hsum && (dgam.defined() || dbet.defined()) && layer_norm_bwd_hsum_ok(n2))
    dhs = at::empty_like(g);
  if (dgam.defined() || dbet.defined())
    part = at::empty({layer_norm_bwd_workspace(n1, n2)}, s.options().dtype(at::kFloat));
  LnFuse f = make_fuse(p, seed);
  f.dhsum = dhs.defined() ? dhs.data_ptr() : nullptr;
  f.dres = e.defined() ? e.data_ptr() : nullptr;
  f.dh = dh.data_ptr();
  if (mixed) f.th = (int)dtype_of(dh);
  if (mixed && dy.scalar_type() == dh.scalar_type()) f.ty = f.th;  // 16-bit y's gradient
  TORCH_CHECK(dy.scalar_type() == s.scalar_type() || f.ty >= 0,
              "add_dropout_layer_norm: dy dtype matches neither s nor h");
  layer_norm_bwd(dy.data_ptr(), s.data_ptr(), dtype_of(s), g.defined() ? g.data_ptr() : nullptr,
                 tw, mean.data_ptr<float>(), invvar.data_ptr<float>(), ds.data_ptr(),
                 dgam.defined() ? dgam.data_ptr() : nullptr,
                 dbet.defined() ? dbet.data_ptr() : nullptr,
                 part.defined() ? part.data_ptr<float>() : nullptr, n1, n2, 0, cur_stream(), &f);
  return {ds, dh, dgam, dbet, dhs};
}

// ============================================================================ BatchNorm
namespace {
struct BNView {
  int64_t outer, C, inner;
  int cl;
  bool cl4;  // 4-D tensor stored channels_last
};

BNView bn_view(const at::Tensor& x) {
  TORCH_CHECK(x.dim() >= 2, "batch norm expects [N, C, ...]");
  BNView v;
  const int64_t N = x.size(0), C = x.size(1);
  int64_t HW = 1;
  for (int64_t d = 2; d < x.dim(); ++d) HW *= x.size(d);
  v.C = C;
  v.cl4 = false;
  if (HW == 1) {
    v.outer = N;
    v.inner = 1;
    v.cl = 1;
  } else if (x.dim() == 4 && !x.is_contiguous() &&
             x.is_contiguous(at::MemoryFormat::ChannelsLast)) {
    v.outer = N * HW;
    v.inner = 1;
    v.cl = 1;
    v.cl4 = true;
  } else {
    v.outer = N;
    v.inner = HW;
    v.cl = 0;
  }
  return v;
}

at::Tensor conform(const at::Tensor& t, const BNView& v) {
  return v.cl4 ? t.contiguous(at::MemoryFormat::ChannelsLast) : t.contiguous();
}

bool aligned16(const at::Tensor& t) { return !t.defined() || ((uintptr_t)t.data_ptr() % 16) == 0; }

// mirrors the NHWC launchers' VEC condition, under which apply writes the mask
bool relu_mask_ok(const BNView& v, bool relu, const at::Tensor& x, const at::Tensor& z,
                  const at::Tensor& y) {
  return relu && x.is_cuda() && v.cl == 1 && v.C % 8 == 0 && aligned16(x) && aligned16(z) &&
         aligned16(y);
}

const uint8_t* mask_ptr(const OptT& m, const at::Tensor& x, const BNView& v) {
  if (!has(m)) return nullptr;
  TORCH_CHECK(x.is_cuda() && v.cl == 1 && m->scalar_type() == at::kByte && m->is_contiguous() &&
                  m->numel() == v.outer * (v.C / 8),
              "batch norm: bad ReLU mask");
  return m->data_ptr<uint8_t>();
}

std::vector<int64_t> reduce_dims(const at::Tensor& x) {
  std::vector<int64_t> d{0};
  for (int64_t i = 2; i < x.dim(); ++i) d.push_back(i);
  return d;
}

at::Tensor chan(const at::Tensor& t, int64_t dim) {
  std::vector<int64_t> shape((size_t)dim, 1);
  shape[1] = t.numel();
  return t.view(shape);
}
}  // namespace

std::tuple<at::Tensor, at::Tensor> bn_local_stats_op(at::Tensor x) {
  BNView v = bn_view(x);
  auto fopt = x.options().dtype(at::kFloat);
  if (!x.is_cuda()) {
    at::Tensor xf = x.to(at::kFloat);
    auto dims = reduce_dims(x);
    at::Tensor mean = xf.mean(dims);
    at::Tensor var = xf.var(dims, /*unbiased=*/false);
    return {mean, var};
  }
  x = conform(x, v);
  at::Tensor mean = at::empty({v.C}, fopt), var = at::empty({v.C}, fopt);
  at::Tensor ws = at::empty({bn_stats_workspace(v.outer, v.C, v.inner, v.cl)}, fopt);
  bn_local_stats(x.data_ptr(), dtype_of(x), v.outer, v.C, v.inner, v.cl, mean.data_ptr<float>(),
                 var.data_ptr<float>(), ws.data_ptr<float>(), cur_stream());
  return {mean, var};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_combine_stats_op(at::Tensor means,
                                                                   at::Tensor vars,
                                                                   at::Tensor counts, double eps,
                                                                   double momentum,
                                                                   OptT running_mean,
                                                                   OptT running_var) {
  means = means.contiguous().to(at::kFloat);
  vars = vars.contiguous().to(at::kFloat);
  counts = counts.contiguous().to(at::kFloat);
  const int64_t world = means.dim() == 1 ? 1 : means.size(0);
  const int64_t C = means.size(-1);
  const bool rs = has(running_mean) && has(running_var);
  const bool fast_rs = !rs || (running_mean->scalar_type() == at::kFloat &&
                               running_var->scalar_type() == at::kFloat &&
                               running_mean->is_contiguous() && running_var->is_contiguous());
  if (!means.is_cuda() || !fast_rs) {
    at::Tensor m2 = means.view({world, C}), v2 = vars.view({world, C});
    at::Tensor n = counts.view({world, 1});
    at::Tensor N = n.sum();
    at::Tensor mean = (m2 * n).sum(0) / N;
    at::Tensor M2 = (v2 * n).sum(0) + ((m2 - mean.unsqueeze(0)).pow(2) * n).sum(0);
    at::Tensor var_b = M2 / N;
    at::Tensor invstd = (var_b + eps).rsqrt();
    if (rs) {
      at::Tensor unb = at::where(N > 1, M2 / (N - 1), var_b);
      c10::NoGradGuard ng;
      running_mean->mul_(1.0 - momentum).add_(mean.to(running_mean->scalar_type()), momentum);
      running_var->mul_(1.0 - momentum).add_(unb.to(running_var->scalar_type()), momentum);
    }
    return {mean, invstd, var_b};
  }
  auto fopt = means.options();
  at::Tensor mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt), var = at::empty({C}, fopt);
  bn_combine_stats(means.data_ptr<float>(), vars.data_ptr<float>(), counts.data_ptr<float>(),
                   (int)world, C, (float)eps, (float)momentum, mean.data_ptr<float>(),
                   invstd.data_ptr<float>(), rs ? running_mean->data_ptr<float>() : nullptr,
                   DType::F32, rs ? running_var->data_ptr() : nullptr, var.data_ptr<float>(),
                   cur_stream());
  return {mean, invstd, var};
}

// SyncBN forward, local part: [mean(C) | var(C) | count] in ONE buffer written by the
// stats kernels (the count by the finalize kernel), ready for the all_gather
// `out`: write into that contiguous fp32 [2C+1] buffer instead (the caller's slot of the
// all_gather destination: the gather then runs in place, no send-buffer copy)
static at::Tensor packed_out(OptT out, int64_t C, const at::TensorOptions& fopt) {
  if (!has(out)) return at::empty({2 * C + 1}, fopt);
  TORCH_CHECK(out->is_cuda() && out->scalar_type() == at::kFloat && out->is_contiguous() &&
                  out->numel() == 2 * C + 1,
              "bn packed stats: out must be a contiguous fp32 [2C+1] GPU tensor");
  return *out;
}

at::Tensor bn_local_stats_packed_op(at::Tensor x, OptT out) {
  c10::NoGradGuard no_grad_;
  BNView v = bn_view(x);
  if (!x.is_cuda()) {
    auto st = bn_local_stats_op(x);
    return at::cat({std::get<0>(st), std::get<1>(st),
                    at::full({1}, (double)(v.outer * v.inner), std::get<0>(st).options())});
  }
  x = conform(x, v);
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor packed = packed_out(out, v.C, fopt);
  at::Tensor ws = at::empty({bn_stats_workspace(v.outer, v.C, v.inner, v.cl)}, fopt);
  float* p = packed.data_ptr<float>();
  bn_local_stats(x.data_ptr(), dtype_of(x), v.outer, v.C, v.inner, v.cl, p, p + v.C,
                 ws.data_ptr<float>(), cur_stream(), p + 2 * v.C);
  return packed;
}

// SyncBN forward, global part: combine the gathered [world, 2C+1] stats; running stats,
// num_batches_tracked and 1/global-count (for the backward) in the same kernel
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_combine_stats_sync_op(
    at::Tensor gathered, double eps, double momentum, OptT running_mean, OptT running_var,
    OptT nbt) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(gathered.dim() == 2 && (gathered.size(1) - 1) % 2 == 0,
              "combine_stats_sync: [world, 2C+1] expected");
  const int64_t world = gathered.size(0), C = (gathered.size(1) - 1) / 2;
  gathered = gathered.contiguous().to(at::kFloat);
  const bool rs = has(running_mean) && has(running_var);
  const bool fast = gathered.is_cuda() &&
                    (!rs || (running_mean->scalar_type() == at::kFloat &&
                             running_var->scalar_type() == at::kFloat &&
                             running_mean->is_contiguous() && running_var->is_contiguous())) &&
                    (!has(nbt) || nbt->scalar_type() == at::kLong);
  if (!fast) {
    at::Tensor means = gathered.narrow(1, 0, C), vars = gathered.narrow(1, C, C);
    at::Tensor counts = gathered.narrow(1, 2 * C, 1).reshape({world});
    auto cs = bn_combine_stats_op(means, vars, counts, eps, momentum, running_mean, running_var);
    if (has(nbt)) nbt->add_(1);
    return {std::get<0>(cs), std::get<1>(cs), counts.sum().reciprocal().reshape({1})};
  }
  // the kernel reads means / vars / counts with row stride C: copy to planar once
  // (world x (2C+1) floats, tiny)
  at::Tensor means = gathered.narrow(1, 0, C).contiguous();
  at::Tensor vars = gathered.narrow(1, C, C).contiguous();
  at::Tensor counts = gathered.narrow(1, 2 * C, 1).contiguous();
  auto fopt = gathered.options();
  at::Tensor mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  at::Tensor inv_total = at::empty({1}, fopt);
  bn_combine_stats(means.data_ptr<float>(), vars.data_ptr<float>(), counts.data_ptr<float>(),
                   (int)world, C, (float)eps, (float)momentum, mean.data_ptr<float>(),
                   invstd.data_ptr<float>(), rs ? running_mean->data_ptr<float>() : nullptr,
                   DType::F32, rs ? running_var->data_ptr() : nullptr, nullptr, cur_stream(),
                   has(nbt) ? reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()) : nullptr,
                   inv_total.data_ptr<float>());
  return {mean, invstd, inv_total};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_forward_local_op(
    at::Tensor x, OptT weight, OptT bias, OptT running_mean, OptT running_var, OptT nbt,
    double eps, double momentum, OptT z, bool relu, bool want_mask) {
  c10::NoGradGuard no_grad_;
  const bool rs = has(running_mean) && has(running_var);
  auto f32c = [](const OptT& t) {
    return t->scalar_type() == at::kFloat && t->is_contiguous() && t->is_cuda();
  };
  const bool fast = x.is_cuda() && (!rs || (f32c(running_mean) && f32c(running_var))) &&
                    (!has(nbt) || (nbt->scalar_type() == at::kLong && nbt->is_cuda()));
  if (!fast) {
    auto st = bn_local_stats_op(x);
    BNView v = bn_view(x);
    at::Tensor counts = at::full({1}, (double)(v.outer * v.inner),
                                 x.options().dtype(at::kFloat));
    auto cs = bn_combine_stats_op(std::get<0>(st), std::get<1>(st), counts, eps, momentum,
                                  running_mean, running_var);
    if (has(nbt)) nbt->add_(1);
    auto ym = want_mask ? bn_apply_mask_op(x, std::get<0>(cs), std::get<1>(cs), weight, bias, z,
                                           relu)
                        : std::make_tuple(bn_apply_op(x, std::get<0>(cs), std::get<1>(cs), weight,
                                                      bias, z, relu),
                                          at::Tensor());
    return {std::get<0>(ym), std::get<0>(cs), std::get<1>(cs), std::get<1>(ym)};
  }
  BNView v = bn_view(x);
  x = conform(x, v);
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({v.C}, fopt), invstd = at::empty({v.C}, fopt);
  at::Tensor ws = at::empty({bn_stats_workspace(v.outer, v.C, v.inner, v.cl)}, fopt);
  bn_local_train_stats(x.data_ptr(), dtype_of(x), v.outer, v.C, v.inner, v.cl,
                       mean.data_ptr<float>(), invstd.data_ptr<float>(),
                       rs ? running_mean->data_ptr<float>() : nullptr,
                       rs ? running_var->data_ptr<float>() : nullptr,
                       has(nbt) ? reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()) : nullptr,
                       (float)eps, (float)momentum, ws.data_ptr<float>(), cur_stream());
  if (want_mask) {
    auto ym = bn_apply_mask_op(x, mean, invstd, weight, bias, z, relu);
    return {std::get<0>(ym), mean, invstd, std::get<1>(ym)};
  }
  at::Tensor y = bn_apply_op(x, mean, invstd, weight, bias, z, relu);
  return {y, mean, invstd, at::Tensor()};
}

std::tuple<at::Tensor, at::Tensor> bn_train_stats_op(at::Tensor x, OptT running_mean,
                                                      OptT running_var, OptT nbt, double eps,
                                                      double momentum) {
  // training statistics only (mean, invstd; running stats + num_batches_tracked
  // updated in the finalize kernel) for consumers that apply the BatchNorm
  // themselves (the ResNet stem's fused BN + ReLU + max-pool)
  c10::NoGradGuard no_grad_;
  const bool rs = has(running_mean) && has(running_var);
  TORCH_CHECK(x.is_cuda() && (!rs || (running_mean->scalar_type() == at::kFloat &&
                                      running_var->scalar_type() == at::kFloat &&
                                      running_mean->is_contiguous() &&
                                      running_var->is_contiguous())) &&
                  (!has(nbt) || nbt->scalar_type() == at::kLong),
              "bn.train_stats: GPU tensor, fp32 contiguous running stats, int64 counter");
  BNView v = bn_view(x);
  x = conform(x, v);
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({v.C}, fopt), invstd = at::empty({v.C}, fopt);
  at::Tensor ws = at::empty({bn_stats_workspace(v.outer, v.C, v.inner, v.cl)}, fopt);
  bn_local_train_stats(x.data_ptr(), dtype_of(x), v.outer, v.C, v.inner, v.cl,
                       mean.data_ptr<float>(), invstd.data_ptr<float>(),
                       rs ? running_mean->data_ptr<float>() : nullptr,
                       rs ? running_var->data_ptr<float>() : nullptr,
                       has(nbt) ? reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()) : nullptr,
                       (float)eps, (float)momentum, ws.data_ptr<float>(), cur_stream());
  return {mean, invstd};
}

static std::tuple<at::Tensor, at::Tensor> bn_apply_impl(at::Tensor x, at::Tensor mean,
                                                        at::Tensor invstd, OptT weight, OptT bias,
                                                        OptT z, bool relu, bool want_mask) {
  BNView v = bn_view(x);
  if (!x.is_cuda()) {
    const int64_t d = x.dim();
    at::Tensor sc = invstd * (has(weight) ? weight->to(at::kFloat) : at::ones_like(invstd));
    at::Tensor sh = (has(bias) ? bias->to(at::kFloat) : at::zeros_like(mean)) - mean * sc;
    at::Tensor y = x.to(at::kFloat) * chan(sc, d) + chan(sh, d);
    if (has(z)) y = y + z->to(at::kFloat);
    if (relu) y = y.clamp_min(0);
    return {y.to(x.scalar_type()), at::Tensor()};
  }
  x = conform(x, v);
  at::Tensor zc = has(z) ? conform(*z, v) : at::Tensor();
  at::Tensor y = at::empty_like(x);
  at::Tensor mask;
  if (want_mask && relu_mask_ok(v, relu, x, zc, y))
    mask = at::empty({v.outer, v.C / 8}, x.options().dtype(at::kByte));
  DType tw = has(weight) ? dtype_of(*weight) : DType::F32;
  at::Tensor w = has(weight) ? weight->contiguous() : at::Tensor();
  at::Tensor b = has(bias) ? bias->contiguous() : at::Tensor();
  bn_apply(x.data_ptr(), dtype_of(x), mean.data_ptr<float>(), invstd.data_ptr<float>(),
           w.defined() ? w.data_ptr() : nullptr, b.defined() ? b.data_ptr() : nullptr, tw,
           zc.defined() ? zc.data_ptr() : nullptr,
           mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, y.data_ptr(), v.outer, v.C,
           v.inner, v.cl, relu ? 1 : 0, cur_stream());
  return {y, mask};
}

at::Tensor bn_apply_op(at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
                       OptT z, bool relu) {
  return std::get<0>(bn_apply_impl(x, mean, invstd, weight, bias, z, relu, false));
}

std::tuple<at::Tensor, at::Tensor> bn_apply_mask_op(at::Tensor x, at::Tensor mean,
                                                    at::Tensor invstd, OptT weight, OptT bias,
                                                    OptT z, bool relu) {
  return bn_apply_impl(x, mean, invstd, weight, bias, z, relu, true);
}

namespace {
// dgamma / dbeta destinations: fresh tensors, or caller-given gradients to ACCUMULATE into
// (DDP bucket views; the finalize adds instead of writing - BNAccumScope)
// (accumulate = false: the given targets are lazily zeroed DDP bucket views, overwritten)
bool grad_targets(const OptT& weight, bool need, const OptT& gw_in, const OptT& gb_in,
                  at::Tensor& gw, at::Tensor& gb, bool accumulate = true) {
  if (!need || !has(weight)) return false;
  if (has(gw_in) && has(gb_in)) {
    TORCH_CHECK(gw_in->is_cuda() && gb_in->is_cuda() && gw_in->is_contiguous() &&
                    gb_in->is_contiguous() && gw_in->numel() == weight->numel() &&
                    gb_in->numel() == weight->numel() &&
                    gw_in->scalar_type() == weight->scalar_type() &&
                    gb_in->scalar_type() == weight->scalar_type(),
                "batch norm: grad_weight / grad_bias targets must match the weight");
    gw = *gw_in;
    gb = *gb_in;
    return accumulate;
  }
  gw = at::empty_like(*weight);
  gb = at::empty_like(*weight);
  return false;
}
}  // namespace

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_reduce_grad_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
    OptT z, bool relu, bool need_wgrad, OptT mask, OptT sum_scale, OptT gw_in, OptT gb_in,
    bool accumulate) {
  BNView v = bn_view(x);
  TORCH_CHECK(!has(mask) || x.is_cuda(), "batch norm: ReLU mask is a GPU-path feature");
  if (!x.is_cuda()) {
    const int64_t d = x.dim();
    at::Tensor xf = x.to(at::kFloat), df = dy.to(at::kFloat);
    if (relu) {
      at::Tensor y = bn_apply_op(x, mean, invstd, weight, bias, z, false).to(at::kFloat);
      df = df * (y > 0).to(at::kFloat);
    }
    auto dims = reduce_dims(x);
    at::Tensor sum_dy = df.sum(dims);
    at::Tensor sum_dy_xmu = (df * (xf - chan(mean, d))).sum(dims);
    at::Tensor gw, gb;
    if (need_wgrad && has(weight)) {
      gw = (sum_dy_xmu * invstd).to(weight->scalar_type());
      gb = sum_dy.to(weight->scalar_type());
      if (has(gw_in) && has(gb_in)) {
        gw_in->add_(gw);
        gb_in->add_(gb);
        gw = *gw_in;
        gb = *gb_in;
      }
    }
    if (has(sum_scale)) {
      sum_dy = sum_dy * *sum_scale;
      sum_dy_xmu = sum_dy_xmu * *sum_scale;
    }
    return {sum_dy, sum_dy_xmu, gw, gb};
  }
  x = conform(x, v);
  dy = conform(dy, v);
  const uint8_t* mk = mask_ptr(mask, x, v);
  at::Tensor zc = (has(z) && !mk) ? conform(*z, v) : at::Tensor();
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor sum_dy = at::empty({v.C}, fopt), sum_dy_xmu = at::empty({v.C}, fopt);
  at::Tensor gw, gb;
  DType tw = has(weight) ? dtype_of(*weight) : DType::F32;
  const bool accum = grad_targets(weight, need_wgrad, gw_in, gb_in, gw, gb, accumulate);
  BNAccumScope accum_scope(accum);
  at::Tensor w = has(weight) ? weight->contiguous() : at::Tensor();
  at::Tensor b = has(bias) ? bias->contiguous() : at::Tensor();
  at::Tensor ws = at::empty({bn_stats_workspace(v.outer, v.C, v.inner, v.cl)}, fopt);
  const float* scale = nullptr;
  if (has(sum_scale)) {
    TORCH_CHECK(sum_scale->is_cuda() && sum_scale->scalar_type() == at::kFloat &&
                    sum_scale->numel() == 1, "reduce_grad: sum_scale must be a 1-element fp32 GPU tensor");
    scale = sum_scale->data_ptr<float>();
    // one [2C] buffer (sum_dy | sum_dy_xmu) for SyncBN's all_reduce
    at::Tensor packed = at::empty({2 * v.C}, fopt);
    sum_dy = packed.narrow(0, 0, v.C);
    sum_dy_xmu = packed.narrow(0, v.C, v.C);
  }
  bn_reduce_grad(dy.data_ptr(), x.data_ptr(), dtype_of(x), mean.data_ptr<float>(),
                 invstd.data_ptr<float>(), w.defined() ? w.data_ptr() : nullptr,
                 b.defined() ? b.data_ptr() : nullptr, tw, relu ? 1 : 0,
                 zc.defined() ? zc.data_ptr() : nullptr, mk, v.outer, v.C, v.inner, v.cl,
                 sum_dy.data_ptr<float>(), sum_dy_xmu.data_ptr<float>(),
                 gw.defined() ? gw.data_ptr() : nullptr, gb.defined() ? gb.data_ptr() : nullptr,
                 ws.data_ptr<float>(), cur_stream(), scale);
  return {sum_dy, sum_dy_xmu, gw, gb};
}

std::tuple<at::Tensor, at::Tensor> bn_backward_elemt_op(at::Tensor dy, at::Tensor x,
                                                        at::Tensor mean, at::Tensor invstd,
                                                        OptT weight, OptT bias, at::Tensor sum_dy,
                                                        at::Tensor sum_dy_xmu, double count,
                                                        OptT z, bool relu, bool want_dz,
                                                        OptT mask) {
  BNView v = bn_view(x);
  TORCH_CHECK(!has(mask) || x.is_cuda(), "batch norm: ReLU mask is a GPU-path feature");
  if (!x.is_cuda()) {
    const int64_t d = x.dim();
    at::Tensor xf = x.to(at::kFloat), df = dy.to(at::kFloat);
    if (relu) {
      at::Tensor y = bn_apply_op(x, mean, invstd, weight, bias, z, false).to(at::kFloat);
      df = df * (y > 0).to(at::kFloat);
    }
    at::Tensor w = has(weight) ? weight->to(at::kFloat) : at::ones_like(invstd);
    at::Tensor mdy = sum_dy / count, mdyx = sum_dy_xmu / count;
    at::Tensor dx = (df - chan(mdy, d) - (xf - chan(mean, d)) * chan(invstd * invstd * mdyx, d)) *
                    chan(invstd * w, d);
    at::Tensor dz = want_dz ? df.to(x.scalar_type()) : at::Tensor();
    return {dx.to(x.scalar_type()), dz};
  }
  x = conform(x, v);
  dy = conform(dy, v);
  const uint8_t* mk = mask_ptr(mask, x, v);
  at::Tensor zc = (has(z) && !mk) ? conform(*z, v) : at::Tensor();
  at::Tensor dx = at::empty_like(x);
  at::Tensor dz = want_dz ? at::empty_like(x) : at::Tensor();
  DType tw = has(weight) ? dtype_of(*weight) : DType::F32;
  at::Tensor w = has(weight) ? weight->contiguous() : at::Tensor();
  at::Tensor b = has(bias) ? bias->contiguous() : at::Tensor();
  bn_backward_elemt(dy.data_ptr(), x.data_ptr(), dtype_of(x), mean.data_ptr<float>(),
                    invstd.data_ptr<float>(), w.defined() ? w.data_ptr() : nullptr,
                    b.defined() ? b.data_ptr() : nullptr, tw, sum_dy.data_ptr<float>(),
                    sum_dy_xmu.data_ptr<float>(), (float)(1.0 / count), relu ? 1 : 0,
                    zc.defined() ? zc.data_ptr() : nullptr, mk, dx.data_ptr(),
                    dz.defined() ? dz.data_ptr() : nullptr, v.outer, v.C, v.inner, v.cl,
                    cur_stream());
  return {dx, dz};
}

// backward_elemt (no ReLU / z / mask) plus the backward sums of a SECOND BatchNorm over the
// same rows whose gradient is this dy (ResNet's downsample BN, whose output was this BN's
// residual input): (dx, sum_dy2, sum_dy_xmu2, gw2, gb2) - that BN then runs only its
// elementwise pass.  GPU, channels-last, C % 8 == 0, 16-byte aligned rows only (the caller
// checks bn.backward_x2_ok).
bool bn_backward_x2_ok(at::Tensor dy, at::Tensor x, at::Tensor x2) {
  if (!(dy.is_cuda() && x.is_cuda() && x2.is_cuda())) return false;
  if (x.sizes() != x2.sizes() || dy.sizes() != x.sizes()) return false;
  if (x.scalar_type() != x2.scalar_type() || dy.scalar_type() != x.scalar_type()) return false;
  if (x.scalar_type() == at::kFloat) return false;
  BNView v = bn_view(x);
  if (!v.cl || v.C % 8 != 0) return false;
  for (const at::Tensor* t : {&dy, &x, &x2}) {
    const at::Tensor c = conform(*t, v);
    if (!c.is_same(*t) || (uintptr_t)t->data_ptr() % 16 != 0) return false;
  }
  return true;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_backward_elemt_x2_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
    at::Tensor sum_dy, at::Tensor sum_dy_xmu, double count, at::Tensor x2, at::Tensor mean2,
    at::Tensor invstd2, OptT weight2, bool need_wgrad2) {
  TORCH_CHECK(bn_backward_x2_ok(dy, x, x2), "backward_elemt_x2: see bn_backward_x2_ok");
  BNView v = bn_view(x);
  auto f32c = [&](const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == v.C,
                "backward_elemt_x2: ", what, " must be fp32 [C]");
  };
  f32c(mean, "mean");
  f32c(invstd, "invstd");
  f32c(mean2, "mean2");
  f32c(invstd2, "invstd2");
  f32c(sum_dy, "sum_dy");
  f32c(sum_dy_xmu, "sum_dy_xmu");
  DType tw = has(weight) ? dtype_of(*weight) : DType::F32;
  TORCH_CHECK(!has(weight2) || dtype_of(*weight2) == tw,
              "backward_elemt_x2: both BNs' weights must share a dtype");
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x);
  at::Tensor sum_dy2 = at::empty({v.C}, fopt), sum_dy_xmu2 = at::empty({v.C}, fopt);
  at::Tensor gw2, gb2;
  const bool accum = grad_targets(weight2, need_wgrad2, c10::nullopt, c10::nullopt, gw2, gb2);
  BNAccumScope accum_scope(accum);
  at::Tensor w = has(weight) ? weight->contiguous() : at::Tensor();
  at::Tensor b = has(bias) ? bias->contiguous() : at::Tensor();
  at::Tensor ws = at::empty({nhwc_backward_x2_workspace(v.outer, v.C, dtype_of(x))}, fopt);
  nhwc_backward_x2(dy.data_ptr(), x.data_ptr(), dtype_of(x), mean.data_ptr<float>(),
                   invstd.data_ptr<float>(), w.defined() ? w.data_ptr() : nullptr,
                   b.defined() ? b.data_ptr() : nullptr, tw, sum_dy.data_ptr<float>(),
                   sum_dy_xmu.data_ptr<float>(), (float)(1.0 / count), dx.data_ptr(), v.outer, v.C,
                   x2.data_ptr(), mean2.data_ptr<float>(), invstd2.data_ptr<float>(),
                   sum_dy2.data_ptr<float>(), sum_dy_xmu2.data_ptr<float>(),
                   gw2.defined() ? gw2.data_ptr() : nullptr, gb2.defined() ? gb2.data_ptr() : nullptr,
                   ws.data_ptr<float>(), cur_stream());
  return {dx, sum_dy2, sum_dy_xmu2, gw2, gb2};
}

// y = relu(BN(x) + BNz(xz)) and its ReLU mask in one pass (the residual BN's output is never
// stored); GPU, channels-last, C % 8 == 0, 16-byte aligned (bn_backward_x2_ok's conditions)
std::tuple<at::Tensor, at::Tensor> bn_apply2_mask_op(at::Tensor x, at::Tensor mean,
                                                     at::Tensor invstd, OptT weight, OptT bias,
                                                     at::Tensor xz, at::Tensor meanz,
                                                     at::Tensor invstdz, OptT weightz,
                                                     OptT biasz) {
  TORCH_CHECK(bn_backward_x2_ok(x, x, xz), "apply2: GPU channels-last 16-bit x / xz of one shape");
  BNView v = bn_view(x);
  DType tw = has(weight) ? dtype_of(*weight) : DType::F32;
  TORCH_CHECK((has(weightz) ? dtype_of(*weightz) : DType::F32) == tw &&
                  (has(bias) ? dtype_of(*bias) : tw) == tw &&
                  (has(biasz) ? dtype_of(*biasz) : tw) == tw,
              "apply2: one parameter dtype");
  for (const at::Tensor* t : {&mean, &invstd, &meanz, &invstdz})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == v.C,
                "apply2: statistics must be fp32 [C]");
  at::Tensor y = at::empty_like(x);
  at::Tensor mask = at::empty({v.outer, v.C / 8}, x.options().dtype(at::kByte));
  auto ptr = [](const OptT& t) -> at::Tensor { return has(t) ? t->contiguous() : at::Tensor(); };
  at::Tensor w = ptr(weight), b = ptr(bias), wz = ptr(weightz), bz = ptr(biasz);
  nhwc_apply2(x.data_ptr(), dtype_of(x), mean.data_ptr<float>(), invstd.data_ptr<float>(),
              w.defined() ? w.data_ptr() : nullptr, b.defined() ? b.data_ptr() : nullptr, tw,
              xz.data_ptr(), meanz.data_ptr<float>(), invstdz.data_ptr<float>(),
              wz.defined() ? wz.data_ptr() : nullptr, bz.defined() ? bz.data_ptr() : nullptr,
              mask.data_ptr<uint8_t>(), y.data_ptr(), v.outer, v.C, cur_stream());
  return {y, mask};
}

// Local (world 1) backward: reduce_grad + backward_elemt.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_backward_local_op(
    at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd, OptT weight, OptT bias,
    OptT z, bool relu, bool need_wgrad, bool want_dz, OptT mask) {
  BNView v = bn_view(x);
  auto r = bn_reduce_grad_op(dy, x, mean, invstd, weight, bias, z, relu, need_wgrad, mask,
                             c10::nullopt);
  const double count = (double)(v.outer * v.inner);
  auto e = bn_backward_elemt_op(dy, x, mean, invstd, weight, bias, std::get<0>(r), std::get<1>(r),
                                count, z, relu, want_dz, mask);
  return {std::get<0>(e), std::get<1>(e), std::get<2>(r), std::get<3>(r)};
}


std::tuple<at::Tensor, at::Tensor> bn_slab_train_stats_op(at::Tensor slab, int64_t count,
                                                          OptT shift, OptT running_mean,
                                                          OptT running_var, OptT nbt,
                                                          double eps, double momentum) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(slab.is_cuda() && slab.dim() == 3 && slab.size(0) == 2 &&
                  slab.scalar_type() == at::kFloat && slab.is_contiguous(),
              "bn slab stats: fp32 [2][C][S] slab expected");
  const int64_t S = slab.size(2), C = slab.size(1);
  auto f32 = [&](const OptT& t, const char* what) -> float* {
    if (!has(t)) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C &&
                    t->is_cuda(),
                "bn slab stats: ", what, " must be a contiguous fp32 [C] GPU tensor");
    return t->data_ptr<float>();
  };
  const float* sp = f32(shift, "shift");
  float* rm = f32(running_mean, "running_mean");
  float* rv = f32(running_var, "running_var");
  long long* nb = nullptr;
  if (has(nbt)) {
    TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "nbt: int64 GPU tensor");
    nb = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  }
  auto fopt = slab.options();
  at::Tensor mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  bn_slab_train_stats(slab.data_ptr<float>(), (int)S, C, count, sp, mean.data_ptr<float>(),
                      invstd.data_ptr<float>(), rm, rv, nb, (float)eps, (float)momentum,
                      cur_stream());
  return {mean, invstd};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_slab_reduce_grad_op(
    at::Tensor slab, at::Tensor invstd, OptT weight, bool need_wgrad, OptT sum_scale,
    OptT gw_in, OptT gb_in, bool accumulate) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(slab.is_cuda() && slab.dim() == 3 && slab.size(0) == 2 &&
                  slab.scalar_type() == at::kFloat && slab.is_contiguous(),
              "bn slab reduce: fp32 [2][C][S] slab expected");
  const int64_t S = slab.size(2), C = slab.size(1);
  TORCH_CHECK(invstd.is_cuda() && invstd.scalar_type() == at::kFloat && invstd.numel() == C,
              "bn slab reduce: invstd must be fp32 [C]");
  auto fopt = slab.options();
  // one [2C] buffer (sum_dy | sum_dy_xmu): SyncBN all-reduces it in place
  at::Tensor packed = at::empty({2 * C}, fopt);
  at::Tensor sum_dy = packed.narrow(0, 0, C), sum_dy_xmu = packed.narrow(0, C, C);
  at::Tensor gw, gb;
  DType tw = has(weight) ? dtype_of(*weight) : DType::F32;
  const bool accum = grad_targets(weight, need_wgrad, gw_in, gb_in, gw, gb, accumulate);
  BNAccumScope accum_scope(accum);
  const float* scale = nullptr;
  if (has(sum_scale)) {
    TORCH_CHECK(sum_scale->is_cuda() && sum_scale->scalar_type() == at::kFloat &&
                    sum_scale->numel() == 1,
                "bn slab reduce: sum_scale must be a 1-element fp32 GPU tensor");
    scale = sum_scale->data_ptr<float>();
  }
  bn_slab_reduce_grad(slab.data_ptr<float>(), (int)S, C, invstd.contiguous().data_ptr<float>(),
                      sum_dy.data_ptr<float>(), sum_dy_xmu.data_ptr<float>(),
                      gw.defined() ? gw.data_ptr() : nullptr, gb.defined() ? gb.data_ptr() : nullptr,
                      tw, cur_stream(), scale);
  return {sum_dy, sum_dy_xmu, gw, gb};
}

at::Tensor bn_slab_packed_stats_op(at::Tensor slab, int64_t count, OptT shift, OptT out) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(slab.is_cuda() && slab.dim() == 3 && slab.size(0) == 2 &&
                  slab.scalar_type() == at::kFloat && slab.is_contiguous(),
              "bn slab stats: fp32 [2][C][S] slab expected");
  const int64_t S = slab.size(2), C = slab.size(1);
  const float* sp = nullptr;
  if (has(shift)) {
    TORCH_CHECK(shift->scalar_type() == at::kFloat && shift->is_contiguous() &&
                    shift->numel() == C,
                "bn slab stats: shift must be contiguous fp32 [C]");
    sp = shift->data_ptr<float>();
  }
  at::Tensor packed = packed_out(out, C, slab.options());
  bn_slab_packed_stats(slab.data_ptr<float>(), (int)S, C, count, sp, packed.data_ptr<float>(),
                       cur_stream());
  return packed;
}

}  // namespace amd
