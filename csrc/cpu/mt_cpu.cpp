// CPU reference implementations (see cpu_ops.h).
#include "cpu_ops.h"

#include <ATen/Parallel.h>

#include <cmath>

namespace amd {
namespace cpu {

namespace {

// fp32 working copy of a tensor (no copy for fp32 inputs).
at::Tensor f32(const at::Tensor& t) {
  return t.scalar_type() == at::kFloat ? t : t.to(at::kFloat);
}
// write an fp32 result back into `dst` (no-op when dst already is that tensor).
void put(at::Tensor& dst, const at::Tensor& src) {
  if (!dst.is_same(src)) dst.copy_(src);
}
inline bool fin(float x) { return std::isfinite(x); }

template <typename F>
void pfor(int64_t n, F&& f) {
  at::parallel_for(0, n, 16384, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) f(i);
  });
}

void set_noop(at::Tensor& noop) { noop.fill_(1); }

}  // namespace

bool noop_set(const at::Tensor& noop) { return noop.defined() && noop.item<int>() != 0; }

void scale(at::Tensor& noop, const TensorLists& l, Scale s) {
  const float sc = s.get();
  bool ok = true;
  for (size_t i = 0; i < l[0].size(); ++i) {
    at::Tensor x = f32(l[0][i]).contiguous();
    const float* px = x.data_ptr<float>();
    at::Tensor y = at::empty_like(x);
    float* py = y.data_ptr<float>();
    int64_t n = x.numel();
    for (int64_t k = 0; k < n; ++k) {
      ok &= fin(px[k]);
      py[k] = px[k] * sc;
    }
    at::Tensor out = l[1][i];
    out.copy_(y);
  }
  if (!ok) set_noop(noop);
}

void check_finite(at::Tensor& noop, const std::vector<at::Tensor>& l) {
  for (const auto& t : l) {
    if (!at::isfinite(t).all().item<bool>()) {
      set_noop(noop);
      return;
    }
  }
}

void axpby(at::Tensor& noop, const TensorLists& l, Scale sa, Scale sb, int arg_to_check) {
  const float a = sa.get(), b = sb.get();
  bool ok = true;
  for (size_t i = 0; i < l[0].size(); ++i) {
    at::Tensor x = f32(l[0][i]).contiguous(), y = f32(l[1][i]).contiguous();
    const float* px = x.data_ptr<float>();
    const float* py = y.data_ptr<float>();
    at::Tensor o = at::empty_like(x);
    float* po = o.data_ptr<float>();
    for (int64_t k = 0; k < x.numel(); ++k) {
      if (arg_to_check == -1) ok &= fin(px[k]) && fin(py[k]);
      else if (arg_to_check == 0) ok &= fin(px[k]);
      else ok &= fin(py[k]);
      po[k] = a * px[k] + b * py[k];
    }
    at::Tensor out = l[2][i];
    out.copy_(o);
  }
  if (!ok) set_noop(noop);
}

void zero(const std::vector<at::Tensor>& l) {
  for (auto t : l) t.zero_();
}

void norm(at::Tensor& noop, const std::vector<at::Tensor>& l, bool max_norm, at::Tensor& out,
          at::Tensor* per_tensor) {
  double total = 0.0;
  bool ok = true;
  for (size_t i = 0; i < l.size(); ++i) {
    at::Tensor x = f32(l[i]).contiguous();
    const float* p = x.data_ptr<float>();
    double acc = 0.0;
    for (int64_t k = 0; k < x.numel(); ++k) {
      ok &= fin(p[k]);
      if (max_norm) acc = std::max(acc, (double)std::fabs(p[k]));
      else acc += (double)p[k] * (double)p[k];
    }
    if (per_tensor) per_tensor->data_ptr<float>()[i] = (float)(max_norm ? acc : std::sqrt(acc));
    total = max_norm ? std::max(total, acc) : total + acc;
  }
  out.data_ptr<float>()[0] = (float)(max_norm ? total : std::sqrt(total));
  if (!ok && noop.defined()) set_noop(noop);
}

static float bias_corr(int on, float beta, int step) {
  return on ? 1.f - std::pow(beta, (float)step) : 1.f;
}

void sgd(at::Tensor& noop, const TensorLists& l, const Sgd& a) {
  if (noop_set(noop)) return;
  const float sc = a.scale.get();
  const bool first =
      a.first_run_flag && a.first_run_flag->defined() ? (a.first_run_flag->item<int>() == 0) : a.first_run;
  const bool has_mom = a.momentum != 0.f;
  for (size_t i = 0; i < l[0].size(); ++i) {
    at::Tensor g = f32(l[0][i]).contiguous();
    at::Tensor p = f32(l[1][i]).contiguous();
    at::Tensor m = f32(l[2][i]).contiguous();
    const float* pg = g.data_ptr<float>();
    float* pp = p.data_ptr<float>();
    float* pm = m.data_ptr<float>();
    pfor(g.numel(), [&](int64_t k) {
      float gi = pg[k] * sc;
      if (a.wd != 0.f && !a.wd_after_momentum) gi += a.wd * pp[k];
      if (has_mom) {
        pm[k] = first ? gi : pm[k] * a.momentum + (1.f - a.dampening) * gi;
        gi = a.nesterov ? gi + a.momentum * pm[k] : pm[k];
      }
      if (a.wd != 0.f && a.wd_after_momentum) gi += a.wd * pp[k];
      pp[k] -= a.lr * gi;
    });
    at::Tensor dst_p = l[1][i];
    put(dst_p, p);
    if (has_mom) {
      at::Tensor dst_m = l[2][i];
      put(dst_m, m);
    }
    if (l.size() == 4) {
      at::Tensor c = l[3][i];
      c.copy_(p);
    }
  }
}

void adam(at::Tensor& noop, const TensorLists& l, const Adam& a) {
  if (noop_set(noop)) return;
  const float sc = a.scale.get();
  const int step = a.step_t && a.step_t->defined() ? a.step_t->item<int>() + 1 : a.step;
  const float bc1 = bias_corr(a.bias_correction, a.b1, step);
  const float bc2 = bias_corr(a.bias_correction, a.b2, step);
  for (size_t i = 0; i < l[0].size(); ++i) {
    at::Tensor g = f32(l[0][i]).contiguous();
    at::Tensor p = f32(l[1][i]).contiguous();
    at::Tensor m = f32(l[2][i]).contiguous();
    at::Tensor v = f32(l[3][i]).contiguous();
    const float* pg = g.data_ptr<float>();
    float* pp = p.data_ptr<float>();
    float* pm = m.data_ptr<float>();
    float* pv = v.data_ptr<float>();
    pfor(g.numel(), [&](int64_t k) {
      float gi = pg[k] * sc;
      if (a.mode == 0) gi += a.wd * pp[k];
      pm[k] = a.b1 * pm[k] + (1.f - a.b1) * gi;
      pv[k] = a.b2 * pv[k] + (1.f - a.b2) * gi * gi;
      float denom = std::sqrt(pv[k] / bc2) + a.eps;
      float upd = (pm[k] / bc1) / denom;
      if (a.mode == 1) upd += a.wd * pp[k];
      pp[k] -= a.lr * upd;
    });
    at::Tensor d1 = l[1][i], d2 = l[2][i], d3 = l[3][i];
    put(d1, p);
    put(d2, m);
    put(d3, v);
    if (l.size() == 5) {
      at::Tensor c = l[4][i];
      c.copy_(p);
    }
  }
}

void lamb(at::Tensor& noop, const TensorLists& l, const Lamb& a) {
  if (noop_set(noop)) return;
  const float sc = a.scale.get();
  const int step = a.step_t && a.step_t->defined() ? a.step_t->item<int>() + 1 : a.step;
  const float bc1 = bias_corr(a.bias_correction, a.b1, step);
  const float bc2 = bias_corr(a.bias_correction, a.b2, step);
  const float beta3 = a.grad_averaging ? 1.f - a.b1 : 1.f;
  const float gn = a.global_norm && a.global_norm->defined() ? a.global_norm->item<float>() : 0.f;
  const float clip = (a.max_grad_norm > 0.f && gn > a.max_grad_norm) ? gn / a.max_grad_norm : 1.f;
  for (size_t i = 0; i < l[0].size(); ++i) {
    at::Tensor g = f32(l[0][i]).contiguous();
    at::Tensor p = f32(l[1][i]).contiguous();
    at::Tensor m = f32(l[2][i]).contiguous();
    at::Tensor v = f32(l[3][i]).contiguous();
    at::Tensor u = at::empty_like(p);
    const float* pg = g.data_ptr<float>();
    float* pp = p.data_ptr<float>();
    float* pm = m.data_ptr<float>();
    float* pv = v.data_ptr<float>();
    float* pu = u.data_ptr<float>();
    double pn = 0, un = 0;
    for (int64_t k = 0; k < g.numel(); ++k) {
      float gi = pg[k] * sc / clip;
      if (a.mode == 0) gi += a.wd * pp[k];
      pm[k] = a.b1 * pm[k] + beta3 * gi;
      pv[k] = a.b2 * pv[k] + (1.f - a.b2) * gi * gi;
      float uu = (pm[k] / bc1) / (std::sqrt(pv[k] / bc2) + a.eps);
      if (a.mode == 1) uu += a.wd * pp[k];
      pu[k] = uu;
      pn += (double)pp[k] * pp[k];
      un += (double)uu * uu;
    }
    float pnorm = (float)std::sqrt(pn), unorm = (float)std::sqrt(un);
    float ratio = a.lr;
    if (a.use_nvlamb || a.wd != 0.f)
      ratio = (pnorm != 0.f && unorm != 0.f) ? a.lr * (pnorm / unorm) : a.lr;
    for (int64_t k = 0; k < g.numel(); ++k) pp[k] -= ratio * pu[k];
    at::Tensor d1 = l[1][i], d2 = l[2][i], d3 = l[3][i];
    put(d1, p);
    put(d2, m);
    put(d3, v);
    if (l.size() == 5) {
      at::Tensor c = l[4][i];
      c.copy_(p);
    }
  }
}

void novograd(at::Tensor& noop, const TensorLists& l, at::Tensor& vt, const at::Tensor& grad_norms,
              bool first_step, const Novo& a) {
  if (noop_set(noop)) return;
  const float sc = a.scale.get();
  const int step = a.step_t && a.step_t->defined() ? a.step_t->item<int>() + 1 : a.step;
  const float bc1 = bias_corr(a.bias_correction, a.b1, step);
  const float bc2 = bias_corr(a.bias_correction, a.b2, step);
  const float beta3 = a.grad_averaging ? 1.f - a.b1 : 1.f;
  float* v = vt.data_ptr<float>();
  const float* gnorm = grad_norms.data_ptr<float>();
  for (size_t i = 0; i < l[0].size(); ++i) {
    float gnv = gnorm[i];
    if (first_step) v[i] = gnv;
    else if (a.norm_type == 2) v[i] = std::sqrt(a.b2 * v[i] * v[i] + (1.f - a.b2) * gnv * gnv);
    else v[i] = a.b2 * v[i] + (1.f - a.b2) * gnv;
    const float inv_denom = 1.f / (v[i] / std::sqrt(bc2) + a.eps);
    at::Tensor g = f32(l[0][i]).contiguous();
    at::Tensor p = f32(l[1][i]).contiguous();
    at::Tensor m = f32(l[2][i]).contiguous();
    const float* pg = g.data_ptr<float>();
    float* pp = p.data_ptr<float>();
    float* pm = m.data_ptr<float>();
    pfor(g.numel(), [&](int64_t k) {
      float gi = pg[k] * sc * inv_denom;
      if (a.mode == 0) gi += a.wd * pp[k];
      pm[k] = a.b1 * pm[k] + beta3 * gi;
      float upd = pm[k] / bc1;
      if (a.mode == 1) upd += a.wd * pp[k];
      pp[k] -= a.lr * upd;
    });
    at::Tensor d1 = l[1][i], d2 = l[2][i];
    put(d1, p);
    put(d2, m);
  }
}

void adagrad(at::Tensor& noop, const TensorLists& l, const Adagrad& a) {
  if (noop_set(noop)) return;
  const float sc = a.scale.get();
  for (size_t i = 0; i < l[0].size(); ++i) {
    at::Tensor g = f32(l[0][i]).contiguous();
    at::Tensor p = f32(l[1][i]).contiguous();
    at::Tensor h = f32(l[2][i]).contiguous();
    const float* pg = g.data_ptr<float>();
    float* pp = p.data_ptr<float>();
    float* ph = h.data_ptr<float>();
    pfor(g.numel(), [&](int64_t k) {
      float gi = pg[k] * sc;
      if (a.mode == 0) gi += a.wd * pp[k];
      ph[k] += gi * gi;
      float upd = gi / (std::sqrt(ph[k]) + a.eps);
      if (a.mode == 1) upd += a.wd * pp[k];
      pp[k] -= a.lr * upd;
    });
    at::Tensor d1 = l[1][i], d2 = l[2][i];
    put(d1, p);
    put(d2, h);
  }
}

void update_loss_scale(at::Tensor& scale, at::Tensor& unskipped, at::Tensor* skipped,
                       const at::Tensor& overflow, float factor, int window, float min_scale,
                       float max_scale, bool dynamic) {
  float* s = scale.data_ptr<float>();
  int* u = unskipped.data_ptr<int>();
  if (overflow.item<int>() != 0) {
    if (dynamic) {
      float ns = *s / factor;
      if (min_scale > 0.f && ns < min_scale) ns = min_scale;
      *s = ns;
    }
    *u = 0;
    if (skipped && skipped->defined()) skipped->data_ptr<int>()[0] += 1;
  } else {
    int nu = *u + 1;
    if (dynamic && nu == window) {
      float ns = *s * factor;
      if (ns > max_scale) ns = max_scale;
      *s = ns;
      nu = 0;
    }
    *u = nu;
  }
}

}  // namespace cpu
}  // namespace amd
