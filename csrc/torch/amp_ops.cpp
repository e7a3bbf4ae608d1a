// amp_C-equivalent operators: validate, pick the CPU or gfx950 path, launch.
//
// Python signatures are Apex-compatible at the facade level
// (apex_example_amd/amp_C.py); here every scalar that may live on the device
// (loss scale, lr, step counter, first-run flag) is accepted as an optional
// tensor so the optimizer step needs no host synchronisation.
#include "amp_ops.h"

#include <cmath>

#include <c10/hip/HIPGraphsC10Utils.h>

#include "../cpu/cpu_ops.h"
#include "common.h"

namespace amd {

namespace {
int* noop_ptr(at::Tensor& noop) {
  if (!noop.defined()) return nullptr;
  TORCH_CHECK(noop.scalar_type() == at::kInt, "noop_flag must be an int32 tensor");
  return noop.data_ptr<int>();
}
cpu::Scale cscale(double v, const c10::optional<at::Tensor>& t, bool inv) {
  return cpu::Scale{v, t.has_value() && t->defined() ? &*t : nullptr, inv};
}
at::Tensor* optp(c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? &*t : nullptr;
}
TensorLists sub(const TensorLists& l, std::initializer_list<int> idx) {
  TensorLists r;
  for (int i : idx) r.push_back(l[(size_t)i]);
  return r;
}
}  // namespace

void mt_scale_op(at::Tensor noop, const TensorLists& lists, double scale,
                 c10::optional<at::Tensor> scale_t, bool invert) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  bool gpu = mt_validate(lists, 2, 2);
  if (!gpu) return cpu::scale(noop, lists, cscale(scale, scale_t, invert));
  const MTPlan& P = mt_plan(lists);
  mt_scale(P.L, dtype_of(lists[0][0]), dtype_of(lists[1][0]), make_scale(scale, scale_t, invert),
           noop_ptr(noop), cur_stream());
}

// Per-dtype-group launch: the kernels are templated on the element type of each
// slot, so lists whose tensors mix dtypes are split into homogeneous groups.
template <typename F>
static void by_dtype_groups(const TensorLists& lists, F&& f) {
  const size_t n = lists[0].size();
  std::vector<std::pair<std::vector<int>, TensorLists>> groups;
  std::vector<std::vector<at::ScalarType>> keys;
  for (size_t i = 0; i < n; ++i) {
    std::vector<at::ScalarType> k;
    for (auto& l : lists) k.push_back(l[i].scalar_type());
    size_t g = 0;
    for (; g < keys.size(); ++g)
      if (keys[g] == k) break;
    if (g == keys.size()) {
      keys.push_back(k);
      groups.emplace_back(std::vector<int>{}, TensorLists(lists.size()));
    }
    groups[g].first.push_back((int)i);
    for (size_t d = 0; d < lists.size(); ++d) groups[g].second[d].push_back(lists[d][i]);
  }
  for (auto& g : groups) f(g.first, g.second);
}

void mt_scale_any_op(at::Tensor noop, const TensorLists& lists, double scale,
                     c10::optional<at::Tensor> scale_t, bool invert) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    mt_scale_op(noop, g, scale, scale_t, invert);
  });
}

void mt_check_finite_op(at::Tensor noop, const std::vector<at::Tensor>& list) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (list.empty()) return;
  TensorLists lists{list};
  bool gpu = mt_validate(lists, 1, 1);
  if (!gpu) return cpu::check_finite(noop, list);
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    mt_check_finite(P.L, dtype_of(g[0][0]), noop_ptr(noop), cur_stream());
  });
}

void mt_axpby_op(at::Tensor noop, const TensorLists& lists, double a, c10::optional<at::Tensor> a_t,
                 bool a_inv, double b, c10::optional<at::Tensor> b_t, bool b_inv,
                 int64_t arg_to_check) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  bool gpu = mt_validate(lists, 3, 3);
  if (!gpu)
    return cpu::axpby(noop, lists, cscale(a, a_t, a_inv), cscale(b, b_t, b_inv), (int)arg_to_check);
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    mt_axpby(P.L, dtype_of(g[0][0]), dtype_of(g[1][0]), dtype_of(g[2][0]), make_scale(a, a_t, a_inv),
             make_scale(b, b_t, b_inv), (int)arg_to_check, noop_ptr(noop), cur_stream());
  });
}

void mt_zero_op(const std::vector<at::Tensor>& list) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (list.empty()) return;
  TensorLists lists{list};
  bool gpu = mt_validate(lists, 1, 1);
  if (!gpu) return cpu::zero(list);
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    mt_fill_zero(P.L, dtype_of(g[0][0]), cur_stream());
  });
}

void mt_copy_if_op(at::Tensor flag, const TensorLists& lists) {
  c10::NoGradGuard no_grad_;
  if (lists.empty() || lists[0].empty()) return;
  TORCH_CHECK(lists.size() == 2, "copy_if: [src, dst] lists expected");
  for (size_t i = 0; i < lists[0].size(); ++i)
    TORCH_CHECK(lists[0][i].scalar_type() == lists[1][i].scalar_type(),
                "copy_if: src / dst dtypes must match");
  bool gpu = mt_validate(lists, 2, 2);
  if (!gpu) {
    if (flag.item<int>() != 0)
      for (size_t i = 0; i < lists[0].size(); ++i) lists[1][i].copy_(lists[0][i]);
    return;
  }
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.is_cuda(), "copy_if: int32 GPU flag");
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    mt_copy_if(P.L, dtype_of(g[0][0]), flag.data_ptr<int>(), cur_stream());
  });
}

std::tuple<at::Tensor, at::Tensor> mt_norm_op(at::Tensor noop, const std::vector<at::Tensor>& list,
                                              bool per_tensor, bool max_norm) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  TORCH_CHECK(!list.empty(), "multi_tensor norm of an empty list");
  TensorLists lists{list};
  bool gpu = mt_validate(lists, 1, 1);
  auto fopt = at::TensorOptions().dtype(at::kFloat).device(list[0].device());
  at::Tensor out = at::zeros({1}, fopt);
  at::Tensor pt = per_tensor ? at::zeros({(int64_t)list.size()}, fopt) : at::empty({0}, fopt);
  if (!gpu) {
    cpu::norm(noop, list, max_norm, out, per_tensor ? &pt : nullptr);
    return {out, pt};
  }
  // Mixed dtypes: norms per group, then combined on device.
  std::vector<at::Tensor> group_globals;
  by_dtype_groups(lists, [&](const std::vector<int>& idx, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    at::Tensor partials = at::empty({P.L.nchunks}, fopt);
    at::Tensor gout = at::empty({1}, fopt);
    at::Tensor gpt = per_tensor ? at::empty({P.L.ntensors}, fopt) : at::Tensor();
    mt_norm_partials(P.L, dtype_of(g[0][0]), max_norm ? 1 : 0, partials.data_ptr<float>(),
                     noop_ptr(noop), cur_stream());
    mt_norm_finalize(P.L, partials.data_ptr<float>(), 1, max_norm ? 1 : 0, gout.data_ptr<float>(),
                     per_tensor ? gpt.data_ptr<float>() : nullptr, cur_stream());
    if (per_tensor) {
      auto index = at::tensor(std::vector<int64_t>(idx.begin(), idx.end()),
                              at::TensorOptions().dtype(at::kLong)).to(list[0].device(), true);
      pt.index_copy_(0, index, gpt);
    }
    group_globals.push_back(gout);
  });
  if (group_globals.size() == 1) {
    out = group_globals[0];
  } else {
    at::Tensor all = at::cat(group_globals);
    out = max_norm ? all.max().reshape({1}) : all.pow(2).sum().sqrt().reshape({1});
  }
  return {out, pt};
}

void mt_sgd_op(at::Tensor noop, const TensorLists& lists, double wd, double momentum,
               double dampening, double lr, c10::optional<at::Tensor> lr_t, bool nesterov,
               bool first_run, c10::optional<at::Tensor> first_run_flag, bool wd_after_momentum,
               double scale, c10::optional<at::Tensor> scale_t, bool scale_inv) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  bool gpu = mt_validate(lists, 3, 4);
  if (!gpu) {
    TORCH_CHECK(!lr_t.has_value() || !lr_t->defined(), "device lr only on GPU");
    cpu::Sgd a{(float)wd, (float)momentum, (float)dampening, (float)lr, nesterov, first_run,
               wd_after_momentum, cscale(scale, scale_t, scale_inv), optp(first_run_flag)};
    return cpu::sgd(noop, lists, a);
  }
  SgdArgs a;
  a.wd = (float)wd;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.lr = (float)lr;
  a.nesterov = nesterov;
  a.first_run = first_run;
  a.wd_after_momentum = wd_after_momentum;
  a.scale = make_scale(scale, scale_t, scale_inv);
  a.lr_ptr = opt_fptr(lr_t);
  a.first_run_flag = opt_iptr(first_run_flag);
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    DType copy = g.size() == 4 ? dtype_of(g[3][0]) : dtype_of(g[1][0]);
    mt_sgd(P.L, (int)g.size(), dtype_of(g[0][0]), dtype_of(g[1][0]), dtype_of(g[2][0]), copy, a,
           noop_ptr(noop), cur_stream());
  });
}

void mt_adam_op(at::Tensor noop, const TensorLists& lists, double lr, c10::optional<at::Tensor> lr_t,
                double beta1, double beta2, double eps, int64_t step,
                c10::optional<at::Tensor> step_t, int64_t mode, bool bias_correction, double wd,
                double scale, c10::optional<at::Tensor> scale_t, bool scale_inv) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  bool gpu = mt_validate(lists, 4, 5);
  if (!gpu) {
    cpu::Adam a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (int)step,
                optp(step_t), (int)mode, bias_correction ? 1 : 0, cscale(scale, scale_t, scale_inv)};
    return cpu::adam(noop, lists, a);
  }
  AdamArgs a;
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.wd = (float)wd;
  a.step = (int)step;
  a.step_ptr = opt_iptr(step_t);
  a.mode = (int)mode;
  a.bias_correction = bias_correction ? 1 : 0;
  a.scale = make_scale(scale, scale_t, scale_inv);
  a.lr_ptr = opt_fptr(lr_t);
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    TORCH_CHECK(g[2][0].scalar_type() == g[1][0].scalar_type() &&
                    g[3][0].scalar_type() == g[1][0].scalar_type(),
                "adam: exp_avg / exp_avg_sq must match the parameter dtype");
    const MTPlan& P = mt_plan(g);
    DType copy = g.size() == 5 ? dtype_of(g[4][0]) : dtype_of(g[1][0]);
    mt_adam(P.L, (int)g.size(), dtype_of(g[0][0]), dtype_of(g[1][0]), copy, a, noop_ptr(noop),
            cur_stream());
  });
}

void mt_lamb_op(at::Tensor noop, const TensorLists& lists, double lr, c10::optional<at::Tensor> lr_t,
                double beta1, double beta2, double eps, int64_t step,
                c10::optional<at::Tensor> step_t, bool bias_correction, double wd,
                bool grad_averaging, int64_t mode, c10::optional<at::Tensor> global_grad_norm,
                double max_grad_norm, bool use_nvlamb, double scale,
                c10::optional<at::Tensor> scale_t, bool scale_inv) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  // lists: [g, p, m, v] or [g, p, m, v, p_copy]; the update u is recomputed in
  // stage 2 from (p, m, v) - no fp32 workspace
  bool gpu = mt_validate(lists, 4, 5);
  if (!gpu) {
    cpu::Lamb a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (int)step,
                optp(step_t), (int)mode, bias_correction ? 1 : 0, grad_averaging ? 1 : 0,
                optp(global_grad_norm), (float)max_grad_norm, use_nvlamb,
                cscale(scale, scale_t, scale_inv)};
    return cpu::lamb(noop, lists, a);
  }
  LambArgs a;
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.wd = (float)wd;
  a.step = (int)step;
  a.step_ptr = opt_iptr(step_t);
  a.mode = (int)mode;
  a.bias_correction = bias_correction ? 1 : 0;
  a.grad_averaging = grad_averaging ? 1 : 0;
  a.global_grad_norm = opt_fptr(global_grad_norm);
  a.max_grad_norm = (float)max_grad_norm;
  a.use_nvlamb = use_nvlamb ? 1 : 0;
  a.scale = make_scale(scale, scale_t, scale_inv);
  a.lr_ptr = opt_fptr(lr_t);
  auto fopt = at::TensorOptions().dtype(at::kFloat).device(lists[0][0].device());
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    TORCH_CHECK(g[2][0].scalar_type() == g[1][0].scalar_type() &&
                    g[3][0].scalar_type() == g[1][0].scalar_type(),
                "lamb: exp_avg / exp_avg_sq must match the parameter dtype");
    TensorLists s1 = sub(g, {0, 1, 2, 3});
    const MTPlan& P1 = mt_plan(s1);
    at::Tensor partials = at::empty({2 * (int64_t)P1.L.nchunks}, fopt);
    at::Tensor norms = at::empty({2 * (int64_t)P1.L.ntensors}, fopt);
    mt_lamb_stage1(P1.L, dtype_of(g[0][0]), dtype_of(g[1][0]), a, partials.data_ptr<float>(),
                   noop_ptr(noop), cur_stream());
    mt_norm_finalize(P1.L, partials.data_ptr<float>(), 2, 0, nullptr, norms.data_ptr<float>(),
                     cur_stream());
    TensorLists s2 = g.size() == 5 ? sub(g, {1, 2, 3, 4}) : sub(g, {1, 2, 3});
    const MTPlan& P2 = mt_plan(s2);
    DType copy = g.size() == 5 ? dtype_of(g[4][0]) : dtype_of(g[1][0]);
    mt_lamb_stage2(P2.L, (int)s2.size(), dtype_of(g[1][0]), copy, a, norms.data_ptr<float>(),
                   norms.data_ptr<float>() + P1.L.ntensors, noop_ptr(noop), cur_stream());
  });
}

// Legacy two-stage LAMB (apex amp_C.multi_tensor_lamb_stage1_cuda / stage2_cuda): GPU only,
// the CPU facade composes the same math from tensor ops (amp_C.py)
void mt_lamb_legacy_stage1_op(at::Tensor noop, const TensorLists& lists, at::Tensor decay,
                              int64_t step, double beta1, double beta2, double eps,
                              at::Tensor global_grad_norm, double max_grad_norm) {
  c10::NoGradGuard no_grad_;
  if (lists.empty() || lists[0].empty()) return;
  TORCH_CHECK(lists.size() == 5, "lamb stage 1: lists [g, p, m, v, u]");
  TORCH_CHECK(mt_validate(lists, 5, 5), "lamb stage 1: GPU tensors only");
  const int64_t n = (int64_t)lists[0].size();
  TORCH_CHECK(decay.is_cuda() && decay.scalar_type() == at::kFloat && decay.numel() == n &&
                  decay.is_contiguous(),
              "lamb stage 1: per_tensor_decay must be a contiguous fp32 GPU tensor [ntensors]");
  TORCH_CHECK(global_grad_norm.is_cuda() && global_grad_norm.scalar_type() == at::kFloat &&
                  global_grad_norm.numel() >= 1,
              "lamb stage 1: global_grad_norm must be an fp32 GPU scalar");
  TORCH_CHECK(step >= 1, "lamb stage 1: step >= 1");
  LambLegacyArgs a{};
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.bc1 = (float)(1.0 - std::pow(beta1, (double)step));
  a.bc2 = (float)(1.0 - std::pow(beta2, (double)step));
  a.global_grad_norm = global_grad_norm.data_ptr<float>();
  a.max_grad_norm = (float)max_grad_norm;
  a.decay = decay.data_ptr<float>();
  for (int d = 2; d < 5; ++d)
    TORCH_CHECK(lists[d][0].scalar_type() == lists[1][0].scalar_type(),
                "lamb stage 1: m / v / u must match the parameter dtype");
  const MTPlan P = mt_plan(lists);
  mt_lamb_legacy_stage1(P.L, dtype_of(lists[0][0]), dtype_of(lists[1][0]), a, noop_ptr(noop),
                        cur_stream());
}

void mt_lamb_legacy_stage2_op(at::Tensor noop, const TensorLists& lists, at::Tensor param_norms,
                              at::Tensor update_norms, double lr, double weight_decay,
                              bool use_nvlamb) {
  c10::NoGradGuard no_grad_;
  if (lists.empty() || lists[0].empty()) return;
  TORCH_CHECK(lists.size() == 2, "lamb stage 2: lists [p, u]");
  TORCH_CHECK(mt_validate(lists, 2, 2), "lamb stage 2: GPU tensors only");
  const int64_t n = (int64_t)lists[0].size();
  for (const at::Tensor* t : {&param_norms, &update_norms})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == n &&
                    t->is_contiguous(),
                "lamb stage 2: per-tensor norms must be contiguous fp32 GPU tensors [ntensors]");
  LambLegacyArgs a{};
  a.lr = (float)lr;
  a.wd = (float)weight_decay;
  a.use_nvlamb = use_nvlamb ? 1 : 0;
  a.param_norms = param_norms.data_ptr<float>();
  a.update_norms = update_norms.data_ptr<float>();
  const MTPlan P = mt_plan(lists);
  mt_lamb_legacy_stage2(P.L, dtype_of(lists[0][0]), dtype_of(lists[1][0]), a, noop_ptr(noop),
                        cur_stream());
}

void mt_novograd_op(at::Tensor noop, const TensorLists& lists, at::Tensor v, at::Tensor grad_norms,
                    bool first_step, double lr, c10::optional<at::Tensor> lr_t, double beta1,
                    double beta2, double eps, int64_t step, c10::optional<at::Tensor> step_t,
                    bool bias_correction, double wd, bool grad_averaging, int64_t mode,
                    int64_t norm_type, double scale, c10::optional<at::Tensor> scale_t,
                    bool scale_inv) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  bool gpu = mt_validate(lists, 3, 3);
  if (!gpu) {
    cpu::Novo a{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (int)step,
                optp(step_t), (int)mode, bias_correction ? 1 : 0, grad_averaging ? 1 : 0,
                (int)norm_type, cscale(scale, scale_t, scale_inv)};
    return cpu::novograd(noop, lists, v, grad_norms, first_step, a);
  }
  TORCH_CHECK(v.is_cuda() && v.scalar_type() == at::kFloat && v.numel() == (int64_t)lists[0].size(),
              "novograd: v must be a float32 device tensor with one entry per parameter");
  NovoArgs a;
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.wd = (float)wd;
  a.step = (int)step;
  a.step_ptr = opt_iptr(step_t);
  a.mode = (int)mode;
  a.bias_correction = bias_correction ? 1 : 0;
  a.grad_averaging = grad_averaging ? 1 : 0;
  a.norm_type = (int)norm_type;
  a.init_zero = 0.f;
  a.scale = make_scale(scale, scale_t, scale_inv);
  a.lr_ptr = opt_fptr(lr_t);
  // grad_norms are unscaled norms of the (scaled) grads -> fold scale in on host side by caller.
  novograd_blend(v.data_ptr<float>(), grad_norms.data_ptr<float>(), (int)v.numel(), a.beta2,
                 a.norm_type, first_step ? 1 : 0, noop_ptr(noop), cur_stream());
  // A single dtype group is required here because v is indexed by tensor position.
  const MTPlan& P = mt_plan(lists);
  for (size_t i = 1; i < lists[0].size(); ++i) {
    TORCH_CHECK(lists[0][i].scalar_type() == lists[0][0].scalar_type() &&
                    lists[1][i].scalar_type() == lists[1][0].scalar_type(),
                "novograd: one dtype per launch");
  }
  mt_novograd(P.L, dtype_of(lists[0][0]), dtype_of(lists[1][0]), a, v.data_ptr<float>(),
              noop_ptr(noop), cur_stream());
}

void mt_adagrad_op(at::Tensor noop, const TensorLists& lists, double lr,
                   c10::optional<at::Tensor> lr_t, double eps, int64_t mode, double wd,
                   double scale, c10::optional<at::Tensor> scale_t, bool scale_inv) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  if (lists.empty() || lists[0].empty()) return;
  bool gpu = mt_validate(lists, 3, 3);
  if (!gpu) {
    cpu::Adagrad a{(float)lr, (float)eps, (float)wd, (int)mode, cscale(scale, scale_t, scale_inv)};
    return cpu::adagrad(noop, lists, a);
  }
  AdagradArgs a;
  a.lr = (float)lr;
  a.eps = (float)eps;
  a.wd = (float)wd;
  a.mode = (int)mode;
  a.scale = make_scale(scale, scale_t, scale_inv);
  a.lr_ptr = opt_fptr(lr_t);
  by_dtype_groups(lists, [&](const std::vector<int>&, const TensorLists& g) {
    const MTPlan& P = mt_plan(g);
    mt_adagrad(P.L, dtype_of(g[0][0]), dtype_of(g[1][0]), a, noop_ptr(noop), cur_stream());
  });
}

void update_loss_scale_op(at::Tensor scale, at::Tensor unskipped, c10::optional<at::Tensor> skipped,
                          at::Tensor overflow, double factor, int64_t window, double min_scale,
                          double max_scale, bool dynamic, c10::optional<at::Tensor> applied) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  TORCH_CHECK(scale.scalar_type() == at::kFloat && unskipped.scalar_type() == at::kInt &&
                  overflow.scalar_type() == at::kInt,
              "update_loss_scale: bad dtypes");
  if (!scale.is_cuda()) {
    if (applied.has_value() && applied->defined()) applied->copy_(scale);
    return cpu::update_loss_scale(scale, unskipped, optp(skipped), overflow, (float)factor,
                                  (int)window, (float)min_scale, (float)max_scale, dynamic);
  }
  update_loss_scale(scale.data_ptr<float>(), unskipped.data_ptr<int>(), opt_iptr(skipped),
                    overflow.data_ptr<int>(), (float)factor, (int)window, (float)min_scale,
                    (float)max_scale, dynamic ? 1 : 0, cur_stream(), opt_fptr(applied));
}

// ------------------------------------------------------------------ StepPlan
StepPlan::StepPlan(std::vector<at::Tensor> owners, TensorLists fixed) : owners_(std::move(owners)) {
  TORCH_CHECK(!owners_.empty() && !fixed.empty(), "StepPlan: empty launch set");
  lists_.reserve(fixed.size() + 1);
  lists_.emplace_back(owners_.size());
  for (auto& l : fixed) {
    TORCH_CHECK(l.size() == owners_.size(), "StepPlan: list sizes differ");
    lists_.push_back(std::move(l));
  }
  gptr_.assign(owners_.size(), nullptr);
  gtype_ = at::ScalarType::Undefined;
  gpu_ = lists_[1][0].is_cuda();
}

bool StepPlan::refresh() {
  for (const auto& t : absent_)
    if (t.grad().defined()) return false;
  bool moved = false;
  for (size_t i = 0; i < owners_.size(); ++i) {
    const at::Tensor& g = owners_[i].grad();
    if (!g.defined()) return false;
    void* p = g.data_ptr();
    if (p == gptr_[i] && g.unsafeGetTensorImpl() == lists_[0][i].unsafeGetTensorImpl()) continue;
    if (gtype_ == at::ScalarType::Undefined) gtype_ = g.scalar_type();
    if (g.scalar_type() != gtype_ || g.numel() != lists_[1][i].numel() || g.is_sparse() ||
        !g.is_non_overlapping_and_dense())
      return false;
    lists_[0][i] = g;
    gptr_[i] = p;
    moved = true;
  }
  if (moved) {
    mt_validate(lists_, 2, kMaxDepth);  // strides of a new grad vs. its param
    fresh_ = false;
    ++gen_;
  }
  return true;
}

namespace {
// a sub-table built inside a graph capture must never be evicted / rebuilt under it
void mark_if_capturing(MTPlan& p) {
  if (c10::hip::currentStreamCaptureStatusMayInitCtx() != c10::hip::CaptureStatus::None)
    p.captured = true;
}
}  // namespace

bool StepPlan::grad_norm_into(at::Tensor out, int64_t slot, at::Tensor flag, double scale,
                              OptT scale_t) {
  c10::NoGradGuard no_grad_;
  if (!refresh()) return false;
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && slot >= 0 &&
                  slot < out.numel(), "grad_norm_into: fp32 output slot");
  at::Tensor dst = out.narrow(0, slot, 1);
  if (!gpu_) {
    dst.copy_(std::get<0>(mt_norm_op(flag, lists_[0], false, false)));
  } else {
    auto fopt = at::TensorOptions().dtype(at::kFloat).device(out.device());
    if (ngen_ != gen_) {
      nplan_ = mt_plan(TensorLists{lists_[0]});
      npart_ = at::empty({(int64_t)nplan_.L.nchunks}, fopt);
      ngen_ = gen_;
    }
    mark_if_capturing(nplan_);
    mt_norm_partials(nplan_.L, dtype_of(lists_[0][0]), 0, npart_.data_ptr<float>(),
                     noop_ptr(flag), cur_stream());
    mt_norm_finalize(nplan_.L, npart_.data_ptr<float>(), 1, 0, dst.data_ptr<float>(), nullptr,
                     cur_stream());
  }
  if (scale_t.has_value() && scale_t->defined()) dst.div_(*scale_t);
  else if (scale != 1.0) dst.mul_(scale);
  return true;
}

bool StepPlan::lamb(at::Tensor noop, double lr, OptT lr_t, double beta1, double beta2, double eps,
                    int64_t step, OptT step_t, bool bias_correction, double wd,
                    bool grad_averaging, int64_t mode, at::Tensor global_grad_norm,
                    double max_grad_norm, bool use_nvlamb, double scale, OptT scale_t,
                    bool scale_inv, bool advance) {
  c10::NoGradGuard no_grad_;
  if (!refresh()) return false;
  const int depth = (int)lists_.size();
  TORCH_CHECK(depth == 4 || depth == 5, "lamb plan: [grads, params, m, v(, copies)]");
  if (!gpu_) {
    mt_lamb_op(noop, lists_, lr, lr_t, beta1, beta2, eps, step, step_t, bias_correction, wd,
               grad_averaging, mode, OptT(global_grad_norm), max_grad_norm, use_nvlamb, scale,
               scale_t, scale_inv);
  } else {
    TORCH_CHECK(lists_[2][0].scalar_type() == lists_[1][0].scalar_type() &&
                    lists_[3][0].scalar_type() == lists_[1][0].scalar_type(),
                "lamb: exp_avg / exp_avg_sq must match the parameter dtype");
    LambArgs a;
    a.lr = (float)lr;
    a.beta1 = (float)beta1;
    a.beta2 = (float)beta2;
    a.eps = (float)eps;
    a.wd = (float)wd;
    a.step = (int)step;
    a.step_ptr = opt_iptr(step_t);
    a.mode = (int)mode;
    a.bias_correction = bias_correction ? 1 : 0;
    a.grad_averaging = grad_averaging ? 1 : 0;
    a.global_grad_norm = global_grad_norm.data_ptr<float>();
    a.max_grad_norm = (float)max_grad_norm;
    a.use_nvlamb = use_nvlamb ? 1 : 0;
    a.scale = make_scale(scale, scale_t, scale_inv);
    a.lr_ptr = opt_fptr(lr_t);
    auto fopt = at::TensorOptions().dtype(at::kFloat).device(lists_[1][0].device());
    if (l1gen_ != gen_) {
      l1plan_ = mt_plan(sub(lists_, {0, 1, 2, 3}));
      l1part_ = at::empty({2 * (int64_t)l1plan_.L.nchunks}, fopt);
      l1norm_ = at::empty({2 * (int64_t)l1plan_.L.ntensors}, fopt);
      l1gen_ = gen_;
    }
    if (!l2ok_) {  // params / state / copies never move: built once
      l2plan_ = mt_plan(depth == 5 ? sub(lists_, {1, 2, 3, 4}) : sub(lists_, {1, 2, 3}));
      l2ok_ = true;
    }
    mark_if_capturing(l1plan_);
    mark_if_capturing(l2plan_);
    mt_lamb_stage1(l1plan_.L, dtype_of(lists_[0][0]), dtype_of(lists_[1][0]), a,
                   l1part_.data_ptr<float>(), noop_ptr(noop), cur_stream());
    mt_norm_finalize(l1plan_.L, l1part_.data_ptr<float>(), 2, 0, nullptr,
                     l1norm_.data_ptr<float>(), cur_stream());
    DType copy = depth == 5 ? dtype_of(lists_[4][0]) : dtype_of(lists_[1][0]);
    mt_lamb_stage2(l2plan_.L, depth - 1, dtype_of(lists_[1][0]), copy, a,
                   l1norm_.data_ptr<float>(), l1norm_.data_ptr<float>() + l1plan_.L.ntensors,
                   noop_ptr(noop), cur_stream());
  }
  if (advance && step_t.has_value() && step_t->defined())
    advance_step_op(*step_t, noop.defined() ? OptT(noop) : OptT());
  return true;
}

// the launch table: built (or fetched from the address cache) once per grad layout
bool StepPlan::gpu_launch_ready() {
  if (!gpu_) return false;
  if (!fresh_) {
    plan_ = mt_plan(lists_);
    fresh_ = true;
    ++rebuilds_;
  } else if (c10::hip::currentStreamCaptureStatusMayInitCtx() != c10::hip::CaptureStatus::None) {
    plan_.captured = true;  // (the plan owns its table: it outlives the graph)
  }
  return true;
}

bool StepPlan::sgd(at::Tensor noop, double wd, double momentum, double dampening, double lr,
                   bool nesterov, bool first_run, OptT first_run_flag, bool wd_after_momentum,
                   double scale, OptT scale_t, bool scale_inv) {
  c10::NoGradGuard no_grad_;
  if (!refresh()) return false;
  const int depth = (int)lists_.size();
  TORCH_CHECK(depth == 3 || depth == 4, "sgd plan: [grads, params, moms(, copies)]");
  if (!gpu_launch_ready()) {
    mt_sgd_op(noop, lists_, wd, momentum, dampening, lr, c10::nullopt, nesterov, first_run,
              first_run_flag, wd_after_momentum, scale, scale_t, scale_inv);
    return true;
  }
  SgdArgs a;
  a.wd = (float)wd;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.lr = (float)lr;
  a.nesterov = nesterov;
  a.first_run = first_run;
  a.wd_after_momentum = wd_after_momentum;
  a.scale = make_scale(scale, scale_t, scale_inv);
  a.lr_ptr = nullptr;
  a.first_run_flag = opt_iptr(first_run_flag);
  DType copy = depth == 4 ? dtype_of(lists_[3][0]) : dtype_of(lists_[1][0]);
  mt_sgd(plan_.L, depth, dtype_of(lists_[0][0]), dtype_of(lists_[1][0]), dtype_of(lists_[2][0]),
         copy, a, noop_ptr(noop), cur_stream());
  return true;
}

bool StepPlan::sgd_pair(StepPlan& o, at::Tensor noop, double wd, double momentum,
                        double dampening, double lr, bool nesterov, bool wd_after_momentum,
                        double scale, OptT scale_t, bool scale_inv, double other_scale,
                        OptT other_scale_t, bool other_scale_inv) {
  c10::NoGradGuard no_grad_;
  if (lists_.size() != 4 || o.lists_.size() != 3) return false;
  if (!refresh() || !o.refresh()) return false;
  if (!gpu_launch_ready() || !o.gpu_launch_ready()) return false;
  auto args = [&](double sv, const OptT& st, bool inv) {
    SgdArgs a;
    a.wd = (float)wd;
    a.momentum = (float)momentum;
    a.dampening = (float)dampening;
    a.lr = (float)lr;
    a.nesterov = nesterov;
    a.first_run = false;
    a.wd_after_momentum = wd_after_momentum;
    a.scale = make_scale(sv, st, inv);
    a.lr_ptr = nullptr;
    a.first_run_flag = nullptr;
    return a;
  };
  return mt_sgd_pair(plan_.L, dtype_of(lists_[0][0]), dtype_of(lists_[1][0]),
                     dtype_of(lists_[3][0]), args(scale, scale_t, scale_inv), o.plan_.L,
                     dtype_of(o.lists_[0][0]), dtype_of(o.lists_[1][0]),
                     args(other_scale, other_scale_t, other_scale_inv), noop_ptr(noop),
                     cur_stream());
}

bool StepPlan::adam(at::Tensor noop, double lr, OptT lr_t, double beta1, double beta2, double eps,
                    int64_t step, OptT step_t, int64_t mode, bool bias_correction, double wd,
                    double scale, OptT scale_t, bool scale_inv, bool advance) {
  c10::NoGradGuard no_grad_;
  if (!refresh()) return false;
  const int depth = (int)lists_.size();
  TORCH_CHECK(depth == 4 || depth == 5, "adam plan: [grads, params, m, v(, copies)]");
  if (!gpu_launch_ready()) {
    mt_adam_op(noop, lists_, lr, lr_t, beta1, beta2, eps, step, step_t, mode, bias_correction, wd,
               scale, scale_t, scale_inv);
  } else {
    AdamArgs a;
    a.lr = (float)lr;
    a.beta1 = (float)beta1;
    a.beta2 = (float)beta2;
    a.eps = (float)eps;
    a.wd = (float)wd;
    a.step = (int)step;
    a.step_ptr = opt_iptr(step_t);
    a.mode = (int)mode;
    a.bias_correction = bias_correction ? 1 : 0;
    a.scale = make_scale(scale, scale_t, scale_inv);
    a.lr_ptr = opt_fptr(lr_t);
    DType copy = depth == 5 ? dtype_of(lists_[4][0]) : dtype_of(lists_[1][0]);
    mt_adam(plan_.L, depth, dtype_of(lists_[0][0]), dtype_of(lists_[1][0]), copy, a,
            noop_ptr(noop), cur_stream());
  }
  if (advance && step_t.has_value() && step_t->defined())
    advance_step_op(*step_t, noop.defined() ? OptT(noop) : OptT());
  return true;
}

void advance_step_op(at::Tensor step, c10::optional<at::Tensor> noop) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  TORCH_CHECK(step.scalar_type() == at::kInt, "step counter must be int32");
  if (!step.is_cuda()) {
    bool skip = noop.has_value() && noop->defined() && noop->item<int>() != 0;
    if (!skip) step.add_(1);
    return;
  }
  advance_step(step.data_ptr<int>(), opt_iptr(noop), cur_stream());
}

void mark_step_done_op(at::Tensor flag, c10::optional<at::Tensor> noop) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  TORCH_CHECK(flag.scalar_type() == at::kInt, "flag must be int32");
  if (!flag.is_cuda()) {
    bool skip = noop.has_value() && noop->defined() && noop->item<int>() != 0;
    if (!skip) flag.fill_(1);
    return;
  }
  mark_step_done(flag.data_ptr<int>(), opt_iptr(noop), cur_stream());
}

void flat_scale_op(at::Tensor in, at::Tensor out, double scale, c10::optional<at::Tensor> scale_t,
                   bool invert, c10::optional<at::Tensor> noop) {
  c10::NoGradGuard no_grad_;  // optimizer / scaler state is never differentiated
  TORCH_CHECK(in.is_contiguous() && (!out.defined() || out.is_contiguous()), "contiguous only");
  if (!in.is_cuda()) {
    float s = (float)scale;
    if (scale_t.has_value() && scale_t->defined()) s = scale_t->item<float>();
    if (invert) s = 1.f / s;
    if (noop.has_value() && noop->defined() && !at::isfinite(in).all().item<bool>()) noop->fill_(1);
    if (out.defined()) out.copy_(in.to(at::kFloat) * s);
    return;
  }
  flat_scale(in.data_ptr(), dtype_of(in), out.defined() ? out.data_ptr() : nullptr,
             out.defined() ? dtype_of(out) : dtype_of(in), in.numel(),
             make_scale(scale, scale_t, invert), opt_iptr(noop), cur_stream());
}

}  // namespace amd
