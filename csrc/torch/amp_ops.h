#pragma once
#include <ATen/ATen.h>
#include <c10/util/Optional.h>

#include <tuple>
#include <vector>

#include "common.h"

namespace amd {

using TensorLists = std::vector<std::vector<at::Tensor>>;
using OptT = c10::optional<at::Tensor>;

void mt_scale_op(at::Tensor noop, const TensorLists& lists, double scale, OptT scale_t, bool invert);
void mt_scale_any_op(at::Tensor noop, const TensorLists& lists, double scale, OptT scale_t,
                     bool invert);
void mt_check_finite_op(at::Tensor noop, const std::vector<at::Tensor>& list);
void mt_axpby_op(at::Tensor noop, const TensorLists& lists, double a, OptT a_t, bool a_inv,
                 double b, OptT b_t, bool b_inv, int64_t arg_to_check);
void mt_zero_op(const std::vector<at::Tensor>& list);
void mt_copy_if_op(at::Tensor flag, const TensorLists& lists);
std::tuple<at::Tensor, at::Tensor> mt_norm_op(at::Tensor noop, const std::vector<at::Tensor>& list,
                                              bool per_tensor, bool max_norm);
void mt_sgd_op(at::Tensor noop, const TensorLists& lists, double wd, double momentum,
               double dampening, double lr, OptT lr_t, bool nesterov, bool first_run,
               OptT first_run_flag, bool wd_after_momentum, double scale, OptT scale_t,
               bool scale_inv);
void mt_adam_op(at::Tensor noop, const TensorLists& lists, double lr, OptT lr_t, double beta1,
                double beta2, double eps, int64_t step, OptT step_t, int64_t mode,
                bool bias_correction, double wd, double scale, OptT scale_t, bool scale_inv);
void mt_lamb_op(at::Tensor noop, const TensorLists& lists, double lr, OptT lr_t, double beta1,
                double beta2, double eps, int64_t step, OptT step_t, bool bias_correction,
                double wd, bool grad_averaging, int64_t mode, OptT global_grad_norm,
                double max_grad_norm, bool use_nvlamb, double scale, OptT scale_t, bool scale_inv);
void mt_lamb_legacy_stage1_op(at::Tensor noop, const TensorLists& lists, at::Tensor decay,
                              int64_t step, double beta1, double beta2, double eps,
                              at::Tensor global_grad_norm, double max_grad_norm);
void mt_lamb_legacy_stage2_op(at::Tensor noop, const TensorLists& lists, at::Tensor param_norms,
                              at::Tensor update_norms, double lr, double weight_decay,
                              bool use_nvlamb);
void mt_novograd_op(at::Tensor noop, const TensorLists& lists, at::Tensor v, at::Tensor grad_norms,
                    bool first_step, double lr, OptT lr_t, double beta1, double beta2, double eps,
                    int64_t step, OptT step_t, bool bias_correction, double wd,
                    bool grad_averaging, int64_t mode, int64_t norm_type, double scale,
                    OptT scale_t, bool scale_inv);
void mt_adagrad_op(at::Tensor noop, const TensorLists& lists, double lr, OptT lr_t, double eps,
                   int64_t mode, double wd, double scale, OptT scale_t, bool scale_inv);
void update_loss_scale_op(at::Tensor scale, at::Tensor unskipped, OptT skipped, at::Tensor overflow,
                          double factor, int64_t window, double min_scale, double max_scale,
                          bool dynamic, OptT applied);
void advance_step_op(at::Tensor step, OptT noop);
void mark_step_done_op(at::Tensor flag, OptT noop);
void flat_scale_op(at::Tensor in, at::Tensor out, double scale, OptT scale_t, bool invert,
                   OptT noop);

// A prepared optimizer launch set (the optimizer-step fast path): the fixed lists
// (params, optimizer state, 16-bit model copies) are converted from Python once;
// the gradient list is read from the owners' .grad each step in C++, and the
// device launch table is re-built only when a gradient moved.  A step is then
// one Python->C++ call per launch set with scalar arguments only.
class StepPlan {
 public:
  StepPlan(std::vector<at::Tensor> owners, TensorLists fixed);
  // false: some owner has no grad / a grad of another dtype, size or layout (the
  // caller re-plans); nothing was launched
  bool refresh();
  bool sgd(at::Tensor noop, double wd, double momentum, double dampening, double lr,
           bool nesterov, bool first_run, OptT first_run_flag, bool wd_after_momentum,
           double scale, OptT scale_t, bool scale_inv);
  // this set and `other` (an fp32 set, e.g. the BatchNorm parameters) in ONE launch
  // (mt_sgd_pair); false when either set cannot (dtypes, CPU, a moved-away grad) - the
  // caller then launches the sets one by one
  bool sgd_pair(StepPlan& other, at::Tensor noop, double wd, double momentum, double dampening,
                double lr, bool nesterov, bool wd_after_momentum, double scale, OptT scale_t,
                bool scale_inv, double other_scale, OptT other_scale_t, bool other_scale_inv);
  bool adam(at::Tensor noop, double lr, OptT lr_t, double beta1, double beta2, double eps,
            int64_t step, OptT step_t, int64_t mode, bool bias_correction, double wd,
            double scale, OptT scale_t, bool scale_inv, bool advance_step);
  // ||grads||_2 of this set into out[slot] (fp32 device vector), unscaled: divided by
  // scale_t when given, else multiplied by scale; `flag` is a scratch overflow flag the
  // norm kernels may write (never the step's noop flag)
  bool grad_norm_into(at::Tensor out, int64_t slot, at::Tensor flag, double scale, OptT scale_t);
  // FusedLAMB's two stages (mt_lamb_op) on cached launch tables: stage 1 + per-tensor
  // norm finalize on [grads, params, m, v], stage 2 on [params, m, v(, copies)]
  bool lamb(at::Tensor noop, double lr, OptT lr_t, double beta1, double beta2, double eps,
            int64_t step, OptT step_t, bool bias_correction, double wd, bool grad_averaging,
            int64_t mode, at::Tensor global_grad_norm, double max_grad_norm, bool use_nvlamb,
            double scale, OptT scale_t, bool scale_inv, bool advance_step);
  // tensors that must stay without a grad (a param gaining one changes the sets)
  void set_absent(std::vector<at::Tensor> absent) { absent_ = std::move(absent); }
  int64_t size() const { return (int64_t)owners_.size(); }
  int64_t rebuilds() const { return rebuilds_; }

 private:
  bool gpu_launch_ready();
  std::vector<at::Tensor> owners_, absent_;
  TensorLists lists_;  // [grads, fixed...]
  std::vector<void*> gptr_;
  at::ScalarType gtype_;
  MTPlan plan_;
  bool gpu_ = false, fresh_ = false;
  int64_t rebuilds_ = 0;
  // sub-launch tables (grad norm, LAMB stage 1 / 2), rebuilt when the grads moved (gen_)
  int64_t gen_ = 0, ngen_ = -1, l1gen_ = -1;
  bool l2ok_ = false;
  MTPlan nplan_, l1plan_, l2plan_;
  at::Tensor npart_, l1part_, l1norm_;
};

void mt_plan_cache_clear();
int64_t mt_plan_cache_size();

}  // namespace amd
