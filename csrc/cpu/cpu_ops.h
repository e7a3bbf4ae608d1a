// C++ CPU implementations of the amp_C / optimizer / norm kernels.
//
// These serve the CPU plumbing configuration (BASELINE.json configs[0]: amp O0,
// world_size=1, no GPU) and are the host reference the HIP kernels are tested
// against.  Same semantics as csrc/hip/*.hip, fp32 math, float64 not used.
#pragma once
#include <ATen/ATen.h>

#include <vector>

namespace amd {
namespace cpu {

using TensorLists = std::vector<std::vector<at::Tensor>>;

struct Scale {
  double val;
  const at::Tensor* t;  // optional CPU float scalar
  bool invert;
  float get() const {
    float v = t && t->defined() ? t->item<float>() : (float)val;
    return invert ? 1.f / v : v;
  }
};

bool noop_set(const at::Tensor& noop);

void scale(at::Tensor& noop, const TensorLists& l, Scale s);
void check_finite(at::Tensor& noop, const std::vector<at::Tensor>& l);
void axpby(at::Tensor& noop, const TensorLists& l, Scale a, Scale b, int arg_to_check);
void zero(const std::vector<at::Tensor>& l);
void norm(at::Tensor& noop, const std::vector<at::Tensor>& l, bool max_norm, at::Tensor& out,
          at::Tensor* per_tensor);

struct Sgd {
  float wd, momentum, dampening, lr;
  bool nesterov, first_run, wd_after_momentum;
  Scale scale;
  at::Tensor* first_run_flag;  // optional int32 [1]
};
void sgd(at::Tensor& noop, const TensorLists& l, const Sgd& a);

struct Adam {
  float lr, b1, b2, eps, wd;
  int step;
  at::Tensor* step_t;  // optional int32 [1] completed-step counter
  int mode, bias_correction;
  Scale scale;
};
void adam(at::Tensor& noop, const TensorLists& l, const Adam& a);

struct Lamb {
  float lr, b1, b2, eps, wd;
  int step;
  at::Tensor* step_t;
  int mode, bias_correction, grad_averaging;
  at::Tensor* global_norm;  // optional float [1]
  float max_grad_norm;
  bool use_nvlamb;
  Scale scale;
};
// lists: [g, p, m, v, u] (+ optional p_copy as 6th)
void lamb(at::Tensor& noop, const TensorLists& l, const Lamb& a);

struct Novo {
  float lr, b1, b2, eps, wd;
  int step;
  at::Tensor* step_t;
  int mode, bias_correction, grad_averaging, norm_type;
  Scale scale;
};
// lists [g, p, m]; v per-tensor norms (float [n]); grad_norms this step's norms
void novograd(at::Tensor& noop, const TensorLists& l, at::Tensor& v, const at::Tensor& grad_norms,
              bool first_step, const Novo& a);

struct Adagrad {
  float lr, eps, wd;
  int mode;
  Scale scale;
};
void adagrad(at::Tensor& noop, const TensorLists& l, const Adagrad& a);

void update_loss_scale(at::Tensor& scale, at::Tensor& unskipped, at::Tensor* skipped,
                       const at::Tensor& overflow, float factor, int window, float min_scale,
                       float max_scale, bool dynamic);

}  // namespace cpu
}  // namespace amd
