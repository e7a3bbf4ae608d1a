// Torch-facing helpers shared by the binding translation units.
#pragma once
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/util/Optional.h>
#include <c10/core/GradMode.h>

#include <vector>

#include "amd_kernels.h"
#include "mt_table.h"

namespace amd {

enum class DType : int { F32 = 0, F16 = 1, BF16 = 2, F64 = 3 };

inline DType dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DType::F32;
    case at::kHalf: return DType::F16;
    case at::kBFloat16: return DType::BF16;
    case at::kDouble: return DType::F64;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return DType::F32;
}

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// A scale factor from Python: value, optional device scalar, optional reciprocal.
inline ScaleArg make_scale(double v, const c10::optional<at::Tensor>& t, bool invert) {
  ScaleArg s;
  s.val = (float)v;
  s.invert = invert ? 1 : 0;
  s.ptr = nullptr;
  if (t.has_value() && t->defined()) {
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= 1, "scale tensor must be float32");
    s.ptr = t->data_ptr<float>();
  }
  return s;
}

inline float* opt_fptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat, "expected float32 tensor");
  return t->data_ptr<float>();
}
inline int* opt_iptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kInt, "expected int32 tensor");
  return t->data_ptr<int>();
}

using TensorLists = std::vector<std::vector<at::Tensor>>;

// Validates `lists` and returns the device launch table: a cached one, or one
// whose chunk list is cached by tensor sizes and whose tensor table is uploaded
// for this call (mt_plan.cpp).  Hold the returned plan until the launch is issued.
struct MTPlan {
  at::Tensor table;  // device bytes (kept alive by the cache, or by this plan)
  at::Tensor host;   // pinned source image (kept alive: graph-captured copies re-read it)
  at::Tensor chunks; // per-call plans: the size-keyed chunk table they point into
  bool captured = false;  // built inside a graph capture: never evicted
  MTLaunch L;
};
MTPlan mt_plan(const TensorLists& lists);

// Shared validation: every list has the same length, matching numel per slot,
// contiguous tensors.  Returns true if the lists live on the GPU.
bool mt_validate(const TensorLists& lists, int min_depth, int max_depth);

}  // namespace amd
