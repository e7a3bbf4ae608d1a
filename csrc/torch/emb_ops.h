// Torch binding of the deterministic embedding weight gradient (csrc/hip/embedding.hip).
#pragma once
#include <ATen/ATen.h>

namespace amd {

// dW [V, H] (dtype out_dtype) of an embedding lookup with ids `idx` (any shape, T ids)
// and output gradient dy [T, H]; padding_idx < 0: none.  Deterministic, no host sync.
at::Tensor embedding_wgrad_op(at::Tensor idx, at::Tensor dy, int64_t V, int64_t padding_idx,
                              c10::ScalarType out_dtype);

}  // namespace amd
