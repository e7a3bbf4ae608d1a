// Fused optimizer kernels over the device-resident multi-tensor table.
//
// Behavioural spec: apex@f3a960f8
//   csrc/multi_tensor_sgd_kernel.cu      -> sgd_kernel
//   csrc/multi_tensor_adam.cu            -> adam_kernel
//   csrc/multi_tensor_lamb.cu (+stage_1/2) -> lamb_stage1_kernel / lamb_stage2_kernel
//   csrc/multi_tensor_novograd.cu        -> novograd_kernel
//   csrc/multi_tensor_adagrad.cu         -> adagrad_kernel
//
// MI355X design:
//  * one launch per (optimizer, dtype-combo) covers every tensor (mt_table.h);
//  * every kernel reads the overflow flag on device and exits -> a skipped amp
//    step costs no host synchronisation;
//  * the loss-scale reciprocal, the lr and the step counter may come from device
//    scalars, so the whole optimizer step is hipGraph-capturable;
//  * LAMB stage 1 emits the per-chunk ||p||^2 and ||u||^2 partials in the same
//    pass that produces u (saves two extra reads of p and u vs apex's
//    stage1 -> l2norm -> l2norm -> stage2 sequence).
#include "mt_device.h"

namespace amd {

__device__ __forceinline__ bool skip_step(const int* noop) { return noop && *noop; }
__device__ __forceinline__ float lr_of(const float* p, float v) { return p ? *p : v; }

// --------------------------------------------------------------------------
// SGD
template <typename TG, typename TP, typename TM, typename TC, int DEPTH>
__global__ void __launch_bounds__(kMTThreads) sgd_kernel(MTLaunch L, SgdArgs a, const int* noop) {
  if (skip_step(noop)) return;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
  const bool first = a.first_run_flag ? (*a.first_run_flag == 0) : (a.first_run != 0);
  const bool has_mom = a.momentum != 0.f;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    int64_t idx = c.start + off;
    float g[8], p[8], m[8];
    ld<TG>(c.t->ptr[0], idx, cnt, vec, g);
    ld<TP>(c.t->ptr[1], idx, cnt, vec, p);
    if (has_mom && !first) ld<TM>(c.t->ptr[2], idx, cnt, vec, m);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * sc;
      if (a.wd != 0.f && !a.wd_after_momentum) gi = fmaf(a.wd, p[i], gi);
      if (has_mom) {
        m[i] = first ? gi : fmaf(m[i], a.momentum, (1.f - a.dampening) * gi);
        gi = a.nesterov ? fmaf(a.momentum, m[i], gi) : m[i];
      }
      if (a.wd != 0.f && a.wd_after_momentum) gi = fmaf(a.wd, p[i], gi);
      p[i] = fmaf(-lr, gi, p[i]);
    }
    st<TP>(c.t->ptr[1], idx, cnt, vec, p);
    if (has_mom) st<TM>(c.t->ptr[2], idx, cnt, vec, m);
    if (DEPTH == 4) st<TC>(c.t->ptr[3], idx, cnt, vec, p);
  }
}

void mt_sgd(const MTLaunch& L, int depth, DType g, DType p, DType m, DType copy, const SgdArgs& a,
            const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  // momentum buffers always share the parameter dtype (zeros_like(p))
  (void)m;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      if (depth == 3) {
        hipLaunchKernelGGL((sgd_kernel<TG, TP, TP, TP, 3>), mt_grid(L), dim3(kMTThreads), 0, st,
                           L, a, noop);
      } else {
        dispatch1(copy, [&](auto tc) {
          using TC = decltype(tc);
          hipLaunchKernelGGL((sgd_kernel<TG, TP, TP, TC, 4>), mt_grid(L), dim3(kMTThreads), 0, st,
                             L, a, noop);
        });
      }
    });
  });
}

// --------------------------------------------------------------------------
// Adam / AdamW
__device__ __forceinline__ void bias_corrections(int bias_correction, float b1, float b2, int step,
                                                 float& bc1, float& bc2) {
  if (bias_correction) {
    bc1 = 1.f - powf(b1, (float)step);
    bc2 = 1.f - powf(b2, (float)step);
  } else {
    bc1 = 1.f;
    bc2 = 1.f;
  }
}

template <typename TG, typename TP, typename TC, int DEPTH>
__global__ void __launch_bounds__(kMTThreads) adam_kernel(MTLaunch L, AdamArgs a, const int* noop) {
  if (skip_step(noop)) return;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
  const int step = a.step_ptr ? (*a.step_ptr + 1) : a.step;
  float bc1, bc2;
  bias_corrections(a.bias_correction, a.beta1, a.beta2, step, bc1, bc2);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    int64_t idx = c.start + off;
    float g[8], p[8], m[8], v[8];
    ld<TG>(c.t->ptr[0], idx, cnt, vec, g);
    ld<TP>(c.t->ptr[1], idx, cnt, vec, p);
    ld<TP>(c.t->ptr[2], idx, cnt, vec, m);
    ld<TP>(c.t->ptr[3], idx, cnt, vec, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * sc;
      if (a.mode == 0) gi = fmaf(a.wd, p[i], gi);
      m[i] = fmaf(a.beta1, m[i], (1.f - a.beta1) * gi);
      v[i] = fmaf(a.beta2, v[i], (1.f - a.beta2) * gi * gi);
      float denom = sqrtf(v[i]) * inv_sqrt_bc2 + a.eps;
      float upd = (m[i] / denom) * step_size;
      if (a.mode == 1) upd = fmaf(lr * a.wd, p[i], upd);
      p[i] -= upd;
    }
    st<TP>(c.t->ptr[1], idx, cnt, vec, p);
    st<TP>(c.t->ptr[2], idx, cnt, vec, m);
    st<TP>(c.t->ptr[3], idx, cnt, vec, v);
    if (DEPTH == 5) st<TC>(c.t->ptr[4], idx, cnt, vec, p);
  }
}

void mt_adam(const MTLaunch& L, int depth, DType g, DType p, DType copy, const AdamArgs& a,
             const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      if (depth == 4) {
        hipLaunchKernelGGL((adam_kernel<TG, TP, TP, 4>), mt_grid(L), dim3(kMTThreads), 0, st, L, a,
                           noop);
      } else {
        dispatch1(copy, [&](auto tc) {
          using TC = decltype(tc);
          hipLaunchKernelGGL((adam_kernel<TG, TP, TC, 5>), mt_grid(L), dim3(kMTThreads), 0, st, L,
                             a, noop);
        });
      }
    });
  });
}

// --------------------------------------------------------------------------
// LAMB
template <typename TG, typename TP>
__global__ void __launch_bounds__(kMTThreads)
    lamb_stage1_kernel(MTLaunch L, LambArgs a, float* partials, const int* noop) {
  __shared__ float scratch[kMTThreads / kWave];
  if (skip_step(noop)) return;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  const float sc = get_scale(a.scale);
  const int step = a.step_ptr ? (*a.step_ptr + 1) : a.step;
  float bc1, bc2;
  bias_corrections(a.bias_correction, a.beta1, a.beta2, step, bc1, bc2);
  const float beta3 = a.grad_averaging ? (1.f - a.beta1) : 1.f;
  float gn = a.global_grad_norm ? *a.global_grad_norm : 0.f;
  const float clip = (a.max_grad_norm > 0.f && gn > a.max_grad_norm) ? gn / a.max_grad_norm : 1.f;
  const float gmul = sc / clip;
  float pn2 = 0.f, un2 = 0.f;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    int64_t idx = c.start + off;
    float g[8], p[8], m[8], v[8], up[8];
    ld<TG>(c.t->ptr[0], idx, cnt, vec, g);
    ld<TP>(c.t->ptr[1], idx, cnt, vec, p);
    ld<TP>(c.t->ptr[2], idx, cnt, vec, m);
    ld<TP>(c.t->ptr[3], idx, cnt, vec, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * gmul;
      if (a.mode == 0) gi = fmaf(a.wd, p[i], gi);
      m[i] = fmaf(a.beta1, m[i], beta3 * gi);
      v[i] = fmaf(a.beta2, v[i], (1.f - a.beta2) * gi * gi);
      float mh = m[i] / bc1;
      float vh = v[i] / bc2;
      float uu = mh / (sqrtf(vh) + a.eps);
      if (a.mode == 1) uu = fmaf(a.wd, p[i], uu);
      up[i] = (i < cnt) ? uu : 0.f;
      float pi = (i < cnt) ? p[i] : 0.f;
      pn2 = fmaf(pi, pi, pn2);
      un2 = fmaf(up[i], up[i], un2);
    }
    st<TP>(c.t->ptr[2], idx, cnt, vec, m);
    st<TP>(c.t->ptr[3], idx, cnt, vec, v);
    st<float>(c.t->ptr[4], idx, cnt, vec, up);
  }
  float rp = block_sum(pn2, scratch);
  float ru = block_sum(un2, scratch);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = rp;
    partials[L.nchunks + blockIdx.x] = ru;
  }
}

template <typename TP, typename TC, int DEPTH>
__global__ void __launch_bounds__(kMTThreads)
    lamb_stage2_kernel(MTLaunch L, LambArgs a, const float* pnorm, const float* unorm,
                       const int* noop) {
  if (skip_step(noop)) return;
  const int tensor = L.chunks[blockIdx.x].tensor;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  const float lr = lr_of(a.lr_ptr, a.lr);
  float ratio = lr;
  if (a.use_nvlamb || a.wd != 0.f) {
    float pn = pnorm[tensor], un = unorm[tensor];
    ratio = (pn != 0.f && un != 0.f) ? lr * (pn / un) : lr;
  }
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    int64_t idx = c.start + off;
    float p[8], up[8];
    ld<TP>(c.t->ptr[0], idx, cnt, vec, p);
    ld<float>(c.t->ptr[1], idx, cnt, vec, up);
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = fmaf(-ratio, up[i], p[i]);
    st<TP>(c.t->ptr[0], idx, cnt, vec, p);
    if (DEPTH == 3) st<TC>(c.t->ptr[2], idx, cnt, vec, p);
  }
}

void mt_lamb_stage1(const MTLaunch& L, DType g, DType p, const LambArgs& a, float* partials,
                    const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((lamb_stage1_kernel<TG, TP>), mt_grid(L), dim3(kMTThreads), 0, st, L, a,
                         partials, noop);
    });
  });
}

void mt_lamb_stage2(const MTLaunch& L, int depth, DType p, DType copy, const LambArgs& a,
                    const float* param_norms, const float* update_norms, const int* noop,
                    hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(p, [&](auto tp) {
    using TP = decltype(tp);
    if (depth == 2) {
      hipLaunchKernelGGL((lamb_stage2_kernel<TP, TP, 2>), mt_grid(L), dim3(kMTThreads), 0, st, L,
                         a, param_norms, update_norms, noop);
    } else {
      dispatch1(copy, [&](auto tc) {
        using TC = decltype(tc);
        hipLaunchKernelGGL((lamb_stage2_kernel<TP, TC, 3>), mt_grid(L), dim3(kMTThreads), 0, st,
                           L, a, param_norms, update_norms, noop);
      });
    }
  });
}

// --------------------------------------------------------------------------
// NovoGrad: per-tensor second moment kept as a norm
__global__ void novograd_blend_kernel(float* v, const float* gn, int n, float beta2, int norm_type,
                                      int first_step, const int* noop) {
  if (skip_step(noop)) return;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float g = gn[i];
  if (first_step) {
    v[i] = g;
  } else if (norm_type == 2) {
    v[i] = sqrtf(beta2 * v[i] * v[i] + (1.f - beta2) * g * g);
  } else {
    v[i] = beta2 * v[i] + (1.f - beta2) * g;
  }
}

void novograd_blend(float* v, const float* grad_norms, int ntensors, float beta2, int norm_type,
                    int first_step, const int* noop, hipStream_t st) {
  if (ntensors == 0) return;
  hipLaunchKernelGGL(novograd_blend_kernel, dim3((ntensors + 255) / 256), dim3(256), 0, st, v,
                     grad_norms, ntensors, beta2, norm_type, first_step, noop);
}

template <typename TG, typename TP>
__global__ void __launch_bounds__(kMTThreads)
    novograd_kernel(MTLaunch L, NovoArgs a, const float* vnorm, const int* noop) {
  if (skip_step(noop)) return;
  const int tensor = L.chunks[blockIdx.x].tensor;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
  const int step = a.step_ptr ? (*a.step_ptr + 1) : a.step;
  float bc1, bc2;
  bias_corrections(a.bias_correction, a.beta1, a.beta2, step, bc1, bc2);
  const float beta3 = a.grad_averaging ? (1.f - a.beta1) : 1.f;
  const float denom = vnorm[tensor] / sqrtf(bc2) + a.eps;
  const float inv_denom = 1.f / denom;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    int64_t idx = c.start + off;
    float g[8], p[8], m[8];
    ld<TG>(c.t->ptr[0], idx, cnt, vec, g);
    ld<TP>(c.t->ptr[1], idx, cnt, vec, p);
    ld<TP>(c.t->ptr[2], idx, cnt, vec, m);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * sc * inv_denom;
      if (a.mode == 0) gi = fmaf(a.wd, p[i], gi);
      m[i] = fmaf(a.beta1, m[i], beta3 * gi);
      float upd = m[i] / bc1;
      if (a.mode == 1) upd = fmaf(a.wd, p[i], upd);
      p[i] = fmaf(-lr, upd, p[i]);
    }
    st<TP>(c.t->ptr[1], idx, cnt, vec, p);
    st<TP>(c.t->ptr[2], idx, cnt, vec, m);
  }
}

void mt_novograd(const MTLaunch& L, DType g, DType p, const NovoArgs& a, const float* v,
                 const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((novograd_kernel<TG, TP>), mt_grid(L), dim3(kMTThreads), 0, st, L, a, v,
                         noop);
    });
  });
}

// --------------------------------------------------------------------------
// Adagrad
template <typename TG, typename TP>
__global__ void __launch_bounds__(kMTThreads)
    adagrad_kernel(MTLaunch L, AdagradArgs a, const int* noop) {
  if (skip_step(noop)) return;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    int64_t idx = c.start + off;
    float g[8], p[8], h[8];
    ld<TG>(c.t->ptr[0], idx, cnt, vec, g);
    ld<TP>(c.t->ptr[1], idx, cnt, vec, p);
    ld<TP>(c.t->ptr[2], idx, cnt, vec, h);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * sc;
      if (a.mode == 0) gi = fmaf(a.wd, p[i], gi);
      h[i] = fmaf(gi, gi, h[i]);
      float upd = gi / (sqrtf(h[i]) + a.eps);
      if (a.mode == 1) upd = fmaf(a.wd, p[i], upd);
      p[i] = fmaf(-lr, upd, p[i]);
    }
    st<TP>(c.t->ptr[1], idx, cnt, vec, p);
    st<TP>(c.t->ptr[2], idx, cnt, vec, h);
  }
}

void mt_adagrad(const MTLaunch& L, DType g, DType p, const AdagradArgs& a, const int* noop,
                hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((adagrad_kernel<TG, TP>), mt_grid(L), dim3(kMTThreads), 0, st, L, a,
                         noop);
    });
  });
}

}  // namespace amd
