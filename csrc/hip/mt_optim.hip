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
//    pass that updates the moments, and stage 2 RECOMPUTES u from (p, m, v)
//    instead of reading an fp32 update workspace: no 4 B/param persistent
//    buffer (1.3 GB for BERT-large) and the same 42 B/param of traffic as
//    apex's stage1 -> l2norm -> l2norm -> stage2 sequence minus its two norm
//    passes;
//  * every kernel is persistent (mt_pgrid: min(#chunks, CUs x k) workgroups
//    walking the chunk list) and issues all of a tile's loads before any
//    arithmetic: the stores of one 8-vector can no longer serialise the loads
//    of the next (the table pointers may alias as far as the compiler knows).
#include <cstdlib>

#include "mt_device.h"

namespace amd {

__device__ __forceinline__ bool skip_step(const int* noop) { return noop && *noop; }
__device__ __forceinline__ float lr_of(const float* p, float v) { return p ? *p : v; }

// --------------------------------------------------------------------------
// SGD
struct SgdConsts {
  float sc, lr;
  bool first, has_mom, load_m;
};
__device__ __forceinline__ SgdConsts sgd_consts(const SgdArgs& a) {
  SgdConsts k;
  k.sc = get_scale(a.scale);
  k.lr = lr_of(a.lr_ptr, a.lr);
  k.first = a.first_run_flag ? (*a.first_run_flag == 0) : (a.first_run != 0);
  k.has_mom = a.momentum != 0.f;
  k.load_m = k.has_mom && !k.first;
  return k;
}

template <typename TG, typename TP, typename TM, typename TC, int DEPTH>
__device__ __forceinline__ void sgd_chunk(const MTLaunch& L, int ch, const SgdArgs& a,
                                          const SgdConsts& k) {
  const TileCtx c = tile_ctx(L, ch);
  const bool al = c.t->aligned;
  float g[kMTUnroll][8], p[kMTUnroll][8], m[kMTUnroll][8];
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    const int off = lane_off(u), cnt = c.n - off;
    if (cnt <= 0) continue;
    const bool vec = al && cnt >= 8;
    const int64_t idx = c.start + off;
    ld<TG>(c.t->ptr[0], idx, cnt, vec, g[u]);
    ld<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
    if (k.load_m) ld<TM>(c.t->ptr[2], idx, cnt, vec, m[u]);
  }
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    const int off = lane_off(u), cnt = c.n - off;
    if (cnt <= 0) continue;
    const bool vec = al && cnt >= 8;
    const int64_t idx = c.start + off;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[u][i] * k.sc;
      if (a.wd != 0.f && !a.wd_after_momentum) gi = fmaf(a.wd, p[u][i], gi);
      if (k.has_mom) {
        m[u][i] = k.first ? gi : fmaf(m[u][i], a.momentum, (1.f - a.dampening) * gi);
        gi = a.nesterov ? fmaf(a.momentum, m[u][i], gi) : m[u][i];
      }
      if (a.wd != 0.f && a.wd_after_momentum) gi = fmaf(a.wd, p[u][i], gi);
      p[u][i] = fmaf(-k.lr, gi, p[u][i]);
    }
    st<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
    if (k.has_mom) st<TM>(c.t->ptr[2], idx, cnt, vec, m[u]);
    if (DEPTH == 4) st<TC>(c.t->ptr[3], idx, cnt, vec, p[u]);
  }
}

template <typename TG, typename TP, typename TM, typename TC, int DEPTH>
__global__ void __launch_bounds__(kMTThreads) sgd_kernel(MTLaunch L, SgdArgs a, const int* noop) {
  if (skip_step(noop)) return;
  const SgdConsts k = sgd_consts(a);
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x)
    sgd_chunk<TG, TP, TM, TC, DEPTH>(L, ch, a, k);
}

// Two launch sets of one param group in ONE launch (FusedSGD's amp O2 step: the
// 16-bit-copy set [g16, p32, m32, c16] and the fp32 BatchNorm set [g32, p32, m32]):
// chunk ids below A.nchunks belong to set A - a block-uniform branch - so the small
// second set costs no launch of its own.
template <typename TGA, typename TCA>
__global__ void __launch_bounds__(kMTThreads)
    sgd_pair_kernel(MTLaunch A, SgdArgs aa, MTLaunch B, SgdArgs ab, const int* noop) {
  if (skip_step(noop)) return;
  const SgdConsts ka = sgd_consts(aa), kb = sgd_consts(ab);
  const int n = A.nchunks + B.nchunks;
  for (int ch = blockIdx.x; ch < n; ch += gridDim.x) {
    if (ch < A.nchunks) sgd_chunk<TGA, float, float, TCA, 4>(A, ch, aa, ka);
    else sgd_chunk<float, float, float, float, 3>(B, ch - A.nchunks, ab, kb);
  }
}

bool mt_sgd_pair(const MTLaunch& A, DType ga, DType pa, DType ca, const SgdArgs& aa,
                 const MTLaunch& B, DType gb, DType pb, const SgdArgs& ab, const int* noop,
                 hipStream_t st) {
  if (pa != DType::F32 || pb != DType::F32 || gb != DType::F32 || ca == DType::F32 ||
      ga == DType::F64 || ca == DType::F64)
    return false;
  MTLaunch both = A;
  both.nchunks = A.nchunks + B.nchunks;
  const dim3 grid = mt_pgrid(both);
  dispatch1(ga, [&](auto tg) {
    dispatch1(ca, [&](auto tc) {
      using TG = decltype(tg);
      using TC = decltype(tc);
      if constexpr (!std::is_same<TC, float>::value)
        hipLaunchKernelGGL((sgd_pair_kernel<TG, TC>), grid, dim3(kMTThreads), 0, st, A, aa, B, ab,
                           noop);
    });
  });
  return true;
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
        hipLaunchKernelGGL((sgd_kernel<TG, TP, TP, TP, 3>), mt_pgrid(L), dim3(kMTThreads), 0, st,
                           L, a, noop);
      } else {
        dispatch1(copy, [&](auto tc) {
          using TC = decltype(tc);
          hipLaunchKernelGGL((sgd_kernel<TG, TP, TP, TC, 4>), mt_pgrid(L), dim3(kMTThreads), 0,
                             st, L, a, noop);
        });
      }
    });
  });
}

// Adam / LAMB keep 4 state arrays per 8-vector: half a tile's vectors per pass
// (64 instead of 128 data VGPRs) doubles the resident waves per SIMD.
constexpr int UA = 2;

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
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
  const int step = a.step_ptr ? (*a.step_ptr + 1) : a.step;
  float bc1, bc2;
  bias_corrections(a.bias_correction, a.beta1, a.beta2, step, bc1, bc2);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const TileCtx c = tile_ctx(L, ch);
    const bool al = c.t->aligned;
#pragma unroll 1
    for (int h = 0; h < kMTUnroll / UA; ++h) {
      float g[UA][8], p[UA][8], m[UA][8], v[UA][8];
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
        ld<TG>(c.t->ptr[0], idx, cnt, vec, g[u]);
        ld<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
        ld<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
        ld<TP>(c.t->ptr[3], idx, cnt, vec, v[u]);
      }
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float gi = g[u][i] * sc;
          if (a.mode == 0) gi = fmaf(a.wd, p[u][i], gi);
          m[u][i] = fmaf(a.beta1, m[u][i], (1.f - a.beta1) * gi);
          v[u][i] = fmaf(a.beta2, v[u][i], (1.f - a.beta2) * gi * gi);
          const float denom = sqrtf(v[u][i]) * inv_sqrt_bc2 + a.eps;
          float upd = (m[u][i] / denom) * step_size;
          if (a.mode == 1) upd = fmaf(lr * a.wd, p[u][i], upd);
          p[u][i] -= upd;
        }
        st<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
        st<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
        st<TP>(c.t->ptr[3], idx, cnt, vec, v[u]);
        if (DEPTH == 5) st<TC>(c.t->ptr[4], idx, cnt, vec, p[u]);
      }
    }
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
        hipLaunchKernelGGL((adam_kernel<TG, TP, TP, 4>), mt_pgrid(L), dim3(kMTThreads), 0, st, L,
                           a, noop);
      } else {
        dispatch1(copy, [&](auto tc) {
          using TC = decltype(tc);
          hipLaunchKernelGGL((adam_kernel<TG, TP, TC, 5>), mt_pgrid(L), dim3(kMTThreads), 0, st,
                             L, a, noop);
        });
      }
    });
  });
}

// --------------------------------------------------------------------------
// LAMB
struct LambConsts {
  float bc1, bc2, beta3, gmul;
};

__device__ __forceinline__ LambConsts lamb_consts(const LambArgs& a) {
  LambConsts k;
  const int step = a.step_ptr ? (*a.step_ptr + 1) : a.step;
  bias_corrections(a.bias_correction, a.beta1, a.beta2, step, k.bc1, k.bc2);
  k.beta3 = a.grad_averaging ? (1.f - a.beta1) : 1.f;
  const float gn = a.global_grad_norm ? *a.global_grad_norm : 0.f;
  const float clip = (a.max_grad_norm > 0.f && gn > a.max_grad_norm) ? gn / a.max_grad_norm : 1.f;
  k.gmul = get_scale(a.scale) / clip;
  return k;
}

// the update direction from the (already updated) moments: stage 1 uses it for
// ||u||, stage 2 recomputes it bit-identically for the parameter update
__device__ __forceinline__ float lamb_update(const LambArgs& a, const LambConsts& k, float m,
                                             float v, float p) {
  const float mh = m / k.bc1;
  const float vh = v / k.bc2;
  float uu = mh / (sqrtf(vh) + a.eps);
  if (a.mode == 1) uu = fmaf(a.wd, p, uu);
  return uu;
}

template <typename TG, typename TP>
__global__ void __launch_bounds__(kMTThreads)
    lamb_stage1_kernel(MTLaunch L, LambArgs a, float* partials, const int* noop) {
  __shared__ float scratch[kMTThreads / kWave];
  if (skip_step(noop)) return;
  const LambConsts k = lamb_consts(a);
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const TileCtx c = tile_ctx(L, ch);
    const bool al = c.t->aligned;
    float pn2 = 0.f, un2 = 0.f;
#pragma unroll 1
    for (int h = 0; h < kMTUnroll / UA; ++h) {
      float g[UA][8], p[UA][8], m[UA][8], v[UA][8];
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
        ld<TG>(c.t->ptr[0], idx, cnt, vec, g[u]);
        ld<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
        ld<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
        ld<TP>(c.t->ptr[3], idx, cnt, vec, v[u]);
      }
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float gi = g[u][i] * k.gmul;
          if (a.mode == 0) gi = fmaf(a.wd, p[u][i], gi);
          m[u][i] = fmaf(a.beta1, m[u][i], k.beta3 * gi);
          v[u][i] = fmaf(a.beta2, v[u][i], (1.f - a.beta2) * gi * gi);
          // m / v are stored in TP: recompute u from the ROUNDED values stage 2 reads
          m[u][i] = to_f32(from_f32<TP>(m[u][i]));
          v[u][i] = to_f32(from_f32<TP>(v[u][i]));
          const float uu = (i < cnt) ? lamb_update(a, k, m[u][i], v[u][i], p[u][i]) : 0.f;
          const float pi = (i < cnt) ? p[u][i] : 0.f;
          pn2 = fmaf(pi, pi, pn2);
          un2 = fmaf(uu, uu, un2);
        }
        st<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
        st<TP>(c.t->ptr[3], idx, cnt, vec, v[u]);
      }
    }
    const float rp = block_sum(pn2, scratch);
    const float ru = block_sum(un2, scratch);
    if (threadIdx.x == 0) {
      partials[ch] = rp;
      partials[L.nchunks + ch] = ru;
    }
  }
}

// stage 2 lists: [p, m, v] or [p, m, v, p_copy]
template <typename TP, typename TC, int DEPTH>
__global__ void __launch_bounds__(kMTThreads)
    lamb_stage2_kernel(MTLaunch L, LambArgs a, const float* pnorm, const float* unorm,
                       const int* noop) {
  if (skip_step(noop)) return;
  const LambConsts k = lamb_consts(a);
  const float lr = lr_of(a.lr_ptr, a.lr);
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const int tensor = L.chunks[ch].tensor;
    const TileCtx c = tile_ctx(L, ch);
    const bool al = c.t->aligned;
#pragma unroll 1
    for (int h = 0; h < kMTUnroll / UA; ++h) {
      float ratio = lr;
      if (a.use_nvlamb || a.wd != 0.f) {
        const float pn = pnorm[tensor], un = unorm[tensor];
        ratio = (pn != 0.f && un != 0.f) ? lr * (pn / un) : lr;
      }
      float p[UA][8], m[UA][8], v[UA][8];
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
        ld<TP>(c.t->ptr[0], idx, cnt, vec, p[u]);
        ld<TP>(c.t->ptr[1], idx, cnt, vec, m[u]);
        ld<TP>(c.t->ptr[2], idx, cnt, vec, v[u]);
      }
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          p[u][i] = fmaf(-ratio, lamb_update(a, k, m[u][i], v[u][i], p[u][i]), p[u][i]);
        st<TP>(c.t->ptr[0], idx, cnt, vec, p[u]);
        if (DEPTH == 4) st<TC>(c.t->ptr[3], idx, cnt, vec, p[u]);
      }
    }
  }
}

// ---------------------------------------------------------------- legacy two-stage LAMB
// (apex csrc/multi_tensor_lamb_stage_1.cu / _2.cu semantics; lists [g, p, m, v, u] and
// [p, u], m / v / u stored in the parameter type)
template <typename TG, typename TP>
__global__ void __launch_bounds__(kMTThreads)
    lamb_legacy1_kernel(MTLaunch L, LambLegacyArgs a, const int* noop) {
  if (skip_step(noop)) return;
  const float gn = *a.global_grad_norm;
  const float inv_clip = gn > a.max_grad_norm ? a.max_grad_norm / gn : 1.f;
  const float ib1 = 1.f / a.bc1, ib2 = 1.f / a.bc2;
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const TileCtx c = tile_ctx(L, ch);
    const float decay = a.decay[L.chunks[ch].tensor];
    const bool al = c.t->aligned;
#pragma unroll 1
    for (int h = 0; h < kMTUnroll / UA; ++h) {
      float g[UA][8], p[UA][8], m[UA][8], v[UA][8];
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
        ld<TG>(c.t->ptr[0], idx, cnt, vec, g[u]);
        ld<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
        ld<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
        ld<TP>(c.t->ptr[3], idx, cnt, vec, v[u]);
      }
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float gi = g[u][i] * inv_clip;
          m[u][i] = fmaf(a.beta1, m[u][i], (1.f - a.beta1) * gi);
          v[u][i] = fmaf(a.beta2, v[u][i], (1.f - a.beta2) * gi * gi);
          const float den = sqrtf(v[u][i] * ib2) + a.eps;
          g[u][i] = fmaf(decay, p[u][i], (m[u][i] * ib1) / den);  // u (in g's registers)
        }
        st<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
        st<TP>(c.t->ptr[3], idx, cnt, vec, v[u]);
        st<TP>(c.t->ptr[4], idx, cnt, vec, g[u]);
      }
    }
  }
}

template <typename TP, typename TU>
__global__ void __launch_bounds__(kMTThreads)
    lamb_legacy2_kernel(MTLaunch L, LambLegacyArgs a, const int* noop) {
  if (skip_step(noop)) return;
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const int tensor = L.chunks[ch].tensor;
    const TileCtx c = tile_ctx(L, ch);
    const bool al = c.t->aligned;
    float ratio = a.lr;
    if (a.use_nvlamb || a.wd != 0.f) {
      const float pn = a.param_norms[tensor], un = a.update_norms[tensor];
      ratio = (pn != 0.f && un != 0.f) ? a.lr * (pn / un) : a.lr;
    }
#pragma unroll 1
    for (int h = 0; h < kMTUnroll / UA; ++h) {
      float p[UA][8], uu[UA][8];
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
        ld<TP>(c.t->ptr[0], idx, cnt, vec, p[u]);
        ld<TU>(c.t->ptr[1], idx, cnt, vec, uu[u]);
      }
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int off = lane_off(h * UA + u), cnt = c.n - off;
        if (cnt <= 0) continue;
        const bool vec = al && cnt >= 8;
        const int64_t idx = c.start + off;
#pragma unroll
        for (int i = 0; i < 8; ++i) p[u][i] = fmaf(-ratio, uu[u][i], p[u][i]);
        st<TP>(c.t->ptr[0], idx, cnt, vec, p[u]);
      }
    }
  }
}

void mt_lamb_legacy_stage1(const MTLaunch& L, DType g, DType p, const LambLegacyArgs& a,
                           const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((lamb_legacy1_kernel<TG, TP>), mt_pgrid(L), dim3(kMTThreads), 0, st, L,
                         a, noop);
    });
  });
}

void mt_lamb_legacy_stage2(const MTLaunch& L, DType p, DType u, const LambLegacyArgs& a,
                           const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(p, [&](auto tp) {
    dispatch1(u, [&](auto tu) {
      using TP = decltype(tp);
      using TU = decltype(tu);
      hipLaunchKernelGGL((lamb_legacy2_kernel<TP, TU>), mt_pgrid(L), dim3(kMTThreads), 0, st, L,
                         a, noop);
    });
  });
}

void mt_lamb_stage1(const MTLaunch& L, DType g, DType p, const LambArgs& a, float* partials,
                    const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((lamb_stage1_kernel<TG, TP>), mt_pgrid(L), dim3(kMTThreads), 0, st, L, a,
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
    if (depth == 3) {
      hipLaunchKernelGGL((lamb_stage2_kernel<TP, TP, 3>), mt_pgrid(L), dim3(kMTThreads), 0, st, L,
                         a, param_norms, update_norms, noop);
    } else {
      dispatch1(copy, [&](auto tc) {
        using TC = decltype(tc);
        hipLaunchKernelGGL((lamb_stage2_kernel<TP, TC, 4>), mt_pgrid(L), dim3(kMTThreads), 0, st,
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
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
  const int step = a.step_ptr ? (*a.step_ptr + 1) : a.step;
  float bc1, bc2;
  bias_corrections(a.bias_correction, a.beta1, a.beta2, step, bc1, bc2);
  const float beta3 = a.grad_averaging ? (1.f - a.beta1) : 1.f;
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const int tensor = L.chunks[ch].tensor;
    const TileCtx c = tile_ctx(L, ch);
    const bool al = c.t->aligned;
    const float inv_denom = 1.f / (vnorm[tensor] / sqrtf(bc2) + a.eps);
    float g[kMTUnroll][8], p[kMTUnroll][8], m[kMTUnroll][8];
#pragma unroll
    for (int u = 0; u < kMTUnroll; ++u) {
      const int off = lane_off(u), cnt = c.n - off;
      if (cnt <= 0) continue;
      const bool vec = al && cnt >= 8;
      const int64_t idx = c.start + off;
      ld<TG>(c.t->ptr[0], idx, cnt, vec, g[u]);
      ld<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
      ld<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
    }
#pragma unroll
    for (int u = 0; u < kMTUnroll; ++u) {
      const int off = lane_off(u), cnt = c.n - off;
      if (cnt <= 0) continue;
      const bool vec = al && cnt >= 8;
      const int64_t idx = c.start + off;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float gi = g[u][i] * sc * inv_denom;
        if (a.mode == 0) gi = fmaf(a.wd, p[u][i], gi);
        m[u][i] = fmaf(a.beta1, m[u][i], beta3 * gi);
        float upd = m[u][i] / bc1;
        if (a.mode == 1) upd = fmaf(a.wd, p[u][i], upd);
        p[u][i] = fmaf(-lr, upd, p[u][i]);
      }
      st<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
      st<TP>(c.t->ptr[2], idx, cnt, vec, m[u]);
    }
  }
}

void mt_novograd(const MTLaunch& L, DType g, DType p, const NovoArgs& a, const float* v,
                 const int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((novograd_kernel<TG, TP>), mt_pgrid(L), dim3(kMTThreads), 0, st, L, a, v,
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
  const float sc = get_scale(a.scale);
  const float lr = lr_of(a.lr_ptr, a.lr);
  for (int ch = blockIdx.x; ch < L.nchunks; ch += gridDim.x) {
    const TileCtx c = tile_ctx(L, ch);
    const bool al = c.t->aligned;
    float g[kMTUnroll][8], p[kMTUnroll][8], h[kMTUnroll][8];
#pragma unroll
    for (int u = 0; u < kMTUnroll; ++u) {
      const int off = lane_off(u), cnt = c.n - off;
      if (cnt <= 0) continue;
      const bool vec = al && cnt >= 8;
      const int64_t idx = c.start + off;
      ld<TG>(c.t->ptr[0], idx, cnt, vec, g[u]);
      ld<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
      ld<TP>(c.t->ptr[2], idx, cnt, vec, h[u]);
    }
#pragma unroll
    for (int u = 0; u < kMTUnroll; ++u) {
      const int off = lane_off(u), cnt = c.n - off;
      if (cnt <= 0) continue;
      const bool vec = al && cnt >= 8;
      const int64_t idx = c.start + off;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float gi = g[u][i] * sc;
        if (a.mode == 0) gi = fmaf(a.wd, p[u][i], gi);
        h[u][i] = fmaf(gi, gi, h[u][i]);
        float upd = gi / (sqrtf(h[u][i]) + a.eps);
        if (a.mode == 1) upd = fmaf(a.wd, p[u][i], upd);
        p[u][i] = fmaf(-lr, upd, p[u][i]);
      }
      st<TP>(c.t->ptr[1], idx, cnt, vec, p[u]);
      st<TP>(c.t->ptr[2], idx, cnt, vec, h[u]);
    }
  }
}

void mt_adagrad(const MTLaunch& L, DType g, DType p, const AdagradArgs& a, const int* noop,
                hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(g, [&](auto tg) {
    dispatch1(p, [&](auto tp) {
      using TG = decltype(tg);
      using TP = decltype(tp);
      hipLaunchKernelGGL((adagrad_kernel<TG, TP>), mt_pgrid(L), dim3(kMTThreads), 0, st, L, a,
                         noop);
    });
  });
}

// --------------------------------------------------------------------------
int device_cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cus[dev] = n > 0 ? n : 256;
  }
  return cus[dev];
}


}  // namespace amd

