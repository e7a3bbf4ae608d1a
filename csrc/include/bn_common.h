// Shared pieces of the BatchNorm kernels (NCHW: batch_norm.hip, NHWC: bn_nhwc.hip).
#pragma once
#include "amd_dev.h"
#include "amd_kernels.h"

#include <type_traits>

namespace amd {

constexpr int kBNThreads = 256;

template <typename F>
static inline void bn_dispatch(DType a, F&& f) {
  switch (a) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    case DType::BF16: f(bf16_t{}); break;
    default: break;
  }
}

static inline bool all_aligned(std::initializer_list<const void*> ps) {
  for (const void* p : ps)
    if (p && ((uintptr_t)p % 16) != 0) return false;
  return true;
}

// y = x*sc + sh with sc = invstd*w, sh = b - mean*sc
__device__ __forceinline__ void chan_affine(const float* mean, const float* invstd, float w,
                                            float b, int c, float& sc, float& sh) {
  float is = invstd[c];
  sc = is * w;
  sh = b - mean[c] * sc;
}

template <typename TW>
__device__ __forceinline__ float wload(const TW* p, int c, float dflt) {
  return p ? to_f32(p[c]) : dflt;
}

// Sum a [split][2][C] partial slab over splits for CH channels per workgroup:
// every thread accumulates a strided subset of the splits, then wave64
// xor-shuffles + one LDS pass across the 4 waves (fixed order: deterministic).
// CH is picked per layer (fin_ch) so narrow layers still get >= 64 workgroups.
template <int CH>
__device__ __forceinline__ void slab_sum(const float* __restrict__ slab, int splits, int C, int c0,
                                         float* out /* __shared__ [2*CH] */) {
  __shared__ float red[kBNThreads / kWave][2 * CH];
  float a[2 * CH];
#pragma unroll
  for (int k = 0; k < 2 * CH; ++k) a[k] = 0.f;
  for (int s = threadIdx.x; s < splits; s += blockDim.x) {
    const float* row = slab + (size_t)s * 2 * C;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if (c0 + k < C) {
        a[k] += row[c0 + k];
        a[CH + k] += row[C + c0 + k];
      }
    }
  }
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < 2 * CH; ++k) a[k] = wave_sum(a[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 2 * CH; ++k) red[wid][k] = a[k];
  }
  __syncthreads();
  if (threadIdx.x < 2 * CH) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) t += red[w][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// Where the statistics go.  Plain mode: mean + biased var (for the SyncBN
// all_gather).  Local-training mode (invstd != nullptr): mean + invstd and, in
// the same kernel, the running-stat momentum update (unbiased var) and the
// module's num_batches_tracked += 1, replacing the separate combine / fill /
// counter launches of a local BatchNorm forward.
struct BNStatsOut {
  float* mean;
  float* var;             // biased var (plain mode) or nullptr
  float* invstd;          // local-training mode
  float* running_mean;    // optional (fp32)
  float* running_var;     // optional (fp32)
  long long* nbt;         // optional num_batches_tracked (int64)
  float eps, momentum;
  float* count_out = nullptr;  // optional: receives count_val (SyncBN packed stats)
  float count_val = 0.f;
};

// slab of shifted sums -> statistics; the shift is re-read from x
template <typename T, int CH>
__global__ void __launch_bounds__(kBNThreads)
    stats_finalize(const T* __restrict__ x, const float* __restrict__ slab, int splits, int C,
                   int64_t count, int64_t shift_stride, BNStatsOut out) {
  __shared__ float sums[2 * CH];
  const int c0 = blockIdx.x * CH;
  slab_sum<CH>(slab, splits, C, c0, sums);
  const int k = threadIdx.x;
  if (k < CH && c0 + k < C) {
    const int c = c0 + k;
    const float shift = to_f32(x[(int64_t)c * shift_stride]);
    double m = (double)sums[k] / (double)count;
    double v = (double)sums[CH + k] / (double)count - m * m;
    if (v < 0.0) v = 0.0;
    const float mean = (float)(shift + m);
    out.mean[c] = mean;
    if (out.var) out.var[c] = (float)v;
    if (out.invstd) out.invstd[c] = rsqrtf((float)v + out.eps);
    if (out.running_mean) {
      const double unb = count > 1 ? v * (double)count / (double)(count - 1) : v;
      out.running_mean[c] = (1.f - out.momentum) * out.running_mean[c] + out.momentum * mean;
      out.running_var[c] = (1.f - out.momentum) * out.running_var[c] + out.momentum * (float)unb;
    }
    if (out.nbt && c == 0) *out.nbt += 1;
    if (out.count_out && c == 0) *out.count_out = out.count_val;
  }
}

// slab of (sum dy', sum dy'*(x-mean)) -> sums + grad_weight/grad_bias
template <typename TW, int CH>
__global__ void __launch_bounds__(kBNThreads)
    reduce_finalize(const float* __restrict__ slab, int splits, int C,
                    const float* __restrict__ invstd, float* __restrict__ sum_dy,
                    float* __restrict__ sum_dy_xmu, TW* __restrict__ gw, TW* __restrict__ gb,
                    const float* __restrict__ sum_scale, int accum) {
  __shared__ float sums[2 * CH];
  const int c0 = blockIdx.x * CH;
  slab_sum<CH>(slab, splits, C, c0, sums);
  const int k = threadIdx.x;
  if (k < CH && c0 + k < C) {
    const int c = c0 + k;
    const float s1 = sums[k], s2 = sums[CH + k];
    // SyncBN: the sums leave pre-divided by the global count (device scalar), so the
    // all_reduce of them yields the means directly; dgamma / dbeta stay local sums
    const float sc = sum_scale ? *sum_scale : 1.f;
    sum_dy[c] = s1 * sc;
    sum_dy_xmu[c] = s2 * sc;
    // accum: add into existing gradients (DDP bucket views) instead of overwriting
    if (gw) gw[c] = from_f32<TW>(s2 * invstd[c] + (accum ? to_f32(gw[c]) : 0.f));
    if (gb) gb[c] = from_f32<TW>(s1 + (accum ? to_f32(gb[c]) : 0.f));
  }
}

// channels per finalize workgroup: keep >= ~128 workgroups where C allows
static inline int fin_ch(int64_t C) { return C >= 1024 ? 8 : C >= 512 ? 4 : C >= 256 ? 2 : 1; }

template <typename F>
static inline void fin_dispatch(int64_t C, F&& f) {
  switch (fin_ch(C)) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    default: f(std::integral_constant<int, 8>{}); break;
  }
}

template <typename T>
static inline void launch_stats_finalize(const T* x, const float* slab, int splits, int64_t C,
                                         int64_t count, int64_t shift_stride,
                                         const BNStatsOut& out, hipStream_t st) {
  fin_dispatch(C, [&](auto ch) {
    constexpr int CH = decltype(ch)::value;
    hipLaunchKernelGGL((stats_finalize<T, CH>), dim3((unsigned)((C + CH - 1) / CH)),
                       dim3(kBNThreads), 0, st, x, slab, splits, (int)C, count, shift_stride,
                       out);
  });
}

template <typename TW>
static inline void launch_reduce_finalize(const float* slab, int splits, int64_t C,
                                          const float* invstd, float* sum_dy, float* sum_dy_xmu,
                                          TW* gw, TW* gb, hipStream_t st,
                                          const float* sum_scale = nullptr) {
  fin_dispatch(C, [&](auto ch) {
    constexpr int CH = decltype(ch)::value;
    hipLaunchKernelGGL((reduce_finalize<TW, CH>), dim3((unsigned)((C + CH - 1) / CH)),
                       dim3(kBNThreads), 0, st, slab, splits, (int)C, invstd, sum_dy, sum_dy_xmu,
                       gw, gb, sum_scale, bn_grad_accumulate() ? 1 : 0);
  });
}

// ---- NHWC launchers (bn_nhwc.hip) -------------------------------------------
// Grid sizing knobs (rows per thread, block caps/floors); settable at run time
// for tuning sweeps (tools/microbench.py bn-tune).
// Defaults from the ResNet-50-weighted sweep on MI355X (profiles/bn_tune.txt):
// reductions -8 %, elementwise passes -18 % vs the first sizing (32/2048, 4/8192).
struct BNTuning {
  // red_rpt 64 -> 32 and elem_rpt 16 -> 8 at the end of round 4, once the elementwise
  // passes stopped computing channel constants per thread (a cheaper prologue favours
  // more, shorter workgroups): ResNet-50 same-box pairs +0.3 .. +0.9 % (profiles/r4/y,
  // profiles/r4/z; docs/PERF.md)
  int red_rpt = 32, red_cap = 1024, red_min = 512;
  int elem_rpt = 8, elem_cap = 16384, elem_min = 0;
  bool elem_auto = false;  // per-shape elem_rpt rule (bn_nhwc.hip elem_rpt_for), opt-in
};
BNTuning& bn_tuning();
int64_t nhwc_splits(int64_t M, int64_t C, bool vec);
// statistics from a channel-major slab of per-tile shifted sums [2][C][S] written by a
// producer kernel's epilogue (conv_igemm.hip); shift may be null (0)
void bn_stats_from_slab(const float* slab, int S, int64_t C, int64_t count, const float* shift,
                        const BNStatsOut& out, hipStream_t st);
void nhwc_stats(const void* x, DType tx, int64_t M, int64_t C, const BNStatsOut& out, float* ws,
                hipStream_t st);
// rmask: optional ReLU bitmask [M][C/8] (apply writes it when the VEC path runs,
// reduce / backward read it instead of recomputing the ReLU condition from z)
void nhwc_apply(const void* x, DType tx, const float* mean, const float* invstd, const void* w,
                const void* b, DType tw, const void* z, uint8_t* rmask, void* y, int64_t M,
                int64_t C, int relu, hipStream_t st);
void nhwc_reduce(const void* dy, const void* x, DType tx, const float* mean, const float* invstd,
                 const void* w, const void* b, DType tw, int relu, const void* z,
                 const uint8_t* rmask, int64_t M, int64_t C, float* sum_dy, float* sum_dy_xmu,
                 void* gw, void* gb, float* ws, hipStream_t st, const float* sum_scale = nullptr);
void nhwc_backward(const void* dy, const void* x, DType tx, const float* mean,
                   const float* invstd, const void* w, const void* b, DType tw,
                   const float* sum_dy, const float* sum_dy_xmu, float inv_count, int relu,
                   const void* z, const uint8_t* rmask, void* dx, void* dz, int64_t M, int64_t C,
                   hipStream_t st);

}  // namespace amd
