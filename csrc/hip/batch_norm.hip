// BatchNorm / SyncBatchNorm kernels for gfx950, NCHW and channels-last (NHWC).
//
// Behavioural spec: apex@f3a960f8 csrc/welford.cu:
// welford_mean_var(_c_last), welford_parallel, batchnorm_forward(_c_last) with
// optional +z and fused ReLU, reduce_bn(_c_last), batchnorm_backward(_c_last),
// relu_bw_c_last.
//
// MI355X design:
//  * every tensor is viewed as [outer, C, inner]: NHWC = [N*H*W, C, 1],
//    NCHW = [N, C, H*W];
//  * per-channel reductions are SPLIT over many workgroups (apex launches one
//    block per channel: 64 blocks for a C=64 layer on a 256-CU chip) and every
//    split writes a partial slab; a second tiny kernel sums the slabs in a fixed
//    order -> deterministic, no float atomics, no inter-workgroup hand-off;
//  * statistics use sums shifted by a per-channel sample value (the channel's
//    first element) so the one-pass sum / sum-of-squares does not cancel;
//  * channels-last: a lane owns 8 consecutive channels (one 16-byte bf16 load)
//    for every row it visits, so the per-channel constants and accumulators stay
//    in registers; NCHW: 16-byte loads along H*W when H*W % 8 == 0;
//  * forward apply fuses (x*scale + shift) [+ residual z] [ReLU]; backward fuses
//    the ReLU mask (recomputed from x, no saved activation) and emits dz for the
//    residual branch.
#include "amd_dev.h"
#include "amd_kernels.h"

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

struct BNGeom {
  int64_t outer, C, inner;
  int channel_last;
  bool vec;        // vector path usable
  int ctile;       // (NHWC) channel vectors per block
  int cblocks;     // (NHWC) grid.y
  int rows_iter;   // (NHWC) rows covered by one block iteration
  int splits;      // reduction splits (grid.x)
};

static BNGeom bn_geom(int64_t outer, int64_t C, int64_t inner, int channel_last, bool aligned) {
  BNGeom g;
  g.outer = outer;
  g.C = C;
  g.inner = inner;
  g.channel_last = channel_last;
  if (channel_last) {
    g.vec = aligned && (C % 8 == 0);
    int64_t cv = g.vec ? C / 8 : C;  // scalar path: one channel per thread
    g.ctile = (int)(cv < kBNThreads ? cv : kBNThreads);
    g.cblocks = (int)((cv + g.ctile - 1) / g.ctile);
    g.rows_iter = kBNThreads / g.ctile;
    int64_t rows = outer;
    int64_t want = (rows + (int64_t)g.rows_iter * 8 - 1) / ((int64_t)g.rows_iter * 8);
    int64_t cap = 1024 / g.cblocks;
    if (cap < 1) cap = 1;
    if (want > cap) want = cap;
    g.splits = (int)(want < 1 ? 1 : want);
  } else {
    g.vec = aligned && (inner % 8 == 0);
    g.ctile = g.cblocks = g.rows_iter = 0;
    int64_t per_ch = outer * inner;
    int64_t want = (2048 + C - 1) / C;
    int64_t maxs = (per_ch + 2047) / 2048;  // >= 2048 elements per split
    if (want > maxs) want = maxs;
    g.splits = (int)(want < 1 ? 1 : want);
  }
  return g;
}

// ============================================================================
// statistics: shifted sums per split -> slab [split][2][C]
// ============================================================================
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
    stats_nhwc(const T* __restrict__ x, int64_t M, int C, int ctile, int rows_iter, int vec,
               float* __restrict__ slab) {
  const int ci = threadIdx.x % ctile;
  const int ri = threadIdx.x / ctile;
  const int cv = blockIdx.y * ctile + ci;
  const int W = vec ? 8 : 1;
  const int c0 = cv * W;
  const bool active = ri < rows_iter && c0 < C;
  const int64_t per = (M + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  int64_t r1 = r0 + per;
  if (r1 > M) r1 = M;
  float k[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = s1[i] = s2[i] = 0.f;
  if (active) {
    if (vec) load8(x + c0, k);  // row 0 of the whole tensor: same shift in every split
    else k[0] = to_f32(x[c0]);
    // 4 rows in flight per thread (independent 16-B loads) before accumulating
    constexpr int U = 4;
    for (int64_t r = r0 + ri; r < r1; r += (int64_t)rows_iter * U) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = r + (int64_t)u * rows_iter;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[u][i] = k[i];  // contributes d = 0 when unused
        if (rr < r1) {
          if (vec) load8(x + rr * C + c0, v[u]);
          else v[u][0] = to_f32(x[rr * C + c0]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float d = v[u][i] - k[i];
          s1[i] += d;
          s2[i] = fmaf(d, d, s2[i]);
        }
    }
  }
  // combine the rows_iter row-groups of the block through LDS
  __shared__ float lds[2][kBNThreads * 8];
  if (threadIdx.x < rows_iter * ctile) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      lds[0][(ri * ctile + ci) * 8 + i] = s1[i];
      lds[1][(ri * ctile + ci) * 8 + i] = s2[i];
    }
  }
  __syncthreads();
  if (ri == 0 && c0 < C) {
    for (int r = 1; r < rows_iter; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s1[i] += lds[0][(r * ctile + ci) * 8 + i];
        s2[i] += lds[1][(r * ctile + ci) * 8 + i];
      }
    }
    float* o = slab + (size_t)blockIdx.x * 2 * C;
    for (int i = 0; i < W; ++i) {
      o[c0 + i] = s1[i];
      o[C + c0 + i] = s2[i];
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kBNThreads)
    stats_nchw(const T* __restrict__ x, int64_t N, int C, int64_t HW, int vec,
               float* __restrict__ slab) {
  __shared__ float scratch[kBNThreads / kWave];
  const int c = blockIdx.y;
  const int64_t L = N * HW;  // elements of this channel
  const float k = to_f32(x[(int64_t)c * HW]);
  float s1 = 0.f, s2 = 0.f;
  if (vec) {
    const int64_t LV = L / 8;
    const int64_t per = (LV + gridDim.x - 1) / gridDim.x;
    const int64_t v0 = (int64_t)blockIdx.x * per;
    int64_t v1 = v0 + per;
    if (v1 > LV) v1 = LV;
    for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      int64_t e = v * 8;
      int64_t n = e / HW, hw = e - n * HW;
      float a[8];
      load8(x + (n * C + c) * HW + hw, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = a[i] - k;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
    }
  } else {
    const int64_t per = (L + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per;
    int64_t e1 = e0 + per;
    if (e1 > L) e1 = L;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      int64_t n = e / HW, hw = e - n * HW;
      float d = to_f32(x[(n * C + c) * HW + hw]) - k;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
  }
  s1 = block_sum(s1, scratch);
  s2 = block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    slab[(size_t)blockIdx.x * 2 * C + c] = s1;
    slab[(size_t)blockIdx.x * 2 * C + C + c] = s2;
  }
}

// Sum the [split][2][C] slab over splits for 8 channels per workgroup: every
// thread accumulates a strided subset of the splits (16 partial sums in
// registers), then wave64 xor-shuffles + one LDS pass across the 4 waves.  A
// channel's splits are thereby read by 256 threads in parallel (the naive
// thread-per-channel loop serialised 1024 dependent loads per channel).
constexpr int kFinCh = 8;
// Result: out[k] = sum of first-half partials of channel c0+k, out[kFinCh+k] =
// second half; valid for every thread after the call.
__device__ __forceinline__ void slab_sum8(const float* __restrict__ slab, int splits, int C, int c0,
                                          float* out /* __shared__ [2*kFinCh] */) {
  __shared__ float red[kBNThreads / kWave][2 * kFinCh];
  float a[2 * kFinCh];
#pragma unroll
  for (int k = 0; k < 2 * kFinCh; ++k) a[k] = 0.f;
  for (int s = threadIdx.x; s < splits; s += blockDim.x) {
    const float* row = slab + (size_t)s * 2 * C;
#pragma unroll
    for (int k = 0; k < kFinCh; ++k) {
      if (c0 + k < C) {
        a[k] += row[c0 + k];
        a[kFinCh + k] += row[C + c0 + k];
      }
    }
  }
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < 2 * kFinCh; ++k) a[k] = wave_sum(a[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 2 * kFinCh; ++k) red[wid][k] = a[k];
  }
  __syncthreads();
  if (threadIdx.x < 2 * kFinCh) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) t += red[w][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// sum slabs -> mean, var_biased (per channel); shift re-read from x
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
    stats_finalize(const T* __restrict__ x, const float* __restrict__ slab, int splits, int C,
                   int64_t count, int64_t shift_stride, float* __restrict__ mean,
                   float* __restrict__ var) {
  __shared__ float sums[2 * kFinCh];
  const int c0 = blockIdx.x * kFinCh;
  slab_sum8(slab, splits, C, c0, sums);
  const int k = threadIdx.x;
  if (k < kFinCh && c0 + k < C) {
    const int c = c0 + k;
    const float shift = to_f32(x[(int64_t)c * shift_stride]);
    double m = (double)sums[k] / (double)count;
    double v = (double)sums[kFinCh + k] / (double)count - m * m;
    mean[c] = (float)(shift + m);
    var[c] = (float)(v > 0.0 ? v : 0.0);
  }
}

static inline dim3 fin_grid(int64_t C) { return dim3((unsigned)((C + kFinCh - 1) / kFinCh)); }

int64_t bn_stats_workspace(int64_t outer, int64_t C, int64_t inner, int channel_last) {
  BNGeom g = bn_geom(outer, C, inner, channel_last, true);
  BNGeom g2 = bn_geom(outer, C, inner, channel_last, false);
  int64_t s = g.splits > g2.splits ? g.splits : g2.splits;
  return s * 2 * C;
}

void bn_local_stats(const void* x, DType tx, int64_t outer, int64_t C, int64_t inner,
                    int channel_last, float* mean, float* var_biased, float* ws, hipStream_t st) {
  const int64_t count = outer * inner;
  if (count == 0 || C == 0) return;
  bool aligned = ((uintptr_t)x % 16) == 0;
  BNGeom g = bn_geom(outer, C, inner, channel_last, aligned);
  bn_dispatch(tx, [&](auto t0) {
    using T = decltype(t0);
    const T* xp = static_cast<const T*>(x);
    if (channel_last) {
      hipLaunchKernelGGL((stats_nhwc<T>), dim3(g.splits, g.cblocks), dim3(kBNThreads), 0, st, xp,
                         outer, (int)C, g.ctile, g.rows_iter, g.vec ? 1 : 0, ws);
      hipLaunchKernelGGL((stats_finalize<T>), fin_grid(C), dim3(kBNThreads), 0, st, xp,
                         ws, g.splits, (int)C, count, (int64_t)1, mean, var_biased);
    } else {
      hipLaunchKernelGGL((stats_nchw<T>), dim3(g.splits, (unsigned)C), dim3(kBNThreads), 0, st, xp,
                         outer, (int)C, inner, g.vec ? 1 : 0, ws);
      hipLaunchKernelGGL((stats_finalize<T>), fin_grid(C), dim3(kBNThreads), 0, st, xp,
                         ws, g.splits, (int)C, count, inner, mean, var_biased);
    }
  });
}

// ============================================================================
// combine across ranks (Chan) + running statistics
// ============================================================================
template <typename TR>
__global__ void __launch_bounds__(256)
    combine_kernel(const float* __restrict__ means, const float* __restrict__ vars,
                   const float* __restrict__ counts, int world, int C, float eps, float momentum,
                   float* __restrict__ mean_out, float* __restrict__ invstd_out,
                   float* __restrict__ running_mean, TR* __restrict__ running_var,
                   float* __restrict__ var_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean = 0.f, m2 = 0.f, n = 0.f;
  for (int w = 0; w < world; ++w) {
    float nb = counts[w];
    welford_combine(mean, m2, n, means[(size_t)w * C + c], vars[(size_t)w * C + c] * nb, nb);
  }
  float var_b = n > 0.f ? m2 / n : 0.f;
  mean_out[c] = mean;
  invstd_out[c] = rsqrtf(var_b + eps);
  if (var_out) var_out[c] = var_b;
  if (running_mean) {
    float unb = n > 1.f ? m2 / (n - 1.f) : var_b;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    float rv = to_f32(running_var[c]);
    running_var[c] = from_f32<TR>((1.f - momentum) * rv + momentum * unb);
  }
}

void bn_combine_stats(const float* means, const float* vars, const float* counts, int world,
                      int64_t C, float eps, float momentum, float* mean_out, float* invstd_out,
                      float* running_mean, DType trm, void* running_var_any, float* var_out,
                      hipStream_t st) {
  (void)trm;
  hipLaunchKernelGGL((combine_kernel<float>), dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st,
                     means, vars, counts, world, (int)C, eps, momentum, mean_out, invstd_out,
                     running_mean, static_cast<float*>(running_var_any), var_out);
}

// ============================================================================
// apply: y = x*scale + shift [+ z] [relu]
// ============================================================================
__device__ __forceinline__ void chan_affine(const float* mean, const float* invstd, float w,
                                            float b, int c, float& sc, float& sh) {
  float is = invstd[c];
  sc = is * w;
  sh = b - mean[c] * sc;
}

template <typename T, typename TW>
__device__ __forceinline__ float wload(const TW* p, int c, float dflt) {
  return p ? to_f32(p[c]) : dflt;
}

template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    apply_nhwc(const T* __restrict__ x, const float* __restrict__ mean,
               const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
               const T* __restrict__ z, T* __restrict__ y, int64_t M, int C, int ctile,
               int rows_iter, int vec, int relu) {
  const int ci = threadIdx.x % ctile;
  const int ri = threadIdx.x / ctile;
  const int cv = blockIdx.y * ctile + ci;
  const int W = vec ? 8 : 1;
  const int c0 = cv * W;
  if (ri >= rows_iter || c0 >= C) return;
  float sc[8], sh[8];
  for (int i = 0; i < W; ++i)
    chan_affine(mean, invstd, wload<T, TW>(w, c0 + i, 1.f), wload<T, TW>(b, c0 + i, 0.f), c0 + i,
                sc[i], sh[i]);
  const int64_t stride = (int64_t)gridDim.x * rows_iter;
  for (int64_t r = (int64_t)blockIdx.x * rows_iter + ri; r < M; r += stride) {
    float v[8], zz[8];
    if (vec) {
      load8(x + r * C + c0, v);
      if (z) load8(z + r * C + c0, zz);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = fmaf(v[i], sc[i], sh[i]);
        if (z) o += zz[i];
        v[i] = relu ? fmaxf(o, 0.f) : o;
      }
      store8(y + r * C + c0, v);
    } else {
      float o = fmaf(to_f32(x[r * C + c0]), sc[0], sh[0]);
      if (z) o += to_f32(z[r * C + c0]);
      y[r * C + c0] = from_f32<T>(relu ? fmaxf(o, 0.f) : o);
    }
  }
}

template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    apply_nchw(const T* __restrict__ x, const float* __restrict__ mean,
               const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
               const T* __restrict__ z, T* __restrict__ y, int64_t N, int C, int64_t HW, int vec,
               int relu) {
  const int64_t total = N * C * HW;
  const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
  if (vec) {
    const int64_t nv = total / 8;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gstride) {
      int64_t e = v * 8;
      int c = (int)((e / HW) % C);
      float sc, sh;
      chan_affine(mean, invstd, wload<T, TW>(w, c, 1.f), wload<T, TW>(b, c, 0.f), c, sc, sh);
      float a[8], zz[8];
      load8(x + e, a);
      if (z) load8(z + e, zz);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = fmaf(a[i], sc, sh);
        if (z) o += zz[i];
        a[i] = relu ? fmaxf(o, 0.f) : o;
      }
      store8(y + e, a);
    }
  } else {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gstride) {
      int c = (int)((e / HW) % C);
      float sc, sh;
      chan_affine(mean, invstd, wload<T, TW>(w, c, 1.f), wload<T, TW>(b, c, 0.f), c, sc, sh);
      float o = fmaf(to_f32(x[e]), sc, sh);
      if (z) o += to_f32(z[e]);
      y[e] = from_f32<T>(relu ? fmaxf(o, 0.f) : o);
    }
  }
}

static inline int elem_grid(int64_t work_items) {
  int64_t b = (work_items + kBNThreads - 1) / kBNThreads;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

static inline int nhwc_apply_grid(const BNGeom& g) {
  int64_t b = (g.outer + g.rows_iter - 1) / g.rows_iter;
  int64_t cap = 4096 / g.cblocks;
  if (cap < 1) cap = 1;
  if (b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

static bool all_aligned(std::initializer_list<const void*> ps) {
  for (const void* p : ps)
    if (p && ((uintptr_t)p % 16) != 0) return false;
  return true;
}

void bn_apply(const void* x, DType tx, const float* mean, const float* invstd,
              const void* weight, const void* bias, DType tw, const void* z, void* y,
              int64_t outer, int64_t C, int64_t inner, int channel_last, int relu,
              hipStream_t st) {
  if (outer * inner * C == 0) return;
  BNGeom g = bn_geom(outer, C, inner, channel_last, all_aligned({x, z, y}));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      const T* xp = static_cast<const T*>(x);
      const T* zp = static_cast<const T*>(z);
      T* yp = static_cast<T*>(y);
      const TW* wp = static_cast<const TW*>(weight);
      const TW* bp = static_cast<const TW*>(bias);
      if (channel_last) {
        hipLaunchKernelGGL((apply_nhwc<T, TW>), dim3(nhwc_apply_grid(g), g.cblocks),
                           dim3(kBNThreads), 0, st, xp, mean, invstd, wp, bp, zp, yp, outer,
                           (int)C, g.ctile, g.rows_iter, g.vec ? 1 : 0, relu);
      } else {
        int64_t items = g.vec ? outer * C * inner / 8 : outer * C * inner;
        hipLaunchKernelGGL((apply_nchw<T, TW>), dim3(elem_grid(items)), dim3(kBNThreads), 0, st, xp,
                           mean, invstd, wp, bp, zp, yp, outer, (int)C, inner, g.vec ? 1 : 0,
                           relu);
      }
    });
  });
}

// ============================================================================
// backward reduce: sum_dy', sum_dy'*(x-mean) per split -> slab, then finalize
// ============================================================================
// dy' = dy * [relu output > 0]; output recomputed as x*scale + shift (+ z)
template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    reduce_nhwc(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
                const float* __restrict__ invstd, const TW* __restrict__ w,
                const TW* __restrict__ b, const T* __restrict__ z, int relu, int64_t M, int C,
                int ctile, int rows_iter, int vec, float* __restrict__ slab) {
  const int ci = threadIdx.x % ctile;
  const int ri = threadIdx.x / ctile;
  const int cv = blockIdx.y * ctile + ci;
  const int W = vec ? 8 : 1;
  const int c0 = cv * W;
  const bool active = ri < rows_iter && c0 < C;
  const int64_t per = (M + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  int64_t r1 = r0 + per;
  if (r1 > M) r1 = M;
  float mu[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mu[i] = sc[i] = sh[i] = s1[i] = s2[i] = 0.f;
  if (active) {
    for (int i = 0; i < W; ++i) {
      mu[i] = mean[c0 + i];
      chan_affine(mean, invstd, wload<T, TW>(w, c0 + i, 1.f), wload<T, TW>(b, c0 + i, 0.f), c0 + i,
                  sc[i], sh[i]);
    }
    constexpr int U = 2;  // 2 rows x (x, dy[, z]) 16-B loads in flight per thread
    for (int64_t r = r0 + ri; r < r1; r += (int64_t)rows_iter * U) {
      float xv[U][8], dv[U][8], zv[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = r + (int64_t)u * rows_iter;
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[u][i] = dv[u][i] = zv[u][i] = 0.f;  // dy=0: no contribution
        if (rr < r1) {
          if (vec) {
            load8(x + rr * C + c0, xv[u]);
            load8(dy + rr * C + c0, dv[u]);
            if (relu && z) load8(z + rr * C + c0, zv[u]);
          } else {
            xv[u][0] = to_f32(x[rr * C + c0]);
            dv[u][0] = to_f32(dy[rr * C + c0]);
            if (relu && z) zv[u][0] = to_f32(z[rr * C + c0]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float d = dv[u][i];
          if (relu) {
            float o = fmaf(xv[u][i], sc[i], sh[i]);
            if (z) o += zv[u][i];
            d = o > 0.f ? d : 0.f;
          }
          s1[i] += d;
          s2[i] = fmaf(d, xv[u][i] - mu[i], s2[i]);
        }
    }
  }
  __shared__ float lds[2][kBNThreads * 8];
  if (threadIdx.x < rows_iter * ctile) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      lds[0][(ri * ctile + ci) * 8 + i] = s1[i];
      lds[1][(ri * ctile + ci) * 8 + i] = s2[i];
    }
  }
  __syncthreads();
  if (ri == 0 && c0 < C) {
    for (int r = 1; r < rows_iter; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s1[i] += lds[0][(r * ctile + ci) * 8 + i];
        s2[i] += lds[1][(r * ctile + ci) * 8 + i];
      }
    }
    float* o = slab + (size_t)blockIdx.x * 2 * C;
    for (int i = 0; i < W; ++i) {
      o[c0 + i] = s1[i];
      o[C + c0 + i] = s2[i];
    }
  }
}

template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    reduce_nchw(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
                const float* __restrict__ invstd, const TW* __restrict__ w,
                const TW* __restrict__ b, const T* __restrict__ z, int relu, int64_t N, int C,
                int64_t HW, int vec, float* __restrict__ slab) {
  __shared__ float scratch[kBNThreads / kWave];
  const int c = blockIdx.y;
  const int64_t L = N * HW;
  const float mu = mean[c];
  float sc, sh;
  chan_affine(mean, invstd, wload<T, TW>(w, c, 1.f), wload<T, TW>(b, c, 0.f), c, sc, sh);
  float s1 = 0.f, s2 = 0.f;
  if (vec) {
    const int64_t LV = L / 8;
    const int64_t per = (LV + gridDim.x - 1) / gridDim.x;
    const int64_t v0 = (int64_t)blockIdx.x * per;
    int64_t v1 = v0 + per;
    if (v1 > LV) v1 = LV;
    for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      int64_t e = v * 8;
      int64_t n = e / HW, hw = e - n * HW;
      int64_t off = (n * C + c) * HW + hw;
      float xv[8], dv[8], zv[8];
      load8(x + off, xv);
      load8(dy + off, dv);
      if (relu && z) load8(z + off, zv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = dv[i];
        if (relu) {
          float o = fmaf(xv[i], sc, sh);
          if (z) o += zv[i];
          d = o > 0.f ? d : 0.f;
        }
        s1 += d;
        s2 = fmaf(d, xv[i] - mu, s2);
      }
    }
  } else {
    const int64_t per = (L + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per;
    int64_t e1 = e0 + per;
    if (e1 > L) e1 = L;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      int64_t n = e / HW, hw = e - n * HW;
      int64_t off = (n * C + c) * HW + hw;
      float xv = to_f32(x[off]);
      float d = to_f32(dy[off]);
      if (relu) {
        float o = fmaf(xv, sc, sh);
        if (z) o += to_f32(z[off]);
        d = o > 0.f ? d : 0.f;
      }
      s1 += d;
      s2 = fmaf(d, xv - mu, s2);
    }
  }
  s1 = block_sum(s1, scratch);
  s2 = block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    slab[(size_t)blockIdx.x * 2 * C + c] = s1;
    slab[(size_t)blockIdx.x * 2 * C + C + c] = s2;
  }
}

template <typename TW>
__global__ void __launch_bounds__(kBNThreads)
    reduce_finalize(const float* __restrict__ slab, int splits, int C,
                    const float* __restrict__ invstd, float* __restrict__ sum_dy,
                    float* __restrict__ sum_dy_xmu, TW* __restrict__ gw, TW* __restrict__ gb) {
  __shared__ float sums[2 * kFinCh];
  const int c0 = blockIdx.x * kFinCh;
  slab_sum8(slab, splits, C, c0, sums);
  const int k = threadIdx.x;
  if (k < kFinCh && c0 + k < C) {
    const int c = c0 + k;
    const float s1 = sums[k], s2 = sums[kFinCh + k];
    sum_dy[c] = s1;
    sum_dy_xmu[c] = s2;
    if (gw) gw[c] = from_f32<TW>(s2 * invstd[c]);
    if (gb) gb[c] = from_f32<TW>(s1);
  }
}

void bn_reduce_grad(const void* dy, const void* x, DType tx, const float* mean,
                    const float* invstd, const void* weight, const void* bias, DType tw,
                    int relu, const void* z, int64_t outer, int64_t C, int64_t inner,
                    int channel_last, float* sum_dy, float* sum_dy_xmu, void* grad_weight,
                    void* grad_bias, float* ws, hipStream_t st) {
  if (outer * inner * C == 0) return;
  BNGeom g = bn_geom(outer, C, inner, channel_last, all_aligned({dy, x, z}));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      const T* dyp = static_cast<const T*>(dy);
      const T* xp = static_cast<const T*>(x);
      const T* zp = static_cast<const T*>(z);
      const TW* wp = static_cast<const TW*>(weight);
      const TW* bp = static_cast<const TW*>(bias);
      if (channel_last) {
        hipLaunchKernelGGL((reduce_nhwc<T, TW>), dim3(g.splits, g.cblocks), dim3(kBNThreads), 0, st,
                           dyp, xp, mean, invstd, wp, bp, zp, relu, outer, (int)C, g.ctile,
                           g.rows_iter, g.vec ? 1 : 0, ws);
      } else {
        hipLaunchKernelGGL((reduce_nchw<T, TW>), dim3(g.splits, (unsigned)C), dim3(kBNThreads), 0,
                           st, dyp, xp, mean, invstd, wp, bp, zp, relu, outer, (int)C, inner,
                           g.vec ? 1 : 0, ws);
      }
      hipLaunchKernelGGL((reduce_finalize<TW>), fin_grid(C), dim3(kBNThreads), 0, st,
                         ws, g.splits, (int)C, invstd, sum_dy, sum_dy_xmu,
                         static_cast<TW*>(grad_weight), static_cast<TW*>(grad_bias));
    });
  });
}

// ============================================================================
// backward elementwise
// ============================================================================
template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    bwd_nhwc(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
             const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
             const float* __restrict__ sum_dy, const float* __restrict__ sum_dy_xmu, float inv_n,
             int relu, const T* __restrict__ z, T* __restrict__ dx, T* __restrict__ dz, int64_t M,
             int C, int ctile, int rows_iter, int vec) {
  const int ci = threadIdx.x % ctile;
  const int ri = threadIdx.x / ctile;
  const int cv = blockIdx.y * ctile + ci;
  const int W = vec ? 8 : 1;
  const int c0 = cv * W;
  if (ri >= rows_iter || c0 >= C) return;
  float mu[8], sc[8], sh[8], k1[8], k2[8], k3[8];
  for (int i = 0; i < W; ++i) {
    const int c = c0 + i;
    const float wc = wload<T, TW>(w, c, 1.f);
    chan_affine(mean, invstd, wc, wload<T, TW>(b, c, 0.f), c, sc[i], sh[i]);
    const float is = invstd[c];
    mu[i] = mean[c];
    // dx = (dy' - mdy - (x-mu)*is^2*mdyx) * is * w  =  dy'*k1 + (x-mu)*k2 + k3
    const float mdy = sum_dy[c] * inv_n, mdyx = sum_dy_xmu[c] * inv_n;
    k1[i] = is * wc;
    k2[i] = -is * is * mdyx * is * wc;
    k3[i] = -mdy * is * wc;
  }
  const int64_t stride = (int64_t)gridDim.x * rows_iter;
  for (int64_t r = (int64_t)blockIdx.x * rows_iter + ri; r < M; r += stride) {
    const int64_t off = r * C + c0;
    if (vec) {
      float xv[8], dv[8], zv[8];
      load8(x + off, xv);
      load8(dy + off, dv);
      if (relu && z) load8(z + off, zv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = dv[i];
        if (relu) {
          float o = fmaf(xv[i], sc[i], sh[i]);
          if (z) o += zv[i];
          d = o > 0.f ? d : 0.f;
        }
        dv[i] = d;
        xv[i] = fmaf(d, k1[i], fmaf(xv[i] - mu[i], k2[i], k3[i]));
      }
      store8(dx + off, xv);
      if (dz) store8(dz + off, dv);
    } else {
      float xv = to_f32(x[off]);
      float d = to_f32(dy[off]);
      if (relu) {
        float o = fmaf(xv, sc[0], sh[0]);
        if (z) o += to_f32(z[off]);
        d = o > 0.f ? d : 0.f;
      }
      dx[off] = from_f32<T>(fmaf(d, k1[0], fmaf(xv - mu[0], k2[0], k3[0])));
      if (dz) dz[off] = from_f32<T>(d);
    }
  }
}

template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    bwd_nchw(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
             const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
             const float* __restrict__ sum_dy, const float* __restrict__ sum_dy_xmu, float inv_n,
             int relu, const T* __restrict__ z, T* __restrict__ dx, T* __restrict__ dz, int64_t N,
             int C, int64_t HW, int vec) {
  const int64_t total = N * C * HW;
  const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
  const int W = vec ? 8 : 1;
  const int64_t nitems = total / W;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < nitems; it += gstride) {
    const int64_t e = it * W;
    const int c = (int)((e / HW) % C);
    const float wc = wload<T, TW>(w, c, 1.f);
    float sc, sh;
    chan_affine(mean, invstd, wc, wload<T, TW>(b, c, 0.f), c, sc, sh);
    const float is = invstd[c], mu = mean[c];
    const float mdy = sum_dy[c] * inv_n, mdyx = sum_dy_xmu[c] * inv_n;
    const float k1 = is * wc, k2 = -is * is * mdyx * is * wc, k3 = -mdy * is * wc;
    float xv[8], dv[8], zv[8];
    if (vec) {
      load8(x + e, xv);
      load8(dy + e, dv);
      if (relu && z) load8(z + e, zv);
    } else {
      xv[0] = to_f32(x[e]);
      dv[0] = to_f32(dy[e]);
      if (relu && z) zv[0] = to_f32(z[e]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i >= W) break;
      float d = dv[i];
      if (relu) {
        float o = fmaf(xv[i], sc, sh);
        if (z) o += zv[i];
        d = o > 0.f ? d : 0.f;
      }
      dv[i] = d;
      xv[i] = fmaf(d, k1, fmaf(xv[i] - mu, k2, k3));
    }
    if (vec) {
      store8(dx + e, xv);
      if (dz) store8(dz + e, dv);
    } else {
      dx[e] = from_f32<T>(xv[0]);
      if (dz) dz[e] = from_f32<T>(dv[0]);
    }
  }
}

void bn_backward_elemt(const void* dy, const void* x, DType tx, const float* mean,
                       const float* invstd, const void* weight, const void* bias, DType tw,
                       const float* sum_dy, const float* sum_dy_xmu, float inv_count,
                       int relu, const void* z, void* dx, void* dz, int64_t outer, int64_t C,
                       int64_t inner, int channel_last, hipStream_t st) {
  if (outer * inner * C == 0) return;
  BNGeom g = bn_geom(outer, C, inner, channel_last, all_aligned({dy, x, z, dx, dz}));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      const T* dyp = static_cast<const T*>(dy);
      const T* xp = static_cast<const T*>(x);
      const T* zp = static_cast<const T*>(z);
      T* dxp = static_cast<T*>(dx);
      T* dzp = static_cast<T*>(dz);
      const TW* wp = static_cast<const TW*>(weight);
      const TW* bp = static_cast<const TW*>(bias);
      if (channel_last) {
        hipLaunchKernelGGL((bwd_nhwc<T, TW>), dim3(nhwc_apply_grid(g), g.cblocks), dim3(kBNThreads),
                           0, st, dyp, xp, mean, invstd, wp, bp, sum_dy, sum_dy_xmu, inv_count,
                           relu, zp, dxp, dzp, outer, (int)C, g.ctile, g.rows_iter,
                           g.vec ? 1 : 0);
      } else {
        int64_t items = g.vec ? outer * C * inner / 8 : outer * C * inner;
        hipLaunchKernelGGL((bwd_nchw<T, TW>), dim3(elem_grid(items)), dim3(kBNThreads), 0, st, dyp,
                           xp, mean, invstd, wp, bp, sum_dy, sum_dy_xmu, inv_count, relu, zp, dxp,
                           dzp, outer, (int)C, inner, g.vec ? 1 : 0);
      }
    });
  });
}

}  // namespace amd
