// Fused LayerNorm / RMSNorm forward + backward for gfx950.
//
// Behavioural spec: apex@f3a960f8 csrc/layer_norm_cuda_kernel.cu (SURVEY.md
// N-13a..d): forward(input, normalized_shape, eps) -> (out, mean, invvar),
// *_affine variants, backward -> dinput (+ dgamma, dbeta).
//
// MI355X design (not a port of apex's (32,4)-thread warp tiling):
//  * one ROW PER WAVE64: a row of n2 <= 2048 is held in registers as VPT
//    16-byte vectors per lane (n2 = 1024 bf16 -> 2 x 16 B per lane); mean and
//    variance are a two-pass register computation + xor-shuffle reductions, no
//    LDS, no Welford divisions;
//  * the backward kernel computes dx AND accumulates dgamma/dbeta partials in
//    the same pass: a lane owns the same 8*VPT columns for every row its wave
//    visits, so the column sums stay in registers across rows; one LDS combine
//    per block then a deterministic column-sum kernel (no float atomics);
//  * a generic block-per-row path covers odd widths / unaligned rows.
#include <type_traits>

#include <cstdlib>

#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

constexpr int kLNThreads = 256;
constexpr int kLNWaves = kLNThreads / kWave;

template <typename F>
static inline void ln_dispatch(DType a, F&& f) {
  switch (a) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    case DType::BF16: f(bf16_t{}); break;
    default: break;
  }
}

// Sublayer-output type of the fused residual LayerNorm: the LN input's own type,
// or (fp32 residual stream under amp O1) the F16 / BF16 type the GEMM produced,
// read and written directly so no cast kernel runs either way.
template <typename T, typename F>
static inline void ln_fuse_h_dispatch(int th, F&& f) {
  if constexpr (std::is_same<T, float>::value) {
    if (th == (int)DType::F16) return f(half_t{});
    if (th == (int)DType::BF16) return f(bf16_t{});
  }
  f(T{});
}
// LN output / its gradient: T, or the 16-bit sublayer type when fu.ty is set
template <typename T, typename TH, typename F>
static inline void ln_fuse_y_dispatch(int ty, F&& f) {
  if constexpr (!std::is_same<T, TH>::value) {
    if (ty >= 0) return f(TH{});
  }
  f(T{});
}

// Residual + dropout fused into the LayerNorm (BERT post-LN / GPT-2 pre-LN
// sublayer joins): forward s = x + keep*h*scale, y = LN(s); backward
// ds = LN'(dy) + ds_ext, dh = keep*ds*scale.  The keep bits are a counter hash of
// (seed, flat element index) regenerated in the backward: no mask tensor.

__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// keep bits of the 8 consecutive elements starting at flat index e (e % 8 == 0)
__device__ __forceinline__ uint32_t drop_keep8(uint32_t seed, uint32_t thresh, int64_t e) {
  if (thresh == 0) return 0xFFu;
  const uint32_t base = drop_mix(seed ^ drop_mix((uint32_t)(e >> 3) ^ ((uint32_t)(e >> 35) * 0x9E3779B1u)));
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) bits |= (drop_mix(base + (uint32_t)i * 0x9E3779B9u) >= thresh ? 1u : 0u) << i;
  return bits;
}

// ---------------------------------------------------------------- forward (fast)
// constant sources for the branch-free loads of the fast LayerNorm kernels (absent gamma / beta / dres)
__device__ const float g_ln_ones_f[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
__device__ const unsigned short g_ln_ones_bf16[8] = {0x3F80, 0x3F80, 0x3F80, 0x3F80,
                                                     0x3F80, 0x3F80, 0x3F80, 0x3F80};
__device__ const unsigned short g_ln_ones_f16[8] = {0x3C00, 0x3C00, 0x3C00, 0x3C00,
                                                    0x3C00, 0x3C00, 0x3C00, 0x3C00};
__device__ const float g_ln_zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
template <typename TW>
__device__ __forceinline__ const TW* ln_ones() {
  if constexpr (std::is_same<TW, float>::value) return g_ln_ones_f;
  else if constexpr (std::is_same<TW, bf16_t>::value) return reinterpret_cast<const TW*>(g_ln_ones_bf16);
  else return reinterpret_cast<const TW*>(g_ln_ones_f16);
}

template <typename T, typename TW, int VPT, bool FUSE = false, typename TH = T, typename TY = T>
__global__ void __launch_bounds__(kLNThreads)
    ln_fwd_fast(const T* __restrict__ x, const TW* __restrict__ gamma, const TW* __restrict__ beta,
                T* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ invvar_out,
                int64_t n1, int n2, float eps, int rms, LnFuse fu = LnFuse{}) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row0 = (int64_t)blockIdx.x * kLNWaves + threadIdx.x / kWave;
  const int64_t wstride = (int64_t)gridDim.x * kLNWaves;
  const float inv_n = 1.f / (float)n2;
  for (int64_t row = row0; row < n1; row += wstride) {
    const T* xr = x + row * n2;
    // the row's loads first, unconditionally (clamped column group): loads inside
    // `if (col < n2)` with the residual store in between made the compiler wait for the
    // previous group's store before each group's loads could be used (as in ln_bwd_fast)
    float v[VPT][8], hv[FUSE ? VPT : 1][8];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int col = (k * kWave + lane) * 8;
      const int cc = col < n2 ? col : 0;
      load8(xr + cc, v[k]);
      if constexpr (FUSE) load8(static_cast<const TH*>(fu.h) + row * n2 + cc, hv[k]);
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int col = (k * kWave + lane) * 8;
      if (col < n2) {
        if constexpr (FUSE) {
          // s = residual + keep * h / (1 - p); s is the LayerNorm input (and the
          // new residual stream), written once for the backward / next sublayer
          const uint32_t keep = drop_keep8(fu.seed, fu.thresh, row * n2 + col);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float t = v[k][i] + (((keep >> i) & 1u) ? hv[k][i] * fu.scale : 0.f);
            v[k][i] = to_f32(from_f32<T>(t));  // normalise s as stored, like the backward
          }
          store8(static_cast<T*>(fu.s) + row * n2 + col, v[k]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] = 0.f;
      }
    }
    float mu = 0.f;
    if (!rms) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < VPT; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[k][i];
      mu = wave_sum(s) * inv_n;
    }
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      int col = (k * kWave + lane) * 8;
      if (col < n2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float d = v[k][i] - mu;
          ss = fmaf(d, d, ss);
        }
      }
    }
    const float var = wave_sum(ss) * inv_n;
    const float iv = rsqrtf(var + eps);
    if (lane == 0) {
      if (mean_out) mean_out[row] = mu;
      invvar_out[row] = iv;
    }
    TY* yr = reinterpret_cast<TY*>(y) + row * n2;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      int col = (k * kWave + lane) * 8;
      if (col >= n2) continue;
      // gamma / beta through selected pointers (1 / 0 when absent): no branch joins
      float g[8], b[8];
      load8(gamma ? gamma + col : ln_ones<TW>(), g);
      load8(beta ? beta + col : reinterpret_cast<const TW*>(g_ln_zero), b);
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = fmaf((v[k][i] - mu) * iv, g[i], b[i]);
      store8(yr + col, o);
    }
  }
}

// ---------------------------------------------------------------- forward (generic)
template <typename T, typename TW>
__global__ void __launch_bounds__(kLNThreads)
    ln_fwd_generic(const T* __restrict__ x, const TW* __restrict__ gamma,
                   const TW* __restrict__ beta, T* __restrict__ y, float* __restrict__ mean_out,
                   float* __restrict__ invvar_out, int64_t n1, int n2, float eps, int rms) {
  __shared__ float scratch[kLNWaves];
  const int64_t row = blockIdx.x;
  if (row >= n1) return;
  const T* xr = x + row * n2;
  float mu = 0.f;
  if (!rms) {
    float s = 0.f;
    for (int c = threadIdx.x; c < n2; c += blockDim.x) s += to_f32(xr[c]);
    mu = block_sum(s, scratch) / (float)n2;
  }
  float ss = 0.f;
  for (int c = threadIdx.x; c < n2; c += blockDim.x) {
    float d = to_f32(xr[c]) - mu;
    ss = fmaf(d, d, ss);
  }
  const float var = block_sum(ss, scratch) / (float)n2;
  const float iv = rsqrtf(var + eps);
  if (threadIdx.x == 0) {
    if (mean_out) mean_out[row] = mu;
    invvar_out[row] = iv;
  }
  T* yr = y + row * n2;
  for (int c = threadIdx.x; c < n2; c += blockDim.x) {
    float xh = (to_f32(xr[c]) - mu) * iv;
    float o = gamma ? fmaf(xh, to_f32(gamma[c]), beta ? to_f32(beta[c]) : 0.f) : xh;
    yr[c] = from_f32<T>(o);
  }
}

static inline int ln_vpt(int64_t n2) { return (int)((n2 + 511) / 512); }

static inline bool ln_fast_ok(const void* x, const void* g, const void* b, const void* y,
                              int64_t n2) {
  auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p % 16) == 0; };
  return n2 % 8 == 0 && n2 <= 2048 && al(x) && al(g) && al(b) && al(y);
}

static inline int ln_grid(int64_t n1) {
  int64_t blocks = (n1 + kLNWaves - 1) / kLNWaves;
  // enough waves to fill 256 CUs several times over; rows loop beyond that
  if (blocks > 8192) blocks = 8192;
  return (int)(blocks > 0 ? blocks : 1);
}

bool layer_norm_fused_ok(const void* x, const void* h, const void* s, const void* gamma,
                         const void* beta, const void* y, int64_t n2) {
  auto al = [](const void* p) { return ((uintptr_t)p % 16) == 0; };
  return ln_fast_ok(x, gamma, beta, y, n2) && al(h) && al(s);
}

void layer_norm_fwd(const void* x, DType tx, const void* gamma, const void* beta, DType tw,
                    void* y, float* mean, float* invvar, int64_t n1, int64_t n2, float eps,
                    int rms, hipStream_t st, const LnFuse* fuse) {
  if (n1 == 0 || n2 == 0) return;
  ln_dispatch(tx, [&](auto t0) {
    ln_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      const T* xp = static_cast<const T*>(x);
      const TW* gp = static_cast<const TW*>(gamma);
      const TW* bp = static_cast<const TW*>(beta);
      T* yp = static_cast<T*>(y);
      if (fuse) {  // caller checked layer_norm_fused_ok
        dim3 grid(ln_grid(n1)), block(kLNThreads);
        auto launch = [&](auto h0) {
          using TH = decltype(h0);
          ln_fuse_y_dispatch<T, TH>(fuse->ty, [&](auto y0) {
          using TY = decltype(y0);
          switch (ln_vpt(n2)) {
            case 1: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 1, true, TH, TY>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms, *fuse); break;
            case 2: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 2, true, TH, TY>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms, *fuse); break;
            case 3: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 3, true, TH, TY>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms, *fuse); break;
            default: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 4, true, TH, TY>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms, *fuse); break;
          }
          });
        };
        ln_fuse_h_dispatch<T>(fuse->th, launch);
      } else if (ln_fast_ok(x, gamma, beta, y, n2)) {
        int vpt = ln_vpt(n2);
        dim3 grid(ln_grid(n1)), block(kLNThreads);
        switch (vpt) {
          case 1: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 1>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms); break;
          case 2: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 2>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms); break;
          case 3: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 3>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms); break;
          default: hipLaunchKernelGGL((ln_fwd_fast<T, TW, 4>), grid, block, 0, st, xp, gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms); break;
        }
      } else {
        hipLaunchKernelGGL((ln_fwd_generic<T, TW>), dim3((unsigned)n1), dim3(kLNThreads), 0, st, xp,
                           gp, bp, yp, mean, invvar, n1, (int)n2, eps, rms);
      }
    });
  });
}

// ---------------------------------------------------------------- backward (fast, fused)
// part layout: [nblocks][R][n2]  (dgamma partial, dbeta partial[, dh partial]); R = 3 with
// HS (fused join: the column sums of dh = the producing dense layer's bias gradient, so
// that layer skips its own column-sum pass over dh)
template <typename T, typename TW, int VPT, bool FUSE = false, typename TH = T, typename TY = T,
          bool HS = false>
__global__ void __launch_bounds__(kLNThreads)
    ln_bwd_fast(const T* __restrict__ dy, const T* __restrict__ x, const TW* __restrict__ gamma,
                const float* __restrict__ mean, const float* __restrict__ invvar,
                T* __restrict__ dx, float* __restrict__ part, int64_t n1, int n2, int rms,
                int one = 0, LnFuse fu = LnFuse{}) {
  // [kLNWaves][R][n2] per-wave partial rows, or [R][n2] with `one` (A/B, off by default)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int R = HS ? 3 : 2;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int64_t row0 = (int64_t)blockIdx.x * kLNWaves + wid;
  const int64_t wstride = (int64_t)gridDim.x * kLNWaves;
  const float inv_n = 1.f / (float)n2;
  const bool want_part = part != nullptr;

  // Register budget (occupancy is what hides the load latency here: every wave walks
  // only a few rows): gamma is NOT kept across rows - it is loaded 8 columns at a
  // time where dg = dy*gamma is formed and dg overwrites dy; xhat overwrites x.
  // 142 -> ~100 VGPRs for the fp32 GPT-2 joins (3 -> 5 waves per SIMD).
  float adg[VPT][8], adb[VPT][8], adh[HS ? VPT : 1][8];
#pragma unroll
  for (int k = 0; k < VPT; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) adg[k][i] = adb[k][i] = 0.f;
  if constexpr (HS) {
#pragma unroll
    for (int k = 0; k < VPT; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) adh[k][i] = 0.f;
  }

  for (int64_t row = row0; row < n1; row += wstride) {
    const float mu = rms ? 0.f : mean[row];
    const float iv = invvar[row];
    // every load of the row first, unconditionally (clamped column, selected pointer for
    // an absent gamma / residual gradient): with `if (col < n2)`, `if (gamma ...)` and
    // `if (fu.dres)` around them the compiler waited vmcnt(0) after each group - about
    // five serial memory round trips per row (ISA of the round-5 build)
    float xv[VPT][8], dv[VPT][8], gv[VPT][8], ev[FUSE ? VPT : 1][8];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int col = (k * kWave + lane) * 8;
      const int cc = col < n2 ? col : 0;
      load8(x + row * n2 + cc, xv[k]);
      load8(reinterpret_cast<const TY*>(dy) + row * n2 + cc, dv[k]);
      load8(gamma ? gamma + cc : ln_ones<TW>(), gv[k]);
      if constexpr (FUSE) {
        load8(fu.dres ? static_cast<const T*>(fu.dres) + row * n2 + cc
                      : reinterpret_cast<const T*>(g_ln_zero), ev[k]);
      }
    }
    float s1 = 0.f, s2 = 0.f;  // sum(dy*g), sum(dy*g*xhat)
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const float* g = gv[k];
      // a column group past n2 read the clamped group 0: it contributes nothing (selected
      // here, after the loads landed - overwriting the load targets right after the
      // loads would make the compiler wait for them there)
      const float ok = (k * kWave + lane) * 8 < n2 ? 1.f : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) dv[k][i] *= ok;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (xv[k][i] - mu) * iv;
        xv[k][i] = xh;  // keep xhat
        if (want_part) {
          adg[k][i] = fmaf(dv[k][i], xh, adg[k][i]);
          adb[k][i] += dv[k][i];
        }
        const float dg = dv[k][i] * g[i];
        dv[k][i] = dg;  // keep dy*gamma
        s1 += dg;
        s2 = fmaf(dg, xh, s2);
      }
    }
    s1 = wave_sum(s1) * inv_n;
    s2 = wave_sum(s2) * inv_n;
    T* dxr = dx + row * n2;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      int col = (k * kWave + lane) * 8;
      if (col >= n2) continue;
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float t = rms ? (dv[k][i] - xv[k][i] * s2) : (dv[k][i] - s1 - xv[k][i] * s2);
        o[i] = t * iv;
      }
      if constexpr (FUSE) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += ev[k][i];  // zeros without a residual gradient
        const uint32_t keep = drop_keep8(fu.seed, fu.thresh, row * n2 + col);
        float hd[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) hd[i] = ((keep >> i) & 1u) ? o[i] * fu.scale : 0.f;
        if constexpr (HS) {
          // the bias gradient sums dh as stored (rounded to TH), like a pass over dh would
#pragma unroll
          for (int i = 0; i < 8; ++i) adh[k][i] += to_f32(from_f32<TH>(hd[i]));
        }
        store8(static_cast<TH*>(fu.dh) + row * n2 + col, hd);
      }
      store8(dxr + col, o);
    }
  }

  if (!want_part) return;
  float* out = part + (size_t)blockIdx.x * R * n2;
  if (one) {
    // ONE [R][n2] LDS row set, the waves adding in turn (wave 0 first: the same order, hence
    // bits, as the per-wave rows below).  Meant to lift the LDS limit of the fp32 GPT-2
    // join (48 KB per block: 3 blocks per CU, below the 5 its registers allow); measured
    // slower end to end (GPT-2-medium 262 vs 264 k tok/s, BERT-large 700.6 vs 705.2 seq/s
    // same box, profiles/r6/ln_ab/), so off by default (layer_norm_bwd_one_row)
#pragma unroll
    for (int w = 0; w < kLNWaves; ++w) {
      if (wid == w) {
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
          int col = (k * kWave + lane) * 8;
          if (col >= n2) continue;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            float* c = lds + col + i;
            c[0] = (w == 0 ? 0.f : c[0]) + adg[k][i];
            c[n2] = (w == 0 ? 0.f : c[n2]) + adb[k][i];
            if constexpr (HS) c[2 * n2] = (w == 0 ? 0.f : c[2 * n2]) + adh[k][i];
          }
        }
      }
      __syncthreads();
    }
    for (int c = threadIdx.x; c < R * n2; c += blockDim.x) out[c] = 0.f + lds[c];
    return;
  }
  // combine the block's waves in LDS, then one partial row pair per block
  float* my = lds + (size_t)wid * R * n2;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    int col = (k * kWave + lane) * 8;
    if (col >= n2) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      my[col + i] = adg[k][i];
      my[n2 + col + i] = adb[k][i];
      if constexpr (HS) my[2 * n2 + col + i] = adh[k][i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < R * n2; c += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kLNWaves; ++w) s += lds[(size_t)w * R * n2 + c];
    out[c] = s;
  }
}

// ---------------------------------------------------------------- backward (generic)
template <typename T, typename TW>
__global__ void __launch_bounds__(kLNThreads)
    ln_bwd_dx_generic(const T* __restrict__ dy, const T* __restrict__ x,
                      const TW* __restrict__ gamma, const float* __restrict__ mean,
                      const float* __restrict__ invvar, T* __restrict__ dx, int64_t n1, int n2,
                      int rms) {
  __shared__ float scratch[kLNWaves];
  const int64_t row = blockIdx.x;
  if (row >= n1) return;
  const float mu = rms ? 0.f : mean[row];
  const float iv = invvar[row];
  const T* xr = x + row * n2;
  const T* dr = dy + row * n2;
  float s1 = 0.f, s2 = 0.f;
  for (int c = threadIdx.x; c < n2; c += blockDim.x) {
    float xh = (to_f32(xr[c]) - mu) * iv;
    float dg = to_f32(dr[c]) * (gamma ? to_f32(gamma[c]) : 1.f);
    s1 += dg;
    s2 = fmaf(dg, xh, s2);
  }
  s1 = block_sum(s1, scratch) / (float)n2;
  s2 = block_sum(s2, scratch) / (float)n2;
  for (int c = threadIdx.x; c < n2; c += blockDim.x) {
    float xh = (to_f32(xr[c]) - mu) * iv;
    float dg = to_f32(dr[c]) * (gamma ? to_f32(gamma[c]) : 1.f);
    float t = rms ? (dg - xh * s2) : (dg - s1 - xh * s2);
    dx[row * n2 + c] = from_f32<T>(t * iv);
  }
}

// column partials for the generic path: grid (ceil(n2/256), nparts)
template <typename T>
__global__ void __launch_bounds__(kLNThreads)
    ln_bwd_colpart_generic(const T* __restrict__ dy, const T* __restrict__ x,
                           const float* __restrict__ mean, const float* __restrict__ invvar,
                           float* __restrict__ part, int64_t n1, int n2, int rows_per_part,
                           int rms) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n2) return;
  int64_t r0 = (int64_t)blockIdx.y * rows_per_part;
  int64_t r1 = r0 + rows_per_part;
  if (r1 > n1) r1 = n1;
  float ag = 0.f, ab = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    float xh = (to_f32(x[r * n2 + c]) - (rms ? 0.f : mean[r])) * invvar[r];
    float d = to_f32(dy[r * n2 + c]);
    ag = fmaf(d, xh, ag);
    ab += d;
  }
  part[(size_t)blockIdx.y * 2 * n2 + c] = ag;
  part[(size_t)blockIdx.y * 2 * n2 + n2 + c] = ab;
}

// sum nparts partial rows -> dgamma, dbeta (TW); fixed order -> deterministic.
// A partial row is [dgamma(n2) | dbeta(n2) (| dh sums(n2))] = R*n2 contiguous floats.  Block =
// 8 column lanes x 32 row lanes; a lane owns 4 adjacent columns (one 16-byte
// load per partial row when n2 is even), the 32 row lanes stride over the
// partials and are combined through LDS.  Grid = ceil(2*n2 / 32) blocks.
constexpr int kCSColLanes = 8, kCSRowLanes = 32, kCSCols = 4 * kCSColLanes;

template <typename TW, bool VEC4>
__global__ void __launch_bounds__(256)
    ln_bwd_colsum(const float* __restrict__ part, int nparts, int n2, TW* __restrict__ dgamma,
                  TW* __restrict__ dbeta, TW* __restrict__ dhsum = nullptr, int R = 2) {
  __shared__ float4 red[kCSRowLanes][kCSColLanes];
  const int cl = threadIdx.x % kCSColLanes;
  const int rl = threadIdx.x / kCSColLanes;
  const int width = R * n2;
  const int c0 = blockIdx.x * kCSCols + cl * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < width) {
    if (VEC4) {
      const float* base = part + c0;
      int p = rl;
      // four loads in flight (two left ~16 dependent L2 round trips per lane at 1,024
      // partial rows: 8-14 us per call in the BERT / GPT-2 steps)
      for (; p + 3 * kCSRowLanes < nparts; p += 4 * kCSRowLanes) {
        float4 a = *reinterpret_cast<const float4*>(base + (size_t)p * width);
        float4 b = *reinterpret_cast<const float4*>(base + (size_t)(p + kCSRowLanes) * width);
        float4 c = *reinterpret_cast<const float4*>(base + (size_t)(p + 2 * kCSRowLanes) * width);
        float4 d = *reinterpret_cast<const float4*>(base + (size_t)(p + 3 * kCSRowLanes) * width);
        acc.x += (a.x + b.x) + (c.x + d.x); acc.y += (a.y + b.y) + (c.y + d.y);
        acc.z += (a.z + b.z) + (c.z + d.z); acc.w += (a.w + b.w) + (c.w + d.w);
      }
      for (; p < nparts; p += kCSRowLanes) {
        float4 a = *reinterpret_cast<const float4*>(base + (size_t)p * width);
        acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
      }
    } else {
      for (int p = rl; p < nparts; p += kCSRowLanes) {
        const float* r = part + (size_t)p * width + c0;
        acc.x += r[0];
        if (c0 + 1 < width) acc.y += r[1];
        if (c0 + 2 < width) acc.z += r[2];
        if (c0 + 3 < width) acc.w += r[3];
      }
    }
  }
  red[rl][cl] = acc;
  __syncthreads();
  for (int h = kCSRowLanes / 2; h > 0; h >>= 1) {
    if (rl < h) {
      float4 o = red[rl + h][cl];
      float4& m = red[rl][cl];
      m.x += o.x; m.y += o.y; m.z += o.z; m.w += o.w;
    }
    __syncthreads();
  }
  if (rl == 0 && c0 < width) {
    float v[4] = {red[0][cl].x, red[0][cl].y, red[0][cl].z, red[0][cl].w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c = c0 + i;
      if (c >= width) break;
      if (c < n2) {
        if (dgamma) dgamma[c] = from_f32<TW>(v[i]);
      } else if (c < 2 * n2) {
        if (dbeta) dbeta[c - n2] = from_f32<TW>(v[i]);
      } else if (dhsum) {
        dhsum[c - 2 * n2] = from_f32<TW>(v[i]);
      }
    }
  }
}

// fast backward grid: at most 1024 blocks x 4 waves walking rows (256 with a row of load
// lookahead measured 126 vs 77 us per GPT-2 join - occupancy, not lookahead, hides the
// latency; a 512 / 2048 cap measured equal, profiles/r4/k/)
static inline int ln_bwd_block_cap() { return 1024; }

static inline int ln_bwd_blocks(int64_t n1) {
  int64_t b = (n1 + kLNWaves - 1) / kLNWaves;
  if (b > ln_bwd_block_cap()) b = ln_bwd_block_cap();
  return (int)(b > 0 ? b : 1);
}
static inline int ln_generic_parts(int64_t n1) {
  int64_t p = (n1 + 31) / 32;
  if (p > 512) p = 512;
  return (int)(p > 0 ? p : 1);
}

static int g_ln_one = 0;
void layer_norm_bwd_one_row(int on) { g_ln_one = on; }
bool layer_norm_bwd_one_row_on() { return g_ln_one != 0; }
static inline int64_t ln_bwd_lds_rows() { return g_ln_one ? 1 : kLNWaves; }

// the dh column sums need a third [kLNWaves][n2] LDS row: within the 64 KB of dynamic LDS
// a launch gets without a raised attribute (n2 <= 1365; any fast-path n2 with one row set)
bool layer_norm_bwd_hsum_ok(int64_t n2) {
  return ln_bwd_lds_rows() * 3 * n2 * (int64_t)sizeof(float) <= 65536;
}

int64_t layer_norm_bwd_workspace(int64_t n1, int64_t n2) {
  int64_t a = (int64_t)ln_bwd_blocks(n1) * 3 * n2;  // (3 rows: with the dh column sums)
  int64_t b = (int64_t)ln_generic_parts(n1) * 2 * n2;
  return a > b ? a : b;
}

void layer_norm_bwd(const void* dy, const void* x, DType tx, const void* gamma, DType tw,
                    const float* mean, const float* invvar, void* dx, void* dgamma, void* dbeta,
                    float* part, int64_t n1, int64_t n2, int rms, hipStream_t st,
                    const LnFuse* fuse) {
  if (n1 == 0 || n2 == 0) return;
  const bool want_wb = dgamma != nullptr || dbeta != nullptr;
  // the dh column sums ride on the dgamma / dbeta partials (fused join only)
  const int R = (fuse && fuse->dhsum && want_wb && layer_norm_bwd_hsum_ok(n2)) ? 3 : 2;
  ln_dispatch(tx, [&](auto t0) {
    ln_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      const T* dyp = static_cast<const T*>(dy);
      const T* xp = static_cast<const T*>(x);
      const TW* gp = static_cast<const TW*>(gamma);
      T* dxp = static_cast<T*>(dx);
      int nparts;
      if (fuse) {  // caller checked alignment / width (layer_norm_fused_ok + dy, dres, dh)
        int blocks = ln_bwd_blocks(n1);
        size_t lds = want_wb ? (size_t)ln_bwd_lds_rows() * R * n2 * sizeof(float) : 0;
        float* pp = want_wb ? part : nullptr;
        dim3 grid(blocks), block(kLNThreads);
        auto launch = [&](auto h0) {
          using TH = decltype(h0);
          ln_fuse_y_dispatch<T, TH>(fuse->ty, [&](auto y0) {
          using TY = decltype(y0);
          auto go = [&](auto hs0) {
            constexpr bool HS = decltype(hs0)::value;
            switch (ln_vpt(n2)) {
              case 1: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 1, true, TH, TY, HS>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one, *fuse); break;
              case 2: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 2, true, TH, TY, HS>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one, *fuse); break;
              case 3: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 3, true, TH, TY, HS>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one, *fuse); break;
              default: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 4, true, TH, TY, HS>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one, *fuse); break;
            }
          };
          if (R == 3) go(std::true_type{});
          else go(std::false_type{});
          });
        };
        ln_fuse_h_dispatch<T>(fuse->th, launch);
        nparts = blocks;
      } else if (ln_fast_ok(x, gamma, nullptr, dx, n2) && ((uintptr_t)dy % 16) == 0) {
        int vpt = ln_vpt(n2);
        int blocks = ln_bwd_blocks(n1);
        size_t lds = want_wb ? (size_t)ln_bwd_lds_rows() * 2 * n2 * sizeof(float) : 0;
        float* pp = want_wb ? part : nullptr;
        dim3 grid(blocks), block(kLNThreads);
        switch (vpt) {
          case 1: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 1>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one); break;
          case 2: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 2>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one); break;
          case 3: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 3>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one); break;
          default: hipLaunchKernelGGL((ln_bwd_fast<T, TW, 4>), grid, block, lds, st, dyp, xp, gp, mean, invvar, dxp, pp, n1, (int)n2, rms, g_ln_one); break;
        }
        nparts = blocks;
      } else {
        hipLaunchKernelGGL((ln_bwd_dx_generic<T, TW>), dim3((unsigned)n1), dim3(kLNThreads), 0, st,
                           dyp, xp, gp, mean, invvar, dxp, n1, (int)n2, rms);
        nparts = ln_generic_parts(n1);
        if (want_wb) {
          int rows_per_part = (int)((n1 + nparts - 1) / nparts);
          hipLaunchKernelGGL((ln_bwd_colpart_generic<T>), dim3((unsigned)((n2 + 255) / 256), nparts),
                             dim3(256), 0, st, dyp, xp, mean, invvar, part, n1, (int)n2,
                             rows_per_part, rms);
        }
      }
      if (want_wb) {
        TW* dhs = R == 3 ? static_cast<TW*>(fuse->dhsum) : nullptr;
        dim3 cgrid((unsigned)((R * n2 + kCSCols - 1) / kCSCols));
        if (n2 % 2 == 0 && ((uintptr_t)part % 16) == 0)
          hipLaunchKernelGGL((ln_bwd_colsum<TW, true>), cgrid, dim3(256), 0, st, part, nparts,
                             (int)n2, static_cast<TW*>(dgamma), static_cast<TW*>(dbeta), dhs, R);
        else
          hipLaunchKernelGGL((ln_bwd_colsum<TW, false>), cgrid, dim3(256), 0, st, part, nparts,
                             (int)n2, static_cast<TW*>(dgamma), static_cast<TW*>(dbeta), dhs, R);
      }
    });
  });
}

}  // namespace amd
