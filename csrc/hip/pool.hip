// Channels-last (NHWC) max pooling for gfx950 (ResNet stem: 3x3, stride 2, pad 1).
//
// Forward: a thread owns 8 consecutive channels (one 16-byte load per window
// tap, VEC path; scalar path for C % 8 != 0) of one output pixel, scans the
// window in (kh, kw) order keeping the FIRST maximum (NaN propagates, as torch),
// writes y and the winning tap index as one byte per element (kh*k + kw).
// BN variant (ResNet stem): the window values are relu(x * scale + shift) with the
// BatchNorm's per-channel affine applied on load - the BN + ReLU output is never
// written to HBM (saves one write + one read of the largest activation of the
// network); values are rounded to T before the comparison so ties and the
// chosen taps match pooling the materialised bf16 tensor.
// Backward is a gather, not a scatter: a thread owns 8 channels of one INPUT
// pixel and sums dy over the <= ceil(k/s)^2 output windows that cover it and
// picked it, so there are no atomics and every dx element is written once.
#include <cstdlib>

#include "amd_dev.h"
#include "amd_kernels.h"
#include "bn_common.h"

namespace amd {

namespace {

constexpr int kPoolThreads = 256;
constexpr int kPoolBNMaxC = 512;  // BN-fused stem max-pool: channels held in LDS

struct PoolBN {
  const float *mean, *invstd, *w, *b;  // fp32 [C]; w / b optional
};

template <typename T, bool VEC, bool BN>
__global__ void __launch_bounds__(kPoolThreads)
    maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx,
                  int N, int H, int W, int C, int OH, int OW, int k, int s, int p, PoolBN bn) {
  constexpr int V = VEC ? 8 : 1;
  const int CV = C / V;
  const int64_t total = (int64_t)N * OH * OW * CV;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    int64_t pix = t / CV;
    const int ow = (int)(pix % OW);
    pix /= OW;
    const int oh = (int)(pix % OH);
    const int n = (int)(pix / OH);
    float best[V];
    int arg[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      best[i] = -INFINITY;
      arg[i] = 0;
    }
    float sc[V], sh[V];
    if constexpr (BN) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = cv * V + i;
        sc[i] = bn.invstd[c] * (bn.w ? bn.w[c] : 1.f);
        sh[i] = (bn.b ? bn.b[c] : 0.f) - bn.mean[c] * sc[i];
      }
    }
    const int h0 = oh * s - p, w0 = ow * s - p;
    for (int kh = 0; kh < k; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= W) continue;
        const T* src = x + (((int64_t)n * H + h) * W + w) * C + cv * V;
        float v[V];
        if constexpr (VEC) load8(src, v);
        else v[0] = to_f32(src[0]);
        if constexpr (BN) {
#pragma unroll
          for (int i = 0; i < V; ++i) v[i] = to_f32(from_f32<T>(fmaxf(fmaf(v[i], sc[i], sh[i]), 0.f)));
        }
        const int tap = kh * k + kw;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          if (v[i] > best[i] || (v[i] != v[i] && best[i] == best[i])) {
            best[i] = v[i];
            arg[i] = tap;
          }
        }
      }
    }
    const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + cv * V;
    if constexpr (VEC) {
      store8(y + o, best);
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lo |= (uint32_t)(arg[i] & 0xff) << (8 * i);
        hi |= (uint32_t)(arg[i + 4] & 0xff) << (8 * i);
      }
      *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
    } else {
      y[o] = from_f32<T>(best[0]);
      idx[o] = (uint8_t)arg[0];
    }
  }
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(kPoolThreads)
    maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx,
                  int N, int H, int W, int C, int OH, int OW, int k, int s, int p) {
  constexpr int V = VEC ? 8 : 1;
  const int CV = C / V;
  const int64_t total = (int64_t)N * H * W * CV;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    int64_t pix = t / CV;
    const int w = (int)(pix % W);
    pix /= W;
    const int h = (int)(pix % H);
    const int n = (int)(pix / H);
    // output windows covering h: oh*s - p <= h <= oh*s - p + k - 1
    int oh0 = h + p - k + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + s - 1) / s;
    int oh1 = (h + p) / s;
    if (oh1 > OH - 1) oh1 = OH - 1;
    int ow0 = w + p - k + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + s - 1) / s;
    int ow1 = (w + p) / s;
    if (ow1 > OW - 1) ow1 = OW - 1;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = h - (oh * s - p);
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int tap = kh * k + (w - (ow * s - p));
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + cv * V;
        if constexpr (VEC) {
          const uint2 ii = *reinterpret_cast<const uint2*>(idx + o);
          float g[8];
          load8(dy + o, g);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const uint32_t word = i < 4 ? ii.x : ii.y;
            const int a = (int)((word >> (8 * (i & 3))) & 0xff);
            if (a == tap) acc[i] += g[i];
          }
        } else {
          if ((int)idx[o] == tap) acc[0] += to_f32(dy[o]);
        }
      }
    }
    const int64_t d = (((int64_t)n * H + h) * W + w) * C + cv * V;
    if constexpr (VEC) store8(dx + d, acc);
    else dx[d] = from_f32<T>(acc[0]);
  }
}

// ResNet stem specialisation (3x3, stride 2, pad 1, 8 channels per lane): every
// window tap (forward) / covering window (backward) is loaded up front with a
// clamped address and a validity flag, so a lane has all 9 (resp. 4 + 4) 16-byte
// loads in flight instead of a loop of dependent, branchy single loads.  Same tap
// order, tie / NaN rule and summation order as the generic kernels above.
typedef unsigned p_u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ void unpack8_any(const p_u32x4& u, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    typedef T t8 __attribute__((ext_vector_type(8)));
    const t8 a = __builtin_bit_cast(t8, u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
}

template <typename T, bool BN>
__global__ void __launch_bounds__(kPoolThreads)
    maxpool3s2_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int N,
                     int H, int W, int C, int OH, int OW, PoolBN bn) {
  static_assert(sizeof(T) == 2, "16-bit activations");
  const int CV = C / 8;
  // BN scale / shift of every channel, once per workgroup into LDS (C <= kPoolBNMaxC,
  // checked on the host): per thread they were 32+ scalar global loads next to the 9
  // 16-byte data loads
  __shared__ __attribute__((aligned(16))) float s_sc[BN ? kPoolBNMaxC : 1];
  __shared__ __attribute__((aligned(16))) float s_sh[BN ? kPoolBNMaxC : 1];
  if constexpr (BN) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float a = bn.invstd[c] * (bn.w ? bn.w[c] : 1.f);
      s_sc[c] = a;
      s_sh[c] = (bn.b ? bn.b[c] : 0.f) - bn.mean[c] * a;
    }
    __syncthreads();
  }
  const int64_t total = (int64_t)N * OH * OW * CV;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    int64_t pix = t / CV;
    const int ow = (int)(pix % OW);
    pix /= OW;
    const int oh = (int)(pix % OH);
    const int n = (int)(pix / OH);
    const int h0 = oh * 2 - 1, w0 = ow * 2 - 1;
    p_u32x4 raw[9];
    unsigned okm = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int h = h0 + kh, w = w0 + kw;
        const bool ok = h >= 0 && h < H && w >= 0 && w < W;
        const int hc = ok ? h : 0, wc = ok ? w : 0;
        okm |= (ok ? 1u : 0u) << (kh * 3 + kw);
        raw[kh * 3 + kw] = *reinterpret_cast<const p_u32x4*>(
            x + (((int64_t)n * H + hc) * W + wc) * C + cv * 8);
      }
    }
    float sc[8], sh[8];
    if constexpr (BN) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sc[i] = s_sc[cv * 8 + i];
        sh[i] = s_sh[cv * 8 + i];
      }
    }
    float best[8];
    int arg[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      best[i] = -INFINITY;
      arg[i] = 0;
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (!((okm >> tap) & 1u)) continue;
      float v[8];
      unpack8_any<T>(raw[tap], v);
      if constexpr (BN) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = to_f32(from_f32<T>(fmaxf(fmaf(v[i], sc[i], sh[i]), 0.f)));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (v[i] > best[i] || (v[i] != v[i] && best[i] == best[i])) {
          best[i] = v[i];
          arg[i] = tap;
        }
      }
    }
    const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + cv * 8;
    store8(y + o, best);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo |= (uint32_t)(arg[i] & 0xff) << (8 * i);
      hi |= (uint32_t)(arg[i + 4] & 0xff) << (8 * i);
    }
    *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
  }
}

// Backward, one thread per 2x2 input block (rows 2i, 2i+1 x cols 2j, 2j+1) x 8
// channels: the block is covered by outputs (i..i+1) x (j..j+1), so the 4 dy / 4 index
// loads of a thread serve 4 input pixels instead of 1 (the per-input form below issues
// 4x the loads for the same bytes).  Per input the contributions are summed in the
// per-input kernel's order ((oh, ow) row-major), so the two are bitwise equal.
//
// BNR (the fused stem's backward, C == 64): dx is the gradient of relu(BN(x)); the kernel
// also forms the BatchNorm-backward sums of the pre-ReLU gradient d = dx * (BN(x) > 0)
// (ReLU condition recomputed from x exactly as reduce_k does, d taken as the stored 16-bit
// dx): sum(d), sum(d * (x - mean)) per channel into a channel-major slab [2][64][gridDim.x]
// - the separate reduction pass over dx and x (822 MB at ResNet-50 bs 256) disappears; x
// is read here once instead.  A thread's channel group (t % 8) is fixed: the grid stride is
// a multiple of 8.
template <typename T, bool BNR = false>
__global__ void __launch_bounds__(kPoolThreads)
    maxpool3s2_bwd2_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                      T* __restrict__ dx, int N, int H, int W, int C, int OH, int OW,
                      const T* __restrict__ xin = nullptr, const float* __restrict__ mean = nullptr,
                      const float* __restrict__ invstd = nullptr,
                      const float* __restrict__ bw = nullptr, const float* __restrict__ bb = nullptr,
                      float* __restrict__ slab = nullptr) {
  static_assert(sizeof(T) == 2, "16-bit activations");
  const int CV = C / 8, BH = (H + 1) / 2, BW = (W + 1) / 2;
  const int64_t total = (int64_t)N * BH * BW * CV;
  float mu[8], sc[8], sh[8], s1[8], s2[8];
  if constexpr (BNR) {
    const int cg = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) % CV);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int ch = cg * 8 + c;
      mu[c] = mean[ch];
      chan_affine(mean, invstd, bw ? bw[ch] : 1.f, bb ? bb[ch] : 0.f, ch, sc[c], sh[c]);
      s1[c] = s2[c] = 0.f;
    }
  }
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    int64_t pix = t / CV;
    const int j = (int)(pix % BW);
    pix /= BW;
    const int i = (int)(pix % BH);
    const int n = (int)(pix / BH);
    // outputs (i + a, j + b), a, b in {0, 1}
    float g[4][8];
    uint32_t wd[4][2];
    bool ok[4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int q = a * 2 + b;
        ok[q] = i + a < OH && j + b < OW;
        const int64_t o = (((int64_t)n * OH + (ok[q] ? i + a : i)) * OW + (ok[q] ? j + b : j)) * C +
                          cv * 8;
        unpack8_any<T>(*reinterpret_cast<const p_u32x4*>(dy + o), g[q]);
        const uint2 w2 = *reinterpret_cast<const uint2*>(idx + o);
        wd[q][0] = w2.x;
        wd[q][1] = w2.y;
      }
    auto tap_of = [&](int q, int c) { return (int)((wd[q][c >> 2] >> (8 * (c & 3))) & 0xff); };
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int h = 2 * i + dh;
      if (h >= H) continue;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int w = 2 * j + dw;
        if (w >= W) continue;
        float acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = 0.f;
        // contributing outputs in (oh, ow) row-major order: even offset -> only a/b = 0
        // (tap 1); odd -> a/b = 0 (tap 2) then 1 (tap 0)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (a == 1 && dh == 0) continue;
          const int kh = dh == 0 ? 1 : (a == 0 ? 2 : 0);
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b == 1 && dw == 0) continue;
            const int kw = dw == 0 ? 1 : (b == 0 ? 2 : 0);
            const int q = a * 2 + b;
            if (!ok[q]) continue;
#pragma unroll
            for (int c = 0; c < 8; ++c)
              if (tap_of(q, c) == kh * 3 + kw) acc[c] += g[q][c];
          }
        }
        const int64_t o = (((int64_t)n * H + h) * W + w) * C + cv * 8;
        store8(dx + o, acc);
        if constexpr (BNR) {
          float xv[8];
          unpack8_any<T>(*reinterpret_cast<const p_u32x4*>(xin + o), xv);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float g = to_f32(from_f32<T>(acc[c]));  // as stored
            const float d = fmaf(xv[c], sc[c], sh[c]) > 0.f ? g : 0.f;
            s1[c] += d;
            s2[c] = fmaf(d, xv[c] - mu[c], s2[c]);
          }
        }
      }
    }
  }
  if constexpr (BNR) {
    // lanes sharing a channel group: t % 8 == lane % 8 -> xor 8, 16, 32; then the waves
    __shared__ float red[2][kPoolThreads / 64][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
      for (int m = 8; m < 64; m <<= 1) {
        s1[c] += __shfl_xor(s1[c], m);
        s2[c] += __shfl_xor(s2[c], m);
      }
    }
    if (lane < 8) {
      const int cg = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) % CV);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        red[0][wv][cg * 8 + c] = s1[c];
        red[1][wv][cg * 8 + c] = s2[c];
      }
    }
    __syncthreads();
    if (threadIdx.x < 128) {
      const int q = threadIdx.x >> 6, ch = threadIdx.x & 63;
      float a = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < kPoolThreads / 64; ++w2) a += red[q][w2][ch];
      slab[((int64_t)q * 64 + ch) * gridDim.x + blockIdx.x] = a;
    }
  }
}

// global average pool backward, NHWC: dx[n, hw, c] = dy[n, c] * inv_hw.  dy is one
// [C] row per image (L2-resident), dx is written once with 16-byte stores in memory
// order - the gradient of x.mean((2, 3)) materialised channels-last directly, instead
// of an expanded view that a later .contiguous() copies with strided 2-byte stores.
template <typename T, bool VEC>
__global__ void __launch_bounds__(kPoolThreads)
    gap_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int64_t N, int64_t HW, int C,
              float inv_hw) {
  constexpr int V = VEC ? 8 : 1;
  const int CV = C / V;
  const int64_t total = N * HW * CV;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    const int64_t n = t / CV / HW;
    float g[V];
    if constexpr (VEC) load8(dy + n * C + cv * V, g);
    else g[0] = to_f32(dy[n * C + cv]);
#pragma unroll
    for (int i = 0; i < V; ++i) g[i] *= inv_hw;
    if constexpr (VEC) store8(dx + t * V, g);
    else dx[t] = from_f32<T>(g[0]);
  }
}

template <typename F>
void pool_dispatch(DType t, F&& f) {
  switch (t) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    case DType::BF16: f(bf16_t{}); break;
    default: break;
  }
}

// the specialised 3x3 / stride-2 / pad-1 kernels (output size floor((H-1)/2)+1)
bool stem_ok(int k, int s, int p, int H, int W, int OH, int OW) {
  return k == 3 && s == 2 && p == 1 && OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1;
}

int pool_grid(int64_t items) {
  int64_t b = (items + kPoolThreads - 1) / kPoolThreads;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

void maxpool2d_nhwc_fwd(const void* x, DType t, void* y, uint8_t* idx, int N, int H, int W, int C,
                        int OH, int OW, int k, int s, int p, hipStream_t st, const float* mean,
                        const float* invstd, const float* bw, const float* bb) {
  const bool vec = C % 8 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 &&
                   ((uintptr_t)idx % 8) == 0;
  const int64_t items = (int64_t)N * OH * OW * (vec ? C / 8 : C);
  if (items == 0) return;
  const PoolBN bn{mean, invstd, bw, bb};
  const bool with_bn = mean != nullptr;
  pool_dispatch(t, [&](auto t0) {
    using T = decltype(t0);
    const dim3 g(pool_grid(items)), b(kPoolThreads);
    const T* xp = static_cast<const T*>(x);
    T* yp = static_cast<T*>(y);
    if constexpr (sizeof(T) == 2) {
      if (vec && stem_ok(k, s, p, H, W, OH, OW) && (!with_bn || C <= kPoolBNMaxC)) {
        if (with_bn)
          hipLaunchKernelGGL((maxpool3s2_fwd_k<T, true>), g, b, 0, st, xp, yp, idx, N, H, W, C,
                             OH, OW, bn);
        else
          hipLaunchKernelGGL((maxpool3s2_fwd_k<T, false>), g, b, 0, st, xp, yp, idx, N, H, W, C,
                             OH, OW, bn);
        return;
      }
    }
    if (vec && with_bn)
      hipLaunchKernelGGL((maxpool_fwd_k<T, true, true>), g, b, 0, st, xp, yp, idx, N, H, W, C,
                         OH, OW, k, s, p, bn);
    else if (vec)
      hipLaunchKernelGGL((maxpool_fwd_k<T, true, false>), g, b, 0, st, xp, yp, idx, N, H, W, C,
                         OH, OW, k, s, p, bn);
    else if (with_bn)
      hipLaunchKernelGGL((maxpool_fwd_k<T, false, true>), g, b, 0, st, xp, yp, idx, N, H, W, C,
                         OH, OW, k, s, p, bn);
    else
      hipLaunchKernelGGL((maxpool_fwd_k<T, false, false>), g, b, 0, st, xp, yp, idx, N, H, W, C,
                         OH, OW, k, s, p, bn);
  });
}

int maxpool_bwd_bn_grid(int N, int H, int W) {
  const int64_t blk = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * 8;
  const int g = pool_grid(blk);
  return g > 2048 ? 2048 : g;
}

bool maxpool2d_nhwc_bwd_bn_ok(int H, int W, int C, int OH, int OW, int k, int s, int p) {
  return C == 64 && stem_ok(k, s, p, H, W, OH, OW);
}

void maxpool2d_nhwc_bwd_bn(const void* dy, const uint8_t* idx, DType t, void* dx, int N, int H,
                           int W, int C, int OH, int OW, const void* x, const float* mean,
                           const float* invstd, const float* bw, const float* bb, float* slab,
                           hipStream_t st) {
  const int grid = maxpool_bwd_bn_grid(N, H, W);
  pool_dispatch(t, [&](auto t0) {
    using T = decltype(t0);
    if constexpr (sizeof(T) == 2) {
      hipLaunchKernelGGL((maxpool3s2_bwd2_k<T, true>), dim3(grid), dim3(kPoolThreads), 0, st,
                         static_cast<const T*>(dy), idx, static_cast<T*>(dx), N, H, W, C, OH, OW,
                         static_cast<const T*>(x), mean, invstd, bw, bb, slab);
    }
  });
}

void maxpool2d_nhwc_bwd(const void* dy, const uint8_t* idx, DType t, void* dx, int N, int H,
                        int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  const bool vec = C % 8 == 0 && ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dx % 16) == 0 &&
                   ((uintptr_t)idx % 8) == 0;
  const int64_t items = (int64_t)N * H * W * (vec ? C / 8 : C);
  if (items == 0) return;
  pool_dispatch(t, [&](auto t0) {
    using T = decltype(t0);
    if constexpr (sizeof(T) == 2) {
      if (vec && stem_ok(k, s, p, H, W, OH, OW)) {
        const int64_t blk = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
        hipLaunchKernelGGL((maxpool3s2_bwd2_k<T, false>), dim3(pool_grid(blk)), dim3(kPoolThreads), 0,
                           st, static_cast<const T*>(dy), idx, static_cast<T*>(dx), N, H, W, C,
                           OH, OW);
        return;
      }
    }
    if (vec)
      hipLaunchKernelGGL((maxpool_bwd_k<T, true>), dim3(pool_grid(items)), dim3(kPoolThreads), 0,
                         st, static_cast<const T*>(dy), idx, static_cast<T*>(dx), N, H, W, C, OH,
                         OW, k, s, p);
    else
      hipLaunchKernelGGL((maxpool_bwd_k<T, false>), dim3(pool_grid(items)), dim3(kPoolThreads), 0,
                         st, static_cast<const T*>(dy), idx, static_cast<T*>(dx), N, H, W, C, OH,
                         OW, k, s, p);
  });
}

void gap_nhwc_bwd(const void* dy, DType t, void* dx, int64_t N, int64_t HW, int C,
                  hipStream_t st) {
  const bool vec = C % 8 == 0 && ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dx % 16) == 0;
  const int64_t items = N * HW * (vec ? C / 8 : C);
  if (items == 0) return;
  const float inv_hw = 1.f / (float)HW;
  pool_dispatch(t, [&](auto t0) {
    using T = decltype(t0);
    if (vec)
      hipLaunchKernelGGL((gap_bwd_k<T, true>), dim3(pool_grid(items)), dim3(kPoolThreads), 0, st,
                         static_cast<const T*>(dy), static_cast<T*>(dx), N, HW, C, inv_hw);
    else
      hipLaunchKernelGGL((gap_bwd_k<T, false>), dim3(pool_grid(items)), dim3(kPoolThreads), 0,
                         st, static_cast<const T*>(dy), static_cast<T*>(dx), N, HW, C, inv_hw);
  });
}

}  // namespace amd
