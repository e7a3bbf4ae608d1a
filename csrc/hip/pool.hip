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
#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

constexpr int kPoolThreads = 256;

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

void maxpool2d_nhwc_bwd(const void* dy, const uint8_t* idx, DType t, void* dx, int N, int H,
                        int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  const bool vec = C % 8 == 0 && ((uintptr_t)dy % 16) == 0 && ((uintptr_t)dx % 16) == 0 &&
                   ((uintptr_t)idx % 8) == 0;
  const int64_t items = (int64_t)N * H * W * (vec ? C / 8 : C);
  if (items == 0) return;
  pool_dispatch(t, [&](auto t0) {
    using T = decltype(t0);
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
