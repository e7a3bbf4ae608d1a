// Bias gradients of dense layers: column sums of a row-major [M, N] 16-bit tensor,
// optionally fused with the GELU backward that produces it.
//
// PyTorch's generic reduction runs dy.sum(0) for [16384 x 1024] bf16 at ~1 TB/s
// (profiles/bert_large_amd_latest.md: 99 launches, 2.9 ms per BERT-large step).
// Here: stage 1 = a split-row pass where a 256-thread block covers 256 columns x
// 8 row lanes (16-byte loads, 8 columns per lane, a wave reads two full 512-byte
// row segments per instruction) and writes fp32 partials [S][N]; stage 2 sums the
// S partials of a column (4 split lanes x 4 independent loads in flight) and
// writes the bias dtype.  Deterministic, no atomics.
//
// The activation-backward modes additionally compute the pre-activation gradient
// in the same pass - dpre = dh * gelu'(pre) (erf or tanh GELU, fused_dense's FFN)
// or dpre = dh * act'(y) from the layer's saved OUTPUT y (ReLU: y > 0; sigmoid:
// y (1 - y); apex.mlp) - write it and its column partials, so the bias gradient
// costs no extra read of dpre.
#include <cstdlib>

#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

constexpr int kCsThreads = 256;
constexpr int kCsCols = 256;   // columns per block (32 lanes x 8)
constexpr int kCsRowLanes = kCsThreads / (kCsCols / 8);

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) { load8(p, v); }

__device__ __forceinline__ float gelu_grad(float x, bool tanh_approx) {
  if (tanh_approx) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (x + k1 * x * x * x);
    const float t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  }
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// MODE 0: column sums of x.  MODE 1: dpre = dh * gelu'(pre) -> out, sums of dpre.
// MODE 2 / 3: dpre = dh * relu'(y) / dh * sigmoid'(y) with y the saved output.
template <int MODE>
__device__ __forceinline__ float act_grad(float p, bool tanh_approx) {
  if constexpr (MODE == 1) return gelu_grad(p, tanh_approx);
  else if constexpr (MODE == 2) return p > 0.f ? 1.f : 0.f;
  else return p * (1.f - p);
}

template <typename T, int MODE>
__global__ void __launch_bounds__(kCsThreads)
    colsum_partial_k(const T* __restrict__ x, const T* __restrict__ pre, T* __restrict__ out,
                     int64_t M, int N, int rows_per_split, bool tanh_approx,
                     float* __restrict__ part) {
  __shared__ float red[kCsRowLanes][kCsCols];
  const int cg = threadIdx.x % (kCsCols / 8), rl = threadIdx.x / (kCsCols / 8);
  const int c0 = blockIdx.x * kCsCols + cg * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  int64_t r1 = r0 + rows_per_split;
  if (r1 > M) r1 = M;
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
  if (c0 < N) {
    // 4 rows per iteration: their 16-byte loads (x and pre) are all issued before any
    // arithmetic, so a thread keeps 4-8 loads in flight instead of one (the FFN's GELU
    // backward [tokens x 4h] ran at ~2.3 TB/s one row at a time)
    constexpr int U = 4;
    int64_t r = r0 + rl;
    for (; r + (U - 1) * kCsRowLanes < r1; r += U * kCsRowLanes) {
      float v[U][8], p[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ld8(x + (r + u * kCsRowLanes) * N + c0, v[u]);
        if constexpr (MODE != 0) ld8(pre + (r + u * kCsRowLanes) * N + c0, p[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (MODE != 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[u][i] *= act_grad<MODE>(p[u][i], tanh_approx);
          store8(out + (r + u * kCsRowLanes) * N + c0, v[u]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] += v[u][i];
      }
    }
    for (; r < r1; r += kCsRowLanes) {
      float v[8];
      ld8(x + r * N + c0, v);
      if constexpr (MODE != 0) {
        float p[8];
        ld8(pre + r * N + c0, p);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] *= act_grad<MODE>(p[i], tanh_approx);
        store8(out + r * N + c0, v);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[rl][cg * 8 + i] = a[i];
  __syncthreads();
  const int c = blockIdx.x * kCsCols + threadIdx.x;
  if (threadIdx.x < kCsCols && c < N) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < kCsRowLanes; ++q) t += red[q][threadIdx.x];
    part[(int64_t)blockIdx.y * N + c] = t;
  }
}

// stage 2: 16 columns x 16 split lanes per block, each lane summing S/16 partials with
// 4 loads in flight - 4x the blocks of a 64-column form and a quarter of its dependent
// load rounds (that form, removed in round 6, ran 6-11 us per call in the BERT / GPT-2
// steps for ~0.5 MB of partials: 16 blocks of latency chains).  Same summation
// order across the partials of one split lane, so deterministic
template <typename TO>
__global__ void __launch_bounds__(256)
    colsum_final16_k(const float* __restrict__ part, int S, int N, TO* __restrict__ out) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    int s = sl;
    for (; s + 48 < S; s += 64) {
#pragma unroll
      for (int i = 0; i < 4; ++i) t[i] += part[(int64_t)(s + 16 * i) * N + c];
    }
    for (; s < S; s += 16) t[0] += part[(int64_t)s * N + c];
  }
  red[sl][cl] = (t[0] + t[1]) + (t[2] + t[3]);
  __syncthreads();
  if (sl == 0 && c < N) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) a += red[q][cl];
    out[c] = from_f32<TO>(a);
  }
}

template <typename TO>
void launch_final(const float* part, int S, int N, TO* out, hipStream_t st) {
  hipLaunchKernelGGL(colsum_final16_k<TO>, dim3((unsigned)((N + 15) / 16)), dim3(256), 0, st,
                     part, S, N, out);
}

__device__ __forceinline__ float gelu_f(float x, bool tanh_approx) {
  if (tanh_approx) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
  }
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}

// h = gelu(pre): a streaming pass with 4 independent 16-byte loads in flight per
// lane (the FFN forward's [tokens x 4h] activation; ATen's GELU ran it at ~4.3 TB/s)
template <typename T>
__global__ void __launch_bounds__(256)
    gelu_fwd_k(const T* __restrict__ x, T* __restrict__ y, int64_t n8, bool tanh_approx) {
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride * U) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n8) load8(x + (i + u * stride) * 8, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i + u * stride >= n8) continue;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u][k] = gelu_f(v[u][k], tanh_approx);
      store8(y + (i + u * stride) * 8, v[u]);
    }
  }
}

}  // namespace

void gelu_fwd(const void* x, void* y, DType t, int64_t n, bool tanh_approx, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  int64_t blocks = (n8 + 256 * 4 - 1) / (256 * 4);
  if (blocks > 8192) blocks = 8192;
  auto go = [&](auto t0) {
    using T = decltype(t0);
    hipLaunchKernelGGL((gelu_fwd_k<T>), dim3((unsigned)blocks), dim3(256), 0, st,
                       static_cast<const T*>(x), static_cast<T*>(y), n8, tanh_approx);
  };
  if (t == DType::BF16) go(bf16_t{});
  else if (t == DType::F16) go(half_t{});
  else go(float{});
}

void colsum_finalize(const float* part, int S, int N, void* out, DType tb, hipStream_t st) {
  if (tb == DType::F32) launch_final(part, S, N, static_cast<float*>(out), st);
  else if (tb == DType::BF16) launch_final(part, S, N, static_cast<bf16_t*>(out), st);
  else launch_final(part, S, N, static_cast<half_t*>(out), st);
}

int colsum_splits(int64_t M, int N) {
  const int cb = (N + kCsCols - 1) / kCsCols;
  int64_t S = (1024 + cb - 1) / cb;        // ~4 blocks per CU (2 per CU measured slower)
  const int64_t max_s = (M + 63) / 64;     // >= 64 rows per split
  if (S > max_s) S = max_s;
  return S < 1 ? 1 : (int)S;
}

void colsum(const void* x, const void* pre, void* out_dpre, DType t, int64_t M, int N,
            int act_mode, float* part, int S, void* bias_grad, DType tb, hipStream_t st) {
  const int rps = (int)((M + S - 1) / S);
  const dim3 grid((unsigned)((N + kCsCols - 1) / kCsCols), (unsigned)S);
  // act_mode: 0 none, 1 GELU (erf), 2 GELU (tanh), 3 ReLU(y), 4 sigmoid(y)
  const bool tanh_approx = act_mode == 2;
  auto launch1 = [&](auto t0) {
    using T = decltype(t0);
    const T* xp = static_cast<const T*>(x);
    const T* pp = static_cast<const T*>(pre);
    T* op = static_cast<T*>(out_dpre);
    switch (act_mode) {
      case 0:
        hipLaunchKernelGGL((colsum_partial_k<T, 0>), grid, dim3(kCsThreads), 0, st, xp, nullptr,
                           nullptr, M, N, rps, false, part);
        break;
      case 3:
        hipLaunchKernelGGL((colsum_partial_k<T, 2>), grid, dim3(kCsThreads), 0, st, xp, pp, op,
                           M, N, rps, false, part);
        break;
      case 4:
        hipLaunchKernelGGL((colsum_partial_k<T, 3>), grid, dim3(kCsThreads), 0, st, xp, pp, op,
                           M, N, rps, false, part);
        break;
      default:
        hipLaunchKernelGGL((colsum_partial_k<T, 1>), grid, dim3(kCsThreads), 0, st, xp, pp, op,
                           M, N, rps, tanh_approx, part);
    }
  };
  if (t == DType::BF16) launch1(bf16_t{});
  else if (t == DType::F16) launch1(half_t{});
  else launch1(float{});
  colsum_finalize(part, S, N, bias_grad, tb, st);
}

}  // namespace amd
