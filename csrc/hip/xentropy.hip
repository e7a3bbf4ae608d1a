// Fused softmax cross entropy with label smoothing for gfx950
// (apex.contrib.xentropy.SoftmaxCrossEntropyLoss semantics).
//
// One workgroup (256 threads = 4 wave64) per row of logits.  The forward makes a
// SINGLE pass over the row: every thread keeps a running (max, sum of exp) pair
// in log2 units plus the plain sum (for smoothing) over 16-byte loads, then a
// wave64 xor-shuffle and one LDS step combine them.  It writes the row loss and
// the row's natural-log log-sum-exp (the only statistic the backward needs).
// The backward re-reads the row once and writes
//   grad = dloss * (softmax - (1 - eps) * onehot(label) - eps / V).
// Logits are read in their own dtype (bf16 / fp16 / fp32): no fp32 copy of the
// [rows, vocab] matrix is ever materialised (for GPT-2-medium that copy alone
// is 1.6 GB per step).  Rows whose label equals padding_idx (or lies outside
// [0, V)) get zero loss and zero gradient.
#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

constexpr int kXT = 256;
constexpr float kL2E = 1.4426950408889634f;

// (m, s) <- (m, s) (+) (m2, s2): combine two running (max, sum 2^(x - max)) pairs
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) {
    m = m2;
    s = s2;
    return;
  }
  if (m2 > m) {
    s = s * exp2f(m - m2) + s2;
    m = m2;
  } else {
    s += s2 * exp2f(m2 - m);
  }
}

// split a row into a scalar head (up to 16-byte alignment), a body of 8-element
// vectors and a scalar tail; `vec_ok` = the companion pointer shares x's alignment
template <typename T>
__device__ __forceinline__ void row_split(const T* row, int V, bool vec_ok, int& head, int& nvec) {
  constexpr int E = 16 / (int)sizeof(T);
  if (!vec_ok) {
    head = 0;
    nvec = 0;
    return;
  }
  const int mis = (int)(((uintptr_t)row % 16) / sizeof(T));
  head = mis ? E - mis : 0;
  if (head > V) head = V;
  nvec = (V - head) / 8;
}

__device__ __forceinline__ bool ignored(int64_t lab, int64_t padding_idx, int V) {
  return lab == padding_idx || lab < 0 || lab >= V;
}

template <typename T, typename TO>
__global__ void __launch_bounds__(kXT)
    xent_fwd_k(const T* __restrict__ x, const int64_t* __restrict__ labels, int V,
               float smoothing, int64_t padding_idx, TO* __restrict__ loss,
               float* __restrict__ lse_out) {
  __shared__ float red[3][kXT / 64];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * (int64_t)V;
  const int tid = threadIdx.x;
  int head, nvec;
  row_split(xr, V, true, head, nvec);
  float m = -INFINITY, s = 0.f, tot = 0.f;  // m, s in log2 units
  if (tid < head) {
    const float v = to_f32(xr[tid]);
    m = v * kL2E;
    s = 1.f;
    tot = v;
  }
  const T* body = xr + head;
  for (int i = tid; i < nvec; i += kXT) {
    float v[8];
    load8(body + (int64_t)i * 8, v);
    float vm = v[0];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      vm = fmaxf(vm, v[j]);
      tot += v[j];
    }
    const float vm2 = vm * kL2E;
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ps += exp2f(fmaf(v[j], kL2E, -vm2));
    lse_merge(m, s, vm2, ps);
  }
  for (int j = head + nvec * 8 + tid; j < V; j += kXT) {
    const float v = to_f32(xr[j]);
    lse_merge(m, s, v * kL2E, 1.f);
    tot += v;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float m2 = __shfl_xor(m, off), s2 = __shfl_xor(s, off);
    lse_merge(m, s, m2, s2);
    tot += __shfl_xor(tot, off);
  }
  const int lane = tid & 63, wid = tid >> 6;
  if (lane == 0) {
    red[0][wid] = m;
    red[1][wid] = s;
    red[2][wid] = tot;
  }
  __syncthreads();
  if (tid == 0) {
    float M = red[0][0], S = red[1][0], TT = red[2][0];
#pragma unroll
    for (int w = 1; w < kXT / 64; ++w) {
      lse_merge(M, S, red[0][w], red[1][w]);
      TT += red[2][w];
    }
    const float lse = (M + log2f(S)) / kL2E;
    const int64_t lab = labels[row];
    float l = 0.f;
    if (!ignored(lab, padding_idx, V)) {
      const float xl = to_f32(xr[lab]);
      l = lse - (1.f - smoothing) * xl - smoothing * TT / (float)V;
    }
    loss[row] = from_f32<TO>(l);
    lse_out[row] = lse;
  }
}

template <typename T, typename TG>
__global__ void __launch_bounds__(kXT)
    xent_bwd_k(const TG* __restrict__ dloss, const T* __restrict__ x,
               const float* __restrict__ lse, const int64_t* __restrict__ labels, int V,
               float smoothing, int64_t padding_idx, T* __restrict__ dx, bool vec_ok) {
  const int64_t row = blockIdx.x;
  const T* xr = x + row * (int64_t)V;
  T* dr = dx + row * (int64_t)V;
  const int tid = threadIdx.x;
  const int64_t lab = labels[row];
  const bool ign = ignored(lab, padding_idx, V);
  const float g = ign ? 0.f : to_f32(dloss[row]);
  const float L2 = lse[row] * kL2E;
  const float sm = smoothing / (float)V, on = 1.f - smoothing;
  int head, nvec;
  row_split(xr, V, vec_ok, head, nvec);
  auto one = [&](int j) {
    const float p = exp2f(fmaf(to_f32(xr[j]), kL2E, -L2));
    dr[j] = from_f32<T>(g * (p - sm - (j == lab ? on : 0.f)));
  };
  if (tid < head) one(tid);
  const T* xb = xr + head;
  T* db = dr + head;
  for (int i = tid; i < nvec; i += kXT) {
    float v[8];
    load8(xb + (int64_t)i * 8, v);
    const int j0 = head + i * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float p = exp2f(fmaf(v[j], kL2E, -L2));
      v[j] = g * (p - sm - (j0 + j == lab ? on : 0.f));
    }
    store8(db + (int64_t)i * 8, v);
  }
  for (int j = head + nvec * 8 + tid; j < V; j += kXT) one(j);
}

template <typename F>
void xdispatch(DType t, F&& f) {
  switch (t) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    case DType::BF16: f(bf16_t{}); break;
    default: break;
  }
}

}  // namespace

void xentropy_fwd(const void* x, DType tx, const int64_t* labels, int64_t rows, int V,
                  float smoothing, int64_t padding_idx, void* loss, DType tloss, float* lse,
                  hipStream_t st) {
  if (rows == 0) return;
  xdispatch(tx, [&](auto t0) {
    using T = decltype(t0);
    xdispatch(tloss, [&](auto o0) {
      using TO = decltype(o0);
      hipLaunchKernelGGL((xent_fwd_k<T, TO>), dim3((unsigned)rows), dim3(kXT), 0, st,
                         static_cast<const T*>(x), labels, V, smoothing, padding_idx,
                         static_cast<TO*>(loss), lse);
    });
  });
}

void xentropy_bwd(const void* dloss, DType tg, const void* x, DType tx, const float* lse,
                  const int64_t* labels, int64_t rows, int V, float smoothing,
                  int64_t padding_idx, void* dx, hipStream_t st) {
  if (rows == 0) return;
  const bool vec_ok = ((uintptr_t)x % 16) == ((uintptr_t)dx % 16);
  xdispatch(tx, [&](auto t0) {
    using T = decltype(t0);
    xdispatch(tg, [&](auto g0) {
      using TG = decltype(g0);
      hipLaunchKernelGGL((xent_bwd_k<T, TG>), dim3((unsigned)rows), dim3(kXT), 0, st,
                         static_cast<const TG*>(dloss), static_cast<const T*>(x), lse, labels, V,
                         smoothing, padding_idx, static_cast<T*>(dx), vec_ok);
    });
  });
}

}  // namespace amd
