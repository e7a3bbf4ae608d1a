// Device-side helpers shared by every gfx950 kernel in this framework.
//
// Design notes (MI355X / CDNA4):
//  * A wavefront is 64 lanes.  Every reduction here is written for wave64:
//    xor-shuffles over offsets 32..1, then one LDS slot per wave.
//  * Memory-bound kernels move 16 B per lane per access (dwordx4); bf16/fp16 are
//    loaded 8 at a time and converted in registers (fp32 math everywhere).
//  * bf16 uses the clang native __bf16 type, which lowers to v_cvt_pk_bf16_f32
//    (round-to-nearest-even) on gfx950; fp16 uses _Float16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amd {

constexpr int kWave = 64;

enum class DType : int { F32 = 0, F16 = 1, BF16 = 2, F64 = 3 };

typedef _Float16 half_t;
typedef __bf16 bf16_t;

template <typename T> struct DTypeOf;
template <> struct DTypeOf<float> { static constexpr DType value = DType::F32; };
template <> struct DTypeOf<half_t> { static constexpr DType value = DType::F16; };
template <> struct DTypeOf<bf16_t> { static constexpr DType value = DType::BF16; };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(half_t x) { return (float)x; }
__device__ __forceinline__ float to_f32(bf16_t x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ half_t from_f32<half_t>(float x) { return (half_t)x; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float x) { return (bf16_t)x; }

__device__ __forceinline__ bool finite_f32(float x) {
  // exponent bits all-ones <=> inf/nan; cheaper than isfinite() on the VALU.
  return (__float_as_uint(x) & 0x7f800000u) != 0x7f800000u;
}

// ---------------------------------------------------------------------------
// 8-wide vector IO: one 16-byte access for 16-bit types, two for fp32.
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef half_t f16x8 __attribute__((ext_vector_type(8)));
typedef bf16_t bf16x8 __attribute__((ext_vector_type(8)));

template <typename T> struct Vec8;

template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    f32x4 a = {v[0], v[1], v[2], v[3]};
    f32x4 b = {v[4], v[5], v[6], v[7]};
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};

template <> struct Vec8<half_t> {
  static __device__ __forceinline__ void load(const half_t* p, float (&v)[8]) {
    f16x8 a = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
  static __device__ __forceinline__ void store(half_t* p, const float (&v)[8]) {
    f16x8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (half_t)v[i];
    *reinterpret_cast<f16x8*>(p) = a;
  }
};

template <> struct Vec8<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float (&v)[8]) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float (&v)[8]) {
    bf16x8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (bf16_t)v[i];
    *reinterpret_cast<bf16x8*>(p) = a;
  }
};

template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) { Vec8<T>::load(p, v); }
template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&v)[8]) { Vec8<T>::store(p, v); }

// Bounded scalar variants for tails / unaligned tensors.
template <typename T>
__device__ __forceinline__ void load8_tail(const T* p, int n, float (&v)[8], float fill = 0.f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (i < n) ? to_f32(p[i]) : fill;
}
template <typename T>
__device__ __forceinline__ void store8_tail(T* p, int n, const float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < n) p[i] = from_f32<T>(v[i]);
}

// ---------------------------------------------------------------------------
// wave64 / block reductions
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, kWave);
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x = fmaxf(x, __shfl_xor(x, off, kWave));
  return x;
}

// Sum over the whole block; result valid in every thread.  `scratch` must hold
// blockDim.x/64 floats.  Deterministic (fixed shuffle + fixed wave order).
__device__ __forceinline__ float block_sum(float x, float* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  x = wave_sum(x);
  __syncthreads();  // protect scratch reuse across calls
  if (lane == 0) scratch[wid] = x;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < nw; ++w) r += scratch[w];
  return r;
}
__device__ __forceinline__ float block_max(float x, float* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  x = wave_max(x);
  __syncthreads();
  if (lane == 0) scratch[wid] = x;
  __syncthreads();
  float r = scratch[0];
  for (int w = 1; w < nw; ++w) r = fmaxf(r, scratch[w]);
  return r;
}

// Chan et al. parallel combine of (mean, M2, count) triples.
__device__ __forceinline__ void welford_combine(float& mean, float& m2, float& n, float mean_b,
                                                float m2_b, float n_b) {
  float nn = n + n_b;
  if (nn == 0.f) return;
  float delta = mean_b - mean;
  float nb_over = n_b / nn;
  mean += delta * nb_over;
  m2 += m2_b + delta * delta * n * nb_over;
  n = nn;
}

// Read a device scalar that is either provided by pointer or by value.
__device__ __forceinline__ float scalar_or(const float* p, float v) { return p ? *p : v; }

}  // namespace amd
