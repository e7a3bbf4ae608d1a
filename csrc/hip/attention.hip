// Fused multi-head attention for gfx950 (head dim 64, bf16 / fp16, optional
// causal mask and dropout): flash-attention style forward and backward on
// v_mfma_f32_32x32x16_{bf16,f16}, written for CDNA4 rather than ported.
//
// Layouts: q, k, v are [B, S, H, 64] views with arbitrary batch / sequence /
// head strides (e.g. slices of a fused qkv projection - no copies); o and the
// gradients are written as contiguous [B, S, H, 64] (so `.view(B, S, H*64)`
// is free); lse is [B, H, S] fp32 in log2 units.
//
// Forward (one wave = 32 queries, workgroup = 4 waves = 128 queries):
//   * "swapped" QK^T: S^T = K . Q^T so a lane owns one query's scores (column
//     on the lane, 16 keys per register file half) and the softmax row is
//     lane-local up to one lane^32 exchange;
//   * the exp'ed scores feed P.V straight from the accumulator registers (an
//     MFMA that sums over the accumulator's row index needs no data movement);
//     V is read from LDS with ds_read_b64_tr_b16 in the matching key order;
//   * K / V tiles (64 keys) are DMA'd HBM -> LDS with global_load_lds, double
//     buffered, K with a (row>>1)&7 chunk swizzle (ds_read_b128 rows), V with a
//     ((row>>1)&1)<<2 swizzle (transposed reads) - both conflict-free;
//   * dropout keeps are a counter-based hash of (seed, b*H+h, query, key) so the
//     backward regenerates them bit-exactly.
// Backward = preprocess (D = rowsum(dO*O)), a dK/dV kernel (workgroup owns 128
// keys, loops over queries, "unswapped" S = Q.K^T so dV = P^T.dO and
// dK = dS^T.Q sum over the register rows) and a dQ kernel (workgroup owns 128
// queries, swapped orientation so dQ = dS.K sums over register rows) - no
// atomics, no LDS transposes of score tiles.
#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short v4s_t __attribute__((ext_vector_type(4)));

constexpr int kAD = 64;          // head dim
constexpr int kAT = 256;         // threads
constexpr int kAKT = 64;         // keys per K/V tile
constexpr int kARow = kAD * 2;   // 128 B per row

template <typename T> struct Frag;
template <> struct Frag<bf16_t> { typedef bf16_t v8 __attribute__((ext_vector_type(8))); };
template <> struct Frag<half_t> { typedef half_t v8 __attribute__((ext_vector_type(8))); };

template <typename T>
__device__ __forceinline__ f32x16_t mfma32(typename Frag<T>::v8 a, typename Frag<T>::v8 b,
                                           f32x16_t c) {
  if constexpr (std::is_same<T, bf16_t>::value)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// LDS images of a [64 rows][64 d] 16-bit tile (128-B rows)
__device__ __forceinline__ int swz_rows(int row, int chunk) {   // for ds_read_b128 row reads
  return row * kARow + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ int swz_tr(int row, int chunk) {     // for transposed reads
  return row * kARow + ((chunk ^ (((row >> 1) & 1) << 2)) << 4);
}

template <typename T>
__device__ __forceinline__ typename Frag<T>::v8 lds_row8(const unsigned char* base, int off) {
  return *reinterpret_cast<const typename Frag<T>::v8*>(base + off);
}

// transposed fragment: element j of this lane = column `col` of rows r0+j (j<4) and
// r1+j-4 (j>=4), rows/cols as the lane's 16-lane group addresses them
template <typename T>
__device__ __forceinline__ typename Frag<T>::v8 lds_tr8(const unsigned char* base, int lo,
                                                        int hi) {
  v4s_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(base + lo));
  v4s_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(base + hi));
  typename Frag<T>::v8 f;
  v4s_t* fp = reinterpret_cast<v4s_t*>(&f);
  fp[0] = a;
  fp[1] = b;
  return f;
}

// byte offset of the 8-byte piece a lane supplies for a transposed read of rows
// [r0, r0+4) x columns [c0, c0+16) of a swz_tr image
__device__ __forceinline__ int tr_addr(int r0, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  return swz_tr(r0 + q, col >> 3) + ((col >> 2) & 1) * 8;
}

// counter-based dropout bits: one 32-bit hash per (query, key pair), 16 bits per key
__device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint32_t bh, uint32_t q,
                                              uint32_t kp) {
  uint32_t x = seed ^ (bh * 0x9E3779B1u) ^ (q * 0x85EBCA77u) ^ (kp * 0xC2B2AE3Du);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool drop_keep(uint32_t h, int key, uint32_t thr16) {
  const uint32_t v = (key & 1) ? (h >> 16) : (h & 0xffffu);
  return v >= thr16;
}

template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  T x = (T)a, y = (T)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

// registers 8s..8s+7 of a 32x32 accumulator as a 16-bit MFMA fragment
template <typename T>
__device__ __forceinline__ typename Frag<T>::v8 acc_frag(const f32x16_t& x, int s) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pack2<T>(x[8 * s + 2 * i], x[8 * s + 2 * i + 1]);
  return __builtin_bit_cast(typename Frag<T>::v8, *reinterpret_cast<uint4*>(w));
}

struct AttnArgs {
  const void* q;
  const void* k;
  const void* v;
  int64_t qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh;  // element strides
  void* o;           // [B][S][H][64]
  float* lse;        // [B][H][S]
  int B, H, S;
  float scale_log2;  // softmax scale * log2(e)
  uint32_t thr16;    // dropout threshold (p * 65536), 0 = no dropout
  float inv_keep;    // 1 / (1 - p)
  uint32_t seed;
};

// ---------------------------------------------------------------------------- forward
template <typename T, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kAT, 2) attn_fwd_k(AttnArgs a) {
  typedef typename Frag<T>::v8 v8;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * 2 * kAKT * kARow];  // 2 x (K, V)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hl = lane >> 5, c32 = lane & 31;
  const int bh = blockIdx.y, b = bh / a.H, hh = bh - b * a.H;
  const int qb0 = blockIdx.x * 128;
  const int q = qb0 + wid * 32 + c32;  // this lane's query
  const T* Q = static_cast<const T*>(a.q) + b * a.qsb + hh * a.qsh;
  const T* K = static_cast<const T*>(a.k) + b * a.ksb + hh * a.ksh;
  const T* V = static_cast<const T*>(a.v) + b * a.vsb + hh * a.vsh;

  // Q^T fragments (B operand of S^T = K . Q^T): d = 16s + 8hl + j
  v8 qf[4];
  {
    const int qq = q < a.S ? q : a.S - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[s] = *reinterpret_cast<const v8*>(Q + qq * a.qss + 16 * s + 8 * hl);
  }

  int nkt = (a.S + kAKT - 1) / kAKT;
  if (CAUSAL) {
    const int last = (qb0 + 127 < a.S ? qb0 + 127 : a.S - 1) / kAKT + 1;
    nkt = last < nkt ? last : nkt;
  }
  // DMA: each wave fills 16 rows of K and of V per tile (2 x 1 KiB instructions each)
  const int lrow = lane >> 3, pch = lane & 7;
  auto issue = [&](int kt, int buf) {
    unsigned char* Kl = lds + buf * 2 * kAKT * kARow;
    unsigned char* Vl = Kl + kAKT * kARow;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wid * 2 + i) * 8 + lrow;
      const int key = kt * kAKT + row;
      const int kk = key < a.S ? key : a.S - 1;
      const int chk = (swz_rows(row, pch) - row * kARow) >> 4;  // logical chunk at pch
      const int chv = (swz_tr(row, pch) - row * kARow) >> 4;
      glds16(K + kk * a.kss + chk * 8, Kl + (wid * 2 + i) * 1024);
      glds16(V + kk * a.vss + chv * 8, Vl + (wid * 2 + i) * 1024);
    }
  };

  f32x16_t o[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) o[0][i] = o[1][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  // loop-invariant LDS offsets
  int koff[2][4];  // [key half t][d step s]: K row 32t + c32, chunk 2s + hl
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) koff[t][s] = swz_rows(32 * t + c32, 2 * s + hl);
  int vlo[2][2][2], vhi[2][2][2];  // [d tile][key half t][k step s]
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r0 = 32 * t + 16 * s + 4 * hl;
        const int c0 = 32 * dt + ((lane >> 4) & 1) * 16;
        vlo[dt][t][s] = tr_addr(r0, c0, lane);
        vhi[dt][t][s] = tr_addr(r0 + 8, c0, lane);
      }

  issue(0, 0);
  for (int kt = 0; kt < nkt; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nkt) issue(kt + 1, (kt + 1) & 1);
    const unsigned char* Kl = lds + (kt & 1) * 2 * kAKT * kARow;
    const unsigned char* Vl = Kl + kAKT * kARow;
    const int k0 = kt * kAKT;
    if (CAUSAL && k0 > qb0 + wid * 32 + 31) continue;  // whole tile masked for this wave

    f32x16_t x[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) x[t][i] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) x[t] = mfma32<T>(lds_row8<T>(Kl, koff[t][s]), qf[s], x[t]);
    }
    // scores -> log2 units, mask, running max
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float sv = x[t][r] * a.scale_log2;
        const int key = k0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (key >= a.S || (CAUSAL && key > q)) sv = -INFINITY;
        x[t][r] = sv;
        tmax = fmaxf(tmax, sv);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(x[t][r] - mnew);
        psum += p;
        x[t][r] = p;
      }
    l = l * alpha + psum;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[0][i] *= alpha;
      o[1][i] *= alpha;
    }
    if (DROP) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const int key = k0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;  // even
          const uint32_t hsh = drop_hash(a.seed, (uint32_t)bh, (uint32_t)q, (uint32_t)(key >> 1));
          x[t][r] = drop_keep(hsh, key, a.thr16) ? x[t][r] * a.inv_keep : 0.f;
          x[t][r + 1] = drop_keep(hsh, key + 1, a.thr16) ? x[t][r + 1] * a.inv_keep : 0.f;
        }
    }
    // O^T[d][q] += V^T[d][key] . P^T[key][q]
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const v8 pf = acc_frag<T>(x[t], s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          o[dt] = mfma32<T>(lds_tr8<T>(Vl, vlo[dt][t][s], vhi[dt][t][s]), pf, o[dt]);
      }
  }

  const float lt = l + __shfl_xor(l, 32);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (q < a.S) {
    T* O = static_cast<T*>(a.o) + (((int64_t)b * a.S + q) * a.H + hh) * kAD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * hl;
        uint2 w;
        w.x = pack2<T>(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
        w.y = pack2<T>(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(O + d) = w;
      }
    if (hl == 0) a.lse[(int64_t)bh * a.S + q] = m + log2f(lt);
  }
}

}  // namespace

void attn_fwd(const AttnLaunch& L, hipStream_t st) {
  AttnArgs a;
  a.q = L.q; a.k = L.k; a.v = L.v;
  a.qsb = L.qsb; a.qss = L.qss; a.qsh = L.qsh;
  a.ksb = L.ksb; a.kss = L.kss; a.ksh = L.ksh;
  a.vsb = L.vsb; a.vss = L.vss; a.vsh = L.vsh;
  a.o = L.o; a.lse = L.lse; a.B = L.B; a.H = L.H; a.S = L.S;
  a.scale_log2 = L.scale * 1.4426950408889634f;
  a.thr16 = L.dropout > 0.f ? (uint32_t)(L.dropout * 65536.f + 0.5f) : 0u;
  a.inv_keep = L.dropout > 0.f ? 65536.f / (65536.f - (float)a.thr16) : 1.f;
  a.seed = L.seed;
  dim3 grid((L.S + 127) / 128, L.B * L.H), block(kAT);
  const bool drop = a.thr16 != 0;
#define ATTN_FWD_LAUNCH(T)                                                                     \
  if (L.causal) {                                                                              \
    if (drop) hipLaunchKernelGGL((attn_fwd_k<T, true, true>), grid, block, 0, st, a);          \
    else hipLaunchKernelGGL((attn_fwd_k<T, true, false>), grid, block, 0, st, a);              \
  } else {                                                                                     \
    if (drop) hipLaunchKernelGGL((attn_fwd_k<T, false, true>), grid, block, 0, st, a);         \
    else hipLaunchKernelGGL((attn_fwd_k<T, false, false>), grid, block, 0, st, a);             \
  }
  if (L.dtype == DType::BF16) {
    ATTN_FWD_LAUNCH(bf16_t)
  } else {
    ATTN_FWD_LAUNCH(half_t)
  }
#undef ATTN_FWD_LAUNCH
}

}  // namespace amd
