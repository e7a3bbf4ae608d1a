// Fused multi-head attention for gfx950 (head dim 64, bf16 / fp16, optional
// causal mask and dropout): flash-attention style forward and backward on
// v_mfma_f32_32x32x16_{bf16,f16}, written for CDNA4 rather than ported.
//
// Layouts: q, k, v are [B, S, H, 64] views with arbitrary batch / sequence /
// head strides (e.g. slices of a fused qkv projection - no copies); o is written
// as contiguous [B, S, H, 64] (so `.view(B, S, H*64)` is free); the gradients
// go to caller-provided strided [B, S, H, 64] views (e.g. slices of one packed
// dqkv buffer); lse is [B, H, Sp] fp32 in log2 units with the row stride Sp a
// multiple of 64 (so the backward can DMA 64-query tiles of it).
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
// Backward = a dQ kernel (workgroup owns 128 queries, swapped orientation so
// dQ = dS.K sums over register rows; it also forms D = rowsum(dO*O) from the dO
// fragments it holds anyway) followed by a dK/dV kernel (workgroup owns 128 keys,
// loops over queries, "unswapped" S = Q.K^T so dV = P^T.dO and dK = dS^T.Q sum
// over the register rows) - no atomics (bitwise reproducible), no LDS transposes
// of score tiles, no preprocess launch.
#include <cstdlib>

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

// LDS DMA (16 bytes per lane into M0 + 16 * lane) as inline asm, NOT the builtin: the
// compiler cannot tell which LDS bytes a pending builtin DMA writes, so it put an
// s_waitcnt vmcnt(0) in front of LDS reads of the CURRENT tile that follow the next
// tile's issue (ISA of the round-5 build: one per forward loop, one to two per dQ / dK-dV
// loop) - every iteration waited out the prefetch it had just started.  Every kernel here
// orders the ring itself (s_waitcnt vmcnt(0) + barrier before a slot is read, the refill
// after the barrier), so the compiler need not know about these writes.
__device__ __forceinline__ uint32_t lds_addr32(const void* l) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)l;
}
__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("global_load_lds_dwordx4 %0, off" : : "v"(g), "{m0}"(lds_addr32(l)) : "memory");
#endif
}

// Tile DMA addressing: a wave-uniform tile base (SGPRs, one scalar multiply-add per
// tile) plus a loop-invariant per-lane 32-bit byte offset (row * row stride + swizzled
// chunk), which selects the saddr form of global_load_lds.  Computing the 64-bit
// address per tile and lane instead (clamped row * stride) cost 8 v_mul_lo_u32 + 4
// v_mad_u64_u32 per forward tile - quarter-rate VALU, ~1/5 of the no-dropout forward's
// VALU cycles.  Only a tile that reaches past S takes the clamped per-lane path.  The
// binding keeps row strides below 2^24 elements so the offsets fit 32 bits.
__device__ __forceinline__ void glds16o(const void* tile_base, uint32_t off, unsigned char* l) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("global_load_lds_dwordx4 %0, %1" : : "v"(off), "s"(tile_base), "{m0}"(lds_addr32(l))
               : "memory");
#endif
}

template <typename T>
__device__ __forceinline__ uint32_t row_off(int row, int64_t stride, int chunk) {
  return (uint32_t)row * (uint32_t)stride * (uint32_t)sizeof(T) + (uint32_t)chunk * 16u;
}

template <typename T>
__device__ __forceinline__ const T* tile_base(const T* p, int row0, int64_t stride) {
  return p + (int64_t)row0 * stride;
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

// Counter-based dropout bits: one 32-bit hash per (query, key QUAD), one byte per key:
// key k keeps its score iff byte (k & 3) of the hash is >= thr8 = round(256 p) (so p is
// quantised to 1/256 and the kept scores are scaled by 256 / (256 - thr8), unbiased for
// the quantised rate).  One hash per four scores instead of per two: the hash was ~half of
// the forward's VALU (267 of 520 per tile, docs/PERF.md round 4).  The hash input is a
// point of a Weyl lattice, base(seed, b*H+h) + q*kDropQ + (key>>2)*kDropK (mod 2^32), so
// a kernel steps from one (query, key quad) to the next with ONE add whose lattice offset
// is a compile-time literal; the mixer uses the full-rate 24-bit multiply
// (v_mul_u32_u24) where the classic 32-bit finalizers need the quarter-rate v_mul_lo_u32.
// tests/test_attention_gpu.py mirrors it bit for bit; tests/test_dropout_hash_cpu.py
// checks the keep rate, byte uniformity and neighbour correlations of the mirror.
constexpr uint32_t kDropQ = 0x85EBCA77u, kDropK = 0xC2B2AE3Du;

__device__ __forceinline__ uint32_t drop_base(uint32_t seed, uint32_t bh) {
  uint32_t x = seed ^ (bh * 0x9E3779B1u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
  x ^= x >> 16;
  x = __umul24(x, 0xE9846Bu) ^ (x >> 24);
  x ^= x >> 13;
  x = __umul24(x, 0x8B3C2Du) ^ (x >> 24);
  x ^= x >> 16;
  return x;
}

// the closed form; the kernels' incremental lattice steps compute exactly this
[[maybe_unused]] __device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint32_t bh, uint32_t q,
                                              uint32_t kquad) {
  return drop_mix(drop_base(seed, bh) + q * kDropQ + kquad * kDropK);
}

// raw v_exp_f32: exp2f() expands to a denormal-safe sequence (compare, select, ldexp:
// 5-6 VALU per score); softmax arguments are <= 0 and a result below 2^-126 may flush
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// keep decision of byte e (= key & 3) of a (query, key quad) hash
__device__ __forceinline__ bool drop_keep8(uint32_t h, int e, uint32_t thr8) {
  return ((h >> (8 * e)) & 0xffu) >= thr8;
}

// one v_cvt_pk_{bf16,f16}_f32 per pair (converting the two floats separately and
// merging the halves cost 4 VALU per pair: ~50 of the forward's ~215 VALU per tile)
template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef T t2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, t2));
}

// registers 8s..8s+7 of a 32x32 accumulator as a 16-bit MFMA fragment
template <typename T>
__device__ __forceinline__ typename Frag<T>::v8 acc_frag(const f32x16_t& x, int s) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pack2<T>(x[8 * s + 2 * i], x[8 * s + 2 * i + 1]);
  return __builtin_bit_cast(typename Frag<T>::v8, *reinterpret_cast<uint4*>(w));
}

// a 32(d) x 32(col) transposed accumulator pair (d = 32dt + row) as the 64 values
// of one [.., 64] 16-bit output row, times `mul`
template <typename T>
__device__ __forceinline__ void store_dT(T* row_ptr, const f32x16_t (&acc)[2], int hl, float mul) {
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * hl;
      uint2 w;
      w.x = pack2<T>(acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul);
      w.y = pack2<T>(acc[dt][4 * g + 2] * mul, acc[dt][4 * g + 3] * mul);
      *reinterpret_cast<uint2*>(row_ptr + d) = w;
    }
}

struct AttnArgs {
  const void* q;
  const void* k;
  const void* v;
  int64_t qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh;  // element strides
  void* o;           // [B][S][H][64]
  float* lse;        // [B][H][lse_stride]
  int B, H, S, lse_stride;
  float scale_log2;  // softmax scale * log2(e)
  uint32_t thr8;     // dropout threshold round(p * 256) on a hash byte, 0 = no dropout
  float inv_keep;    // 1 / (1 - p)
  uint32_t seed;
};

// ---------------------------------------------------------------------------- forward
// Block -> (tile, b*H+h).  Dispatch order is the flattened block id (x fastest) and
// consecutive ids go to consecutive XCDs, so: (1) the tiles of one head are gridDim.y
// ids apart - the same XCD whenever B*H % 8 == 0, so that head's K/V (fwd, dQ) or
// Q/dO (dK/dV) stream through one L2 instead of up to 8; (2) under a causal mask the
// tiles with the most work are dispatched first (longest-processing-time order: the
// last query tiles in fwd / dQ, the first key tiles in dK/dV), so the light diagonal
// tiles fill the tail instead of a few heavy ones.
__device__ __forceinline__ void tile_of_block(bool causal, bool heavy_high, int& tile, int& bh) {
  const int nt = gridDim.x, nbh = gridDim.y;
  const int id = blockIdx.x + blockIdx.y * nt;
  const int t = id / nbh;
  bh = id - t * nbh;
  tile = (causal && heavy_high) ? nt - 1 - t : t;
}

// the other 32-lane half's value of x (lane ^ 32) on the VALU (v_permlane32_swap)
// instead of an LDS round trip (ds_bpermute)
__device__ __forceinline__ float max_halves(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

template <typename T, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kAT, 2) attn_fwd_k(AttnArgs a) {
  typedef typename Frag<T>::v8 v8;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * 2 * kAKT * kARow];  // 2 x (K, V)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform to the compiler
  const int hl = lane >> 5, c32 = lane & 31;
  int tile, bh;
  tile_of_block(CAUSAL, true, tile, bh);
  const int b = bh / a.H, hh = bh - b * a.H;
  const int qb0 = tile * 128;
  const int q = qb0 + wid * 32 + c32;  // this lane's query
  // dropout lattice point of (q, key quad hl) at key tile 0
  const uint32_t dbase = DROP ? drop_base(a.seed, (uint32_t)bh) + (uint32_t)q * kDropQ +
                                    (uint32_t)hl * kDropK
                              : 0u;
  const T* Q = static_cast<const T*>(a.q) + b * a.qsb + hh * a.qsh;
  const T* K = static_cast<const T*>(a.k) + b * a.ksb + hh * a.ksh;
  const T* V = static_cast<const T*>(a.v) + b * a.vsb + hh * a.vsh;

  // Q^T fragments (B operand of S^T = K . Q^T): d = 16s + 8hl + j
  v8 qf[4];
  {
    const int qq = q < a.S ? q : a.S - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[s] = *reinterpret_cast<const v8*>(Q + (int64_t)qq * a.qss + 16 * s + 8 * hl);
  }

  int nkt = (a.S + kAKT - 1) / kAKT;
  if (CAUSAL) {
    const int last = (qb0 + 127 < a.S ? qb0 + 127 : a.S - 1) / kAKT + 1;
    nkt = last < nkt ? last : nkt;
  }
  // DMA: each wave fills 16 rows of K and of V per tile (2 x 1 KiB instructions each)
  const int lrow = lane >> 3, pch = lane & 7;
  uint32_t kof[2], vof[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wid * 2 + i) * 8 + lrow;
    kof[i] = row_off<T>(row, a.kss, (swz_rows(row, pch) - row * kARow) >> 4);  // logical chunk at pch
    vof[i] = row_off<T>(row, a.vss, (swz_tr(row, pch) - row * kARow) >> 4);
  }
  auto issue = [&](int kt, int buf) {
    unsigned char* Kl = lds + buf * 2 * kAKT * kARow;
    unsigned char* Vl = Kl + kAKT * kARow;
    if ((kt + 1) * kAKT <= a.S) {
      const T* kb = tile_base(K, kt * kAKT, a.kss);
      const T* vb = tile_base(V, kt * kAKT, a.vss);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        glds16o(kb, kof[i], Kl + (wid * 2 + i) * 1024);
        glds16o(vb, vof[i], Vl + (wid * 2 + i) * 1024);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wid * 2 + i) * 8 + lrow;
      const int key = kt * kAKT + row;
      const int kk = key < a.S ? key : a.S - 1;
      const int chk = (swz_rows(row, pch) - row * kARow) >> 4;  // logical chunk at pch
      const int chv = (swz_tr(row, pch) - row * kARow) >> 4;
      glds16(K + (int64_t)kk * a.kss + chk * 8, Kl + (wid * 2 + i) * 1024);
      glds16(V + (int64_t)kk * a.vss + chv * 8, Vl + (wid * 2 + i) * 1024);
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

  auto step = [&](int kt, int buf) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nkt) issue(kt + 1, buf ^ 1);
    const unsigned char* Kl = lds + buf * 2 * kAKT * kARow;
    const unsigned char* Vl = Kl + kAKT * kARow;
    const int k0 = kt * kAKT;
    if (CAUSAL && k0 > qb0 + wid * 32 + 31) return;  // whole tile masked for this wave

    f32x16_t x[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) x[t][i] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) x[t] = mfma32<T>(lds_row8<T>(Kl, koff[t][s]), qf[s], x[t]);
    }
    // mask (boundary / diagonal tiles only: the test is wave-uniform), running
    // max on the raw scores, then one fma + exp2 per score in log2 units
    const bool need_mask =
        (k0 + kAKT > a.S) || (CAUSAL && k0 + kAKT - 1 > qb0 + wid * 32);
    if (need_mask) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= a.S || (CAUSAL && key > q)) x[t][r] = -INFINITY;
        }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, x[t][r]);
    tmax = max_halves(tmax);
    const float mnew = fmaxf(m, tmax * a.scale_log2);
    // the O / l rescale by exp2(m - mnew) is skipped while no query of the wave
    // raised its running max (alpha == 1 exactly: same math, 32 fewer multiplies
    // per tile - the common case once the first tiles have set the max)
    const bool grow = __any(mnew != m);
    const float alpha = grow ? fexp2(m - mnew) : 1.f;
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(fmaf(x[t][r], a.scale_log2, -mnew));
        psum += p;
        x[t][r] = p;
      }
    l = l * alpha + psum;
    if (grow) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o[0][i] *= alpha;
        o[1][i] *= alpha;
      }
    }
    if (DROP) {  // dropped P (the 1/(1-p) factor is applied to O once, at the store)
      const uint32_t tb = dbase + (uint32_t)(k0 >> 2) * kDropK;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
          // key quad (k0 + 32t + 8rq + 4hl) >> 2 (keys + r & 3): a literal lattice step
          const uint32_t hsh = drop_mix(tb + (uint32_t)(8 * t + 2 * rq) * kDropK);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            x[t][4 * rq + e] = drop_keep8(hsh, e, a.thr8) ? x[t][4 * rq + e] : 0.f;
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
  };
  issue(0, 0);
  for (int kt = 0; kt < nkt; ++kt) step(kt, kt & 1);

  const float lt = l + __shfl_xor(l, 32);
  const float inv = lt > 0.f ? (DROP ? a.inv_keep : 1.f) / lt : 0.f;
  if (q < a.S) {
    store_dT<T>(static_cast<T*>(a.o) + (((int64_t)b * a.S + q) * a.H + hh) * kAD, o, hl, inv);
    if (hl == 0) a.lse[(int64_t)bh * a.lse_stride + q] = m + log2f(lt);
  }
}

// ---------------------------------------------------------------------------- backward
struct AttnBwdArgs {
  const void* q;
  const void* k;
  const void* v;
  const void* o;
  const void* dout;
  int64_t qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss, osh, dsb, dss, dsh;
  void* dq;
  void* dk;
  void* dv;
  int64_t dqsb, dqss, dqsh, dksb, dkss, dksh, dvsb, dvss, dvsh;
  const float* lse;  // [B][H][lse_stride] log2 units
  float* D;          // [B][H][lse_stride] rowsum(dO * O)
  int B, H, S, lse_stride;
  float scale, scale_log2;
  uint32_t thr8;
  float inv_keep;
  uint32_t seed;
};

// dK / dV: a workgroup owns 128 keys (32 per wave, one per lane column), loops
// over 64-query tiles.  Scores are computed unswapped, S[q][key] = Q . K^T with
// the wave's K^T / V^T fragments held in registers, so the 16 accumulator
// registers are 16 queries and dV^T = dO^T . P, dK^T = Q^T . dS consume P / dS
// straight from the accumulators (the MFMA sums over their register rows).  Q
// and dO tiles sit in LDS twice: a row image (A operand of S and dP) and a
// transposed-read image (A operand of dV^T / dK^T); the tile's lse / D values
// ride the same DMA ring (no plain global loads inside the loop, which would
// make the compiler's vmcnt waits drain the prefetch).
template <typename T, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kAT, 2) attn_bwd_dkdv_k(AttnBwdArgs a) {
  typedef typename Frag<T>::v8 v8;
  constexpr int IMG = kAKT * kARow;     // 8 KiB
  constexpr int BUF = 4 * IMG + 1024;   // Q rows, Q tr, dO rows, dO tr, {lse, D}
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform to the compiler
  const int hl = lane >> 5, c32 = lane & 31;
  int tile, bh;
  tile_of_block(CAUSAL, false, tile, bh);
  const int b = bh / a.H, hh = bh - b * a.H;
  const int kb0 = tile * 128;
  const int kw0 = kb0 + wid * 32;
  const int key = kw0 + c32;
  const int kk = key < a.S ? key : a.S - 1;
  // dropout lattice point of (query key & 3, this lane's key quad)
  const uint32_t kdrop = DROP ? drop_base(a.seed, (uint32_t)bh) + (uint32_t)(key >> 2) * kDropK +
                                    (uint32_t)(key & 3) * kDropQ
                              : 0u;
  const T* Q = static_cast<const T*>(a.q) + b * a.qsb + hh * a.qsh;
  const T* dO = static_cast<const T*>(a.dout) + b * a.dsb + hh * a.dsh;
  const float* lse = a.lse + (int64_t)bh * a.lse_stride;
  const float* Dr = a.D + (int64_t)bh * a.lse_stride;

  // K^T / V^T fragments (B operands): key = this lane's column, d = 16s + 8hl + j
  v8 kf[4], vf[4];
  {
    const T* K = static_cast<const T*>(a.k) + b * a.ksb + hh * a.ksh + (int64_t)kk * a.kss;
    const T* V = static_cast<const T*>(a.v) + b * a.vsb + hh * a.vsh + (int64_t)kk * a.vss;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = *reinterpret_cast<const v8*>(K + 16 * s + 8 * hl);
      vf[s] = *reinterpret_cast<const v8*>(V + 16 * s + 8 * hl);
    }
  }

  const int nqt = (a.S + kAKT - 1) / kAKT;
  const int qt0 = CAUSAL ? kb0 / kAKT : 0;
  const int lrow = lane >> 3, pch = lane & 7;
  auto issue = [&](int qt, int buf) {
    unsigned char* base = lds + buf * BUF;
    if (wid == 0) {  // lanes 0-15: lse[q0 .. q0+63], 16-31: D[...], 32-63: pad (lse again)
      const int seg = (lane >> 4) & 1, part = lane & 15;
      const float* src = (seg ? Dr : lse) + qt * kAKT + part * 4;
      glds16(src, base + 4 * IMG);
    }
    // (per-lane 64-bit addresses: the 32-bit offset form needs 8 more VGPRs here and
    // spilled at this kernel's ~250)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wid * 2 + i) * 8 + lrow;
      const int qr = qt * kAKT + row;
      const int qc = qr < a.S ? qr : a.S - 1;
      const int chr = (swz_rows(row, pch) - row * kARow) >> 4;
      const int cht = (swz_tr(row, pch) - row * kARow) >> 4;
      const T* qrow = Q + (int64_t)qc * a.qss;
      const T* drow = dO + (int64_t)qc * a.dss;
      unsigned char* dst = base + (wid * 2 + i) * 1024;
      glds16(qrow + chr * 8, dst);
      glds16(qrow + cht * 8, dst + IMG);
      glds16(drow + chr * 8, dst + 2 * IMG);
      glds16(drow + cht * 8, dst + 3 * IMG);
    }
  };

  f32x16_t dv[2], dk[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dv[0][i] = dv[1][i] = dk[0][i] = dk[1][i] = 0.f;

  int roff[2][4];  // [query half][d step]: row 32h + c32, chunk 2s + hl
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < 4; ++s) roff[h][s] = swz_rows(32 * h + c32, 2 * s + hl);
  int tlo[2][2][2], thi[2][2][2];  // [d tile][query half][k step]
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r0 = 32 * h + 16 * s + 4 * hl;
        const int c0 = 32 * dt + ((lane >> 4) & 1) * 16;
        tlo[dt][h][s] = tr_addr(r0, c0, lane);
        thi[dt][h][s] = tr_addr(r0 + 8, c0, lane);
      }

  if (qt0 < nqt) issue(qt0, 0);
  for (int qt = qt0; qt < nqt; ++qt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (qt + 1 < nqt) issue(qt + 1, (qt + 1 - qt0) & 1);
    const unsigned char* base = lds + ((qt - qt0) & 1) * BUF;
    const unsigned char* Qr = base;
    const unsigned char* Qt = base + IMG;
    const unsigned char* Or = base + 2 * IMG;
    const unsigned char* Ot = base + 3 * IMG;
    const float* st_lse = reinterpret_cast<const float*>(base + 4 * IMG);
    const float* st_D = st_lse + 64;
    const int q0 = qt * kAKT;
    // the four stages of one 32-query half h (S / dP products, softmax backward,
    // mask, dV / dK products)
    auto sdp = [&](int h, f32x16_t& sc, f32x16_t& dp) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] = dp[i] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc = mfma32<T>(lds_row8<T>(Qr, roff[h][s]), kf[s], sc);
        dp = mfma32<T>(lds_row8<T>(Or, roff[h][s]), vf[s], dp);
      }
    };
    auto softmax_bwd = [&](int h, f32x16_t& sc, f32x16_t& dp) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int li = 32 * h + 8 * g + 4 * hl;  // local query of register 4g
        const float4 lv = *reinterpret_cast<const float4*>(st_lse + li);
        const float4 dd = *reinterpret_cast<const float4*>(st_D + li);
        const float lsev[4] = {lv.x, lv.y, lv.z, lv.w};
        const float Dv[4] = {dd.x, dd.y, dd.z, dd.w};
        // keep bits: one hash covers a (query, key quad); the 4 lanes of a key quad
        // each hash one of the group's 4 queries (query li + (key & 3)) and read the
        // other three over DPP (quad_perm broadcast of lane e), so a lane computes ONE
        // hash per 4 queries
        uint32_t hq[4];
        if (DROP) {
          const uint32_t qhb = kdrop + (uint32_t)(q0 + 32 * h + 4 * hl) * kDropQ;
          const uint32_t v = drop_mix(qhb + (uint32_t)(8 * g) * kDropQ);
          hq[0] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);
          hq[1] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xF, 0xF, false);
          hq[2] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xF, 0xF, false);
          hq[3] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xF, 0xF, false);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          bool keep = true;
          if (DROP) keep = drop_keep8(hq[e], key & 3, a.thr8);
          float p = fexp2(fmaf(sc[r], a.scale_log2, -lsev[e]));
          // dropped dP scaled by 1/(1-p); the dropped P feeding dV^T is left unscaled
          // (the factor is applied to dV once, at the store)
          const float dpz = DROP ? (keep ? dp[r] * a.inv_keep : 0.f) : dp[r];
          sc[r] = (DROP && !keep) ? 0.f : p;
          dp[r] = p * (dpz - Dv[e]);
        }
      }
    };
    auto mask = [&](int h, f32x16_t& sc, f32x16_t& dp) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = q0 + 32 * h + 8 * (r >> 2) + 4 * hl + (r & 3);
        if (!(q < a.S && !(CAUSAL && key > q))) sc[r] = dp[r] = 0.f;
      }
    };
    auto accum = [&](int h, const f32x16_t& sc, const f32x16_t& dp) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const v8 pf = acc_frag<T>(sc, s);
        const v8 sf = acc_frag<T>(dp, s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma32<T>(lds_tr8<T>(Ot, tlo[dt][h][s], thi[dt][h][s]), pf, dv[dt]);
          dk[dt] = mfma32<T>(lds_tr8<T>(Qt, tlo[dt][h][s], thi[dt][h][s]), sf, dk[dt]);
        }
      }
    };
    // wave-uniform: no (query, key) of the whole 64 x 32 tile needs a mask - the
    // common case runs both halves as ONE straight-line block, so the compiler can
    // put half 1's S / dP MFMAs beside half 0's softmax VALU and half 0's dV / dK
    // MFMAs beside half 1's (a block split by a mask branch serialises them)
    const bool clean = (q0 + kAKT <= a.S) && (!CAUSAL || kw0 + 31 <= q0);
    if (clean) {
      f32x16_t sc0, dp0, sc1, dp1;
      sdp(0, sc0, dp0);
      sdp(1, sc1, dp1);
      softmax_bwd(0, sc0, dp0);
      accum(0, sc0, dp0);
      softmax_bwd(1, sc1, dp1);
      accum(1, sc1, dp1);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int qh0 = q0 + 32 * h;
        if (CAUSAL && qh0 + 31 < kw0) continue;  // every query of this half precedes every key
        f32x16_t sc, dp;
        sdp(h, sc, dp);
        softmax_bwd(h, sc, dp);
        // wave-uniform: does any (query, key) of this 32 x 32 block need a mask?
        if ((qh0 + 31 >= a.S) || (CAUSAL && kw0 + 31 > qh0)) mask(h, sc, dp);
        accum(h, sc, dp);
      }
    }
  }

  if (key < a.S) {
    store_dT<T>(static_cast<T*>(a.dv) + b * a.dvsb + (int64_t)key * a.dvss + hh * a.dvsh, dv, hl,
                DROP ? a.inv_keep : 1.f);
    store_dT<T>(static_cast<T*>(a.dk) + b * a.dksb + (int64_t)key * a.dkss + hh * a.dksh, dk, hl,
                a.scale);
  }
}

// dQ: a workgroup owns 128 queries (one per lane column), loops over 64-key
// tiles in the forward's swapped orientation S^T[key][q] = K . Q^T, so a lane's
// lse / D are scalars and dQ^T = K^T . dS^T consumes dS^T from the accumulator.
// K sits in LDS as a row image (A of S^T) and a transposed image (A of dQ^T);
// V as a row image (A of dP^T = V . dO^T).
template <typename T, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kAT, 2) attn_bwd_dq_k(AttnBwdArgs a) {
  typedef typename Frag<T>::v8 v8;
  constexpr int IMG = kAKT * kARow;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * 3 * IMG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform to the compiler
  const int hl = lane >> 5, c32 = lane & 31;
  int tile, bh;
  tile_of_block(CAUSAL, true, tile, bh);
  const int b = bh / a.H, hh = bh - b * a.H;
  const int qb0 = tile * 128;
  const int q = qb0 + wid * 32 + c32;
  const int qq = q < a.S ? q : a.S - 1;
  const uint32_t dbase = DROP ? drop_base(a.seed, (uint32_t)bh) + (uint32_t)q * kDropQ +
                                    (uint32_t)hl * kDropK
                              : 0u;
  const T* K = static_cast<const T*>(a.k) + b * a.ksb + hh * a.ksh;
  const T* V = static_cast<const T*>(a.v) + b * a.vsb + hh * a.vsh;

  v8 qf[4], of[4];
  {
    const T* Qp = static_cast<const T*>(a.q) + b * a.qsb + hh * a.qsh + (int64_t)qq * a.qss;
    const T* Op = static_cast<const T*>(a.dout) + b * a.dsb + hh * a.dsh + (int64_t)qq * a.dss;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = *reinterpret_cast<const v8*>(Qp + 16 * s + 8 * hl);
      of[s] = *reinterpret_cast<const v8*>(Op + 16 * s + 8 * hl);
    }
  }
  const float lse_q = a.lse[(int64_t)bh * a.lse_stride + qq];
  // D = rowsum(dO * O) of this lane's query, from the dO fragments already in
  // registers (the two 32-lane halves hold complementary d ranges); written for the
  // dK / dV kernel, which runs after this one (no separate preprocess launch)
  float D_q;
  {
    const T* Opr = static_cast<const T*>(a.o) + b * a.osb + hh * a.osh + (int64_t)qq * a.oss;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const v8 ov = *reinterpret_cast<const v8*>(Opr + 16 * s + 8 * hl);
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf((float)of[s][j], (float)ov[j], part);
    }
    D_q = part + __shfl_xor(part, 32);
    if (hl == 0 && q < a.S) a.D[(int64_t)bh * a.lse_stride + q] = D_q;
  }

  int nkt = (a.S + kAKT - 1) / kAKT;
  if (CAUSAL) {
    const int last = (qb0 + 127 < a.S ? qb0 + 127 : a.S - 1) / kAKT + 1;
    nkt = last < nkt ? last : nkt;
  }
  const int lrow = lane >> 3, pch = lane & 7;
  uint32_t kro[2], kto[2], vro[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wid * 2 + i) * 8 + lrow;
    const int chr = (swz_rows(row, pch) - row * kARow) >> 4;
    kro[i] = row_off<T>(row, a.kss, chr);
    kto[i] = row_off<T>(row, a.kss, (swz_tr(row, pch) - row * kARow) >> 4);
    vro[i] = row_off<T>(row, a.vss, chr);
  }
  // images per buffer: 0 = K rows, 1 = K transposed, 2 = V rows
  auto issue = [&](int kt, int buf) {
    unsigned char* base = lds + buf * 3 * IMG;
    if ((kt + 1) * kAKT <= a.S) {
      const T* kb = tile_base(K, kt * kAKT, a.kss);
      const T* vb = tile_base(V, kt * kAKT, a.vss);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        unsigned char* dst = base + (wid * 2 + i) * 1024;
        glds16o(kb, kro[i], dst);
        glds16o(kb, kto[i], dst + IMG);
        glds16o(vb, vro[i], dst + 2 * IMG);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wid * 2 + i) * 8 + lrow;
      const int kr = kt * kAKT + row;
      const int kc = kr < a.S ? kr : a.S - 1;
      const int chr = (swz_rows(row, pch) - row * kARow) >> 4;
      const int cht = (swz_tr(row, pch) - row * kARow) >> 4;
      const T* krow = K + (int64_t)kc * a.kss;
      unsigned char* dst = base + (wid * 2 + i) * 1024;
      glds16(krow + chr * 8, dst);
      glds16(krow + cht * 8, dst + IMG);
      glds16(V + (int64_t)kc * a.vss + chr * 8, dst + 2 * IMG);
    }
  };

  f32x16_t dq[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) dq[0][i] = dq[1][i] = 0.f;
  int koff[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) koff[t][s] = swz_rows(32 * t + c32, 2 * s + hl);
  int tlo[2][2][2], thi[2][2][2];  // [d tile][key half][k step]
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r0 = 32 * t + 16 * s + 4 * hl;
        const int c0 = 32 * dt + ((lane >> 4) & 1) * 16;
        tlo[dt][t][s] = tr_addr(r0, c0, lane);
        thi[dt][t][s] = tr_addr(r0 + 8, c0, lane);
      }

  issue(0, 0);
  for (int kt = 0; kt < nkt; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nkt) issue(kt + 1, (kt + 1) & 1);
    const unsigned char* base = lds + (kt & 1) * 3 * IMG;
    const unsigned char* Kr = base;
    const unsigned char* Kt = base + IMG;
    const unsigned char* Vr = base + 2 * IMG;
    const int k0 = kt * kAKT;
    if (CAUSAL && k0 > qb0 + wid * 32 + 31) continue;
    const uint32_t tb = dbase + (uint32_t)(k0 >> 2) * kDropK;
    // stages of one 32-key half t: S^T / dP^T products, dS^T, mask, dQ^T product
    auto sdp = [&](int t, f32x16_t& sc, f32x16_t& dp) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] = dp[i] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sc = mfma32<T>(lds_row8<T>(Kr, koff[t][s]), qf[s], sc);
        dp = mfma32<T>(lds_row8<T>(Vr, koff[t][s]), of[s], dp);
      }
    };
    auto dsoft = [&](int t, f32x16_t& sc, const f32x16_t& dp) {
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        uint32_t hsh = 0;
        // key quad (k0 + 32t + 8rq + 4hl) >> 2: a literal lattice step
        if (DROP) hsh = drop_mix(tb + (uint32_t)(8 * t + 2 * rq) * kDropK);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * rq + e;
          float dpr = dp[r];
          if (DROP) dpr = drop_keep8(hsh, e, a.thr8) ? dpr * a.inv_keep : 0.f;
          sc[r] = fexp2(fmaf(sc[r], a.scale_log2, -lse_q)) * (dpr - D_q);
        }
      }
    };
    auto mask = [&](int t, f32x16_t& sc) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (!(key < a.S && !(CAUSAL && key > q))) sc[r] = 0.f;
      }
    };
    auto accum = [&](int t, const f32x16_t& sc) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const v8 sf = acc_frag<T>(sc, s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          dq[dt] = mfma32<T>(lds_tr8<T>(Kt, tlo[dt][t][s], thi[dt][t][s]), sf, dq[dt]);
      }
    };
    f32x16_t sc0, dp0, sc1, dp1;
    sdp(0, sc0, dp0);
    sdp(1, sc1, dp1);
    // wave-uniform; unmasked tiles run as one straight-line block (half 0's dQ MFMAs
    // beside half 1's softmax VALU)
    const bool need_mask = (k0 + kAKT > a.S) || (CAUSAL && k0 + kAKT - 1 > qb0 + wid * 32);
    if (!need_mask) {
      dsoft(0, sc0, dp0);
      accum(0, sc0);
      dsoft(1, sc1, dp1);
      accum(1, sc1);
    } else {
      dsoft(0, sc0, dp0);
      dsoft(1, sc1, dp1);
      mask(0, sc0);
      mask(1, sc1);
      accum(0, sc0);
      accum(1, sc1);
    }
  }
  if (q < a.S)
    store_dT<T>(static_cast<T*>(a.dq) + b * a.dqsb + (int64_t)q * a.dqss + hh * a.dqsh, dq, hl,
                a.scale);
}

// host: the byte threshold of a dropout rate (round(256 p); p >= 255.5 / 256 drops all)
// keep decisions compare one hash byte with round(256 p): the rate is quantised to 1/256
// (ops/attention.py effective_dropout warns where that moves it by more than 2 %), and a
// rate below 1/512 still drops (threshold 1), never silently turns dropout off
static uint32_t drop_thr8(float p) {
  if (!(p > 0.f)) return 0u;
  const float t = p * 256.f + 0.5f;
  return t >= 256.f ? 256u : (t < 1.f ? 1u : (uint32_t)t);
}


}  // namespace

int attn_lse_stride(int S) { return (S + kAKT - 1) / kAKT * kAKT; }

void attn_fwd(const AttnLaunch& L, hipStream_t st) {
  AttnArgs a;
  a.q = L.q; a.k = L.k; a.v = L.v;
  a.qsb = L.qsb; a.qss = L.qss; a.qsh = L.qsh;
  a.ksb = L.ksb; a.kss = L.kss; a.ksh = L.ksh;
  a.vsb = L.vsb; a.vss = L.vss; a.vsh = L.vsh;
  a.o = L.o; a.lse = L.lse; a.B = L.B; a.H = L.H; a.S = L.S;
  a.lse_stride = L.lse_stride;
  a.scale_log2 = L.scale * 1.4426950408889634f;
  a.thr8 = drop_thr8(L.dropout);
  a.inv_keep = a.thr8 >= 256u ? 0.f : 256.f / (256.f - (float)a.thr8);
  a.seed = L.seed;
  dim3 grid((L.S + 127) / 128, L.B * L.H), block(kAT);
  const bool drop = a.thr8 != 0;
#define ATTN_FWD_LAUNCH(T)                                                                                \
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

void attn_bwd(const AttnBwdLaunch& L, hipStream_t st) {
  AttnBwdArgs a;
  a.q = L.q; a.k = L.k; a.v = L.v; a.o = L.o; a.dout = L.dout;
  a.qsb = L.qsb; a.qss = L.qss; a.qsh = L.qsh;
  a.ksb = L.ksb; a.kss = L.kss; a.ksh = L.ksh;
  a.vsb = L.vsb; a.vss = L.vss; a.vsh = L.vsh;
  a.osb = L.osb; a.oss = L.oss; a.osh = L.osh;
  a.dsb = L.dsb; a.dss = L.dss; a.dsh = L.dsh;
  a.dq = L.dq; a.dk = L.dk; a.dv = L.dv;
  a.dqsb = L.dqsb; a.dqss = L.dqss; a.dqsh = L.dqsh;
  a.dksb = L.dksb; a.dkss = L.dkss; a.dksh = L.dksh;
  a.dvsb = L.dvsb; a.dvss = L.dvss; a.dvsh = L.dvsh;
  a.lse = L.lse; a.D = L.D; a.lse_stride = L.lse_stride;
  a.B = L.B; a.H = L.H; a.S = L.S;
  a.scale = L.scale;
  a.scale_log2 = L.scale * 1.4426950408889634f;
  a.thr8 = drop_thr8(L.dropout);
  a.inv_keep = a.thr8 >= 256u ? 0.f : 256.f / (256.f - (float)a.thr8);
  a.seed = L.seed;
  dim3 grid((L.S + 127) / 128, L.B * L.H), block(kAT);
  const bool drop = a.thr8 != 0;
#define DQ_LAUNCH(T, C, D) hipLaunchKernelGGL((attn_bwd_dq_k<T, C, D>), grid, block, 0, st, a)
#define ATTN_BWD_LAUNCH(T)                                                                     \
  if (L.causal) {                                                                              \
    if (drop) {                                                                                \
      DQ_LAUNCH(T, true, true);                                                                \
      hipLaunchKernelGGL((attn_bwd_dkdv_k<T, true, true>), grid, block, 0, st, a);             \
    } else {                                                                                   \
      DQ_LAUNCH(T, true, false);                                                               \
      hipLaunchKernelGGL((attn_bwd_dkdv_k<T, true, false>), grid, block, 0, st, a);            \
    }                                                                                          \
  } else {                                                                                     \
    if (drop) {                                                                                \
      DQ_LAUNCH(T, false, true);                                                               \
      hipLaunchKernelGGL((attn_bwd_dkdv_k<T, false, true>), grid, block, 0, st, a);            \
    } else {                                                                                   \
      DQ_LAUNCH(T, false, false);                                                              \
      hipLaunchKernelGGL((attn_bwd_dkdv_k<T, false, false>), grid, block, 0, st, a);           \
    }                                                                                          \
  }
  if (L.dtype == DType::BF16) {
    ATTN_BWD_LAUNCH(bf16_t)
  } else {
    ATTN_BWD_LAUNCH(half_t)
  }
#undef ATTN_BWD_LAUNCH
#undef DQ_LAUNCH
}

}  // namespace amd
