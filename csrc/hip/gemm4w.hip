// C[M, N] = A[M, K] . B[N, K]^T on the gfx950 matrix cores with ONE wave per SIMD: a
// 256 x 256 workgroup tile, 4 wave64s (2 x 2), a 128 x 128 fp32 accumulator per wave
// (64 MFMA tiles of 16 x 16 = 256 accumulator registers), bf16 / fp16 in.
//
// Why this shape (docs/PERF.md, round 4 PMC comparison): an 8-wave 128 x 64-per-wave
// kernel (round 4's gemm8p, removed in round 6) reads 1.5x the LDS bytes per MFMA of a
// 128 x 128-per-wave tile and its two waves per SIMD spent ~29 % of their cycles parked in
// s_waitcnt / s_barrier.
// Here each wave owns its SIMD's matrix pipe: per 32-deep k-step it reads 8 A + 8 B
// fragments (16 ds_read_b128, 16 KB per wave) for 64 MFMAs, i.e. 1/4 KB of LDS per
// 16x16x32 MFMA instead of 3/8 KB.
//
// K loop (64-deep K-tiles, two LDS slots of 64 KB = A 32 KB + B 32 KB, 128-byte rows
// with a (row >> 1) & 7 XOR swizzle of the 16-byte chunks applied on the DMA's source
// side):
//
//   k-step 0 of tile t: 64 MFMAs on F0 (registers)   | read F1 (tile t, k 32..63)
//   k-step 1 of tile t: lgkmcnt(0); vmcnt(0) (tile t+1 landed); s_barrier;
//                       64 MFMAs on F1               | read F0 (tile t+1, k 0..31)
//                                                    | DMA tile t+2 into tile t's slot
//
// Fragments are register double-buffered (F0 / F1, 64 VGPRs each), so the LDS reads of
// a step run under the previous step's MFMAs; the MFMAs go out in groups of 4 with one
// fragment read and (k-step 1) one DMA piece between groups, pinned by sched_barrier.
// A tile's DMA is issued one K-tile ahead (2 k-steps = 128 MFMAs of lead) and retired
// by ONE vmcnt(0) + s_barrier per K-tile.  Tiles past the end re-fetch the last tile
// into the slot no longer read, so every K-tile issues the same instruction stream.
//
// The MFMA takes B as its first operand, so each accumulator holds C^T: a lane owns 4
// CONSECUTIVE columns of one row, written to the LDS output tile as one 8-byte store
// (rows padded to 528 B: conflict-free), instead of 4 two-byte stores.  Epilogues:
// plain store; bias + GELU keeping the pre-activation; dGELU from the saved
// pre-activation + the bias gradient's per-tile column sums.
//
// M may be ragged (rows past M re-read row M-1 and are never stored); N % 256 == 0,
// K % 64 == 0.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int uint4_t __attribute__((ext_vector_type(4)));

constexpr int kW4T = 256;             // threads: 4 waves, one per SIMD
constexpr int kW4Op = 32768;          // one operand of one K-tile: 256 rows x 128 B
constexpr int kW4Slot = 2 * kW4Op;    // A + B

__device__ __forceinline__ void w4_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int w4_xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

__device__ __forceinline__ float w4_gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float w4_dgelu_erf(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// The MFMA as inline asm with the accumulator TIED in AGPRs ("+a"): the builtin form
// lets the register allocator pick a destination other than srcC, and with 256
// accumulator registers (the whole AGPR file) it then shuffles accumulators through
// VGPRs and scratch every iteration (520 v_accvgpr moves + 33 spilled VGPRs per K-tile
// in the first build).  No hazard padding is needed inside the loop: an accumulator is
// re-used 64 MFMAs later, and a fragment register is rewritten >= 8 MFMA groups after
// its last MFMA read; the epilogue starts behind s_nop padding (w4_mfma_drain).
// (B, A) operand order: the accumulator is C^T (row index from B, column index from A).
template <typename T> struct W4T;
template <> struct W4T<bf16_t> {
  typedef bf16x8 v8;
  static __device__ __forceinline__ void mma(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  }
  // C = 0: the first k-step of an output tile (no zeroing pass, and every definition of
  // the accumulators is an AGPR asm output, so they never migrate to VGPRs)
  static __device__ __forceinline__ void mma0(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  }
};
template <> struct W4T<half_t> {
  typedef f16x8 v8;
  static __device__ __forceinline__ void mma(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  }
  static __device__ __forceinline__ void mma0(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  }
};

// wait states between the last MFMA and the first VALU read of its accumulators (the
// compiler cannot see inside the asm): 4 x 8 >= the 16x16x32 write -> read requirement
__device__ __forceinline__ void w4_mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

// LDS row swizzle: the 16-byte chunk c of row R sits at physical chunk c ^ w4_key(R).
// Conflict-free for the 16-row ds_read_b128 lane groups of both fragment orders used
// below (A rows in natural order; B rows permuted, see w4_brow) - found by exhaustive
// search over XOR keys of row bits 1..4.
__device__ __forceinline__ int w4_key(int R) { return ((R >> 1) & 7) ^ (((R >> 4) & 1) << 1); }

// B fragment j's MFMA row r (the C column it produces) maps to LDS row
// (j >> 1) * 32 + (r >> 2) * 8 + (j & 1) * 4 + (r & 3) of the wave's 128-row B panel, so
// the lane (r = fr, fg) of fragments 2p and 2p+1 holds the 8 CONSECUTIVE columns
// p*32 + fg*8 .. +7 of its C row: one 16-byte store per (row block i, pair p).
__device__ __forceinline__ int w4_brow(int par, int fr) {
  return (fr >> 2) * 8 + par * 4 + (fr & 3);
}

// tanh-GELU as x * sigmoid(2u), u = k0 (x + k1 x^3): one v_exp, one v_rcp and 4 VALU per
// value (the libm tanhf is ~40 VALU, and at one wave per SIMD nothing hides the epilogue)
constexpr float kGk0 = 0.7978845608028654f, kGk1 = 0.044715f, kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float w4_sig2u(float x, float x2) {  // sigmoid(2u)
  const float z = x * fmaf(x2, -2.f * kGk0 * kGk1 * kLog2e, -2.f * kGk0 * kLog2e);  // -2u log2 e
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}
__device__ __forceinline__ float w4_gelu_t(float x) { return x * w4_sig2u(x, x * x); }
// d/dx x s(x) = s + x s (1 - s) 2u', 2u' = 2 k0 (1 + 3 k1 x^2)
__device__ __forceinline__ float w4_dgelu_t(float x) {
  const float x2 = x * x, sg = w4_sig2u(x, x2);
  return fmaf(x * sg * (1.f - sg), fmaf(6.f * kGk0 * kGk1, x2, 2.f * kGk0), sg);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t w4_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// One output tile per workgroup.  Measured and removed (round 5, profiles/r5/gemm4w_bench.md):
// a persistent grid walking tiles b, b + G, ... as one flattened K-tile stream (1-4 %
// slower: tile bookkeeping and spills around the in-loop epilogue cost more than the
// prologues it hid), k-half LDS regions (5-6 % slower), two DMA pieces per MFMA group
// (5-11 % slower), two fragment reads per group (within +-3 %).
// TANH: the GELU flavour of EPI 1 / 2 (tanh approximation, else erf).
template <typename TT, int EPI, bool TANH>
__global__ void __launch_bounds__(kW4T, 1) gemm4w_k(GemmArgs p) {
  typedef typename W4T<TT>::v8 v8;
  // the ring + 2 KB for the bias-gradient column sums of EPI 2 (4 KB: the two statistics
  // sums of EPI 3)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * kW4Slot + (EPI == 3 ? 4096 : 2048)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = p.N >> 8, mtiles = (p.M + 255) >> 8;
  const int b = w4_xcd_remap(blockIdx.x, gridDim.x);
  const int KT = p.K >> 6;
  const int gm_ = p.group_m;
  // this workgroup's tile -> (m0, n0) in the grouped order (group_m m-tiles x ntn)
  auto tile_mn = [&](int& m0, int& n0) {
    const int id = b;
    int tm, tn;
    if (gm_ > 1) {
      const int gsz = gm_ * ntn, g = id / gsz;
      const int first = g * gm_, rows = min(gm_, mtiles - first), rr = id - g * gsz;
      tm = first + rr % rows;
      tn = rr / rows;
    } else {
      tm = id / ntn;
      tn = id - tm * ntn;
    }
    m0 = tm * 256;
    n0 = tn * 256;
  };

  // DMA: buffer loads straight into LDS (buffer_load_dwordx4 ... lds): a wave-uniform
  // descriptor per operand panel, the K-tile's byte offset in soffset, a per-lane voffset
  // - no per-load VALU (the flat form cost a 64-bit v_lshl_add_u64 per piece in the MFMA
  // issue stream).  Wave w fills rows w*64 .. w*64+63 of each operand as 8
  // wave-instructions of 8 rows: lane -> (row + lane/8, physical chunk lane%8) fetching
  // the logical chunk the swizzle stores there.
  const int lrow = lane >> 3, pch = lane & 7;
  uint32_t offA[8], offB[8];
  int tm0, tn0;
  tile_mn(tm0, tn0);
  // operand panels of the tile (wave-uniform descriptors, per-lane 32-bit offsets)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rr = wid * 64 + i * 8 + lrow;
    const int ch = pch ^ w4_key(i * 8 + lrow);
    const int ar = min(tm0 + rr, p.M - 1) - tm0;  // rows past M re-read row M-1
    offA[i] = (uint32_t)ar * (uint32_t)p.lda * (uint32_t)sizeof(TT) + (uint32_t)ch * 16u;
    offB[i] = (uint32_t)rr * (uint32_t)p.ldb * (uint32_t)sizeof(TT) + (uint32_t)ch * 16u;
  }
  const __amdgpu_buffer_rsrc_t rA = w4_rsrc(static_cast<const TT*>(p.A) + (int64_t)tm0 * p.lda, 0xffffffffu);
  const __amdgpu_buffer_rsrc_t rB = w4_rsrc(static_cast<const TT*>(p.B) + (int64_t)tn0 * p.ldb, 0xffffffffu);
  // the 16 pieces (8 A + 8 B wave-instructions) of K-tile T go to slot T & 1; past the
  // end the last K-tile is re-fetched into the free slot (uniform stream).  ld_next()
  // steps the load cursor by one K-tile
  int ld_kb = 0, ld_T = 0;
  auto ld_next = [&]() {
    if (ld_T + 1 >= KT) return;  // keep re-fetching the last K-tile
    ++ld_T;
    ld_kb = ld_T * 128;  // byte offset of the K-tile in a row
  };
  auto piece = [&](int T, int q) {
    unsigned char* dst = lds + (T & 1) * kW4Slot + (q >> 3) * kW4Op + wid * 8192 + (q & 7) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 8 ? rA : rB,
                                             (__attribute__((address_space(3))) void*)dst, 16,
                                             q < 8 ? offA[q] : offB[q - 8], ld_kb, 0, 0);
  };

  // fragment reads: A row wm*128 + i*16 + fr; B row w4_brow; logical chunk ks*4 + fg;
  // the key depends on the fragment's parity (row bit 4 for A, the +4 for B)
  const int fr = lane & 15, fg = lane >> 4;
  int offRA[2][2], offRB[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int ra = par * 16 + fr, rb = w4_brow(par, fr);
      offRA[ks][par] = ra * 128 + (((ks * 4 + fg) ^ w4_key(ra)) << 4);
      offRB[ks][par] = rb * 128 + (((ks * 4 + fg) ^ w4_key(rb)) << 4);
    }
  v8 fa0[8], fb0[8], fa1[8], fb1[8];
  // n-th read of a k-step, in the order the next k-step's MFMA groups consume them
  // (group g uses A[g / 2] and B[(g & 1) * 4 .. +3]): B0-3, A0, B4-7, A1 .. A7.  LDS reads
  // return in order, so each group's counted lgkmcnt wait covers only reads issued >= 8
  // groups earlier (in natural order B4-7 came last and stalled every k-step's start).
  auto rd_order = [](int n) { return n < 4 ? 8 + n : n == 4 ? 0 : n < 9 ? 7 + n : n - 8; };
  // read one fragment (r < 8: A[r], else B[r - 8]) of k-step ks of the tile in `slot`
  auto rd = [&](int slot, int ks, int r, v8(&fa)[8], v8(&fb)[8]) {
    const unsigned char* base = lds + slot * kW4Slot;
    if (r < 8) {
      fa[r] = *reinterpret_cast<const v8*>(base + offRA[ks][r & 1] + (wm * 128 + (r & 6) * 16) * 128);
    } else {
      const int j = r - 8;
      fb[j] = *reinterpret_cast<const v8*>(base + kW4Op + offRB[ks][j & 1] +
                                           (wn * 128 + (j >> 1) * 32) * 128);
    }
  };

  f32x4_t acc[8][8];  // defined by the first k-step of each tile (mma0)

  // ---- epilogue of one output tile, straight from the accumulators: lane (fr, fg) holds,
  // for row block i and column pair q, the 8 consecutive columns wn*128 + q*32 + fg*8 ..
  // +7 of row wm*128 + i*16 + fr (C^T accumulators of B fragments 2q, 2q+1).  Buffer
  // stores against a descriptor that ends at row M: rows past M are dropped by the
  // hardware, so every store instruction issues.
  float* red = reinterpret_cast<float*>(lds + 2 * kW4Slot);
  auto epilogue = [&](int m0, int n0) {
    const uint32_t rows = (uint32_t)min(256, p.M - m0);
    const uint32_t cbytes = (uint32_t)(rows - 1) * (uint32_t)p.ldc * sizeof(TT) + (uint32_t)p.N * sizeof(TT);
    const __amdgpu_buffer_rsrc_t rC = w4_rsrc(static_cast<TT*>(p.C) + (int64_t)m0 * p.ldc, cbytes);
    const __amdgpu_buffer_rsrc_t rX =
        w4_rsrc(p.aux ? static_cast<TT*>(p.aux) + (int64_t)m0 * p.ldc : p.C, p.aux ? cbytes : 0u);
    const int ccol = wn * 128 + fg * 8;  // + q * 32
    float bias[4][8];
    if constexpr (EPI == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = n0 + ccol + q * 32 + e;
          bias[q][e] = !p.bias ? 0.f
                       : p.bias_f32 ? static_cast<const float*>(p.bias)[c]
                                    : (float)static_cast<const TT*>(p.bias)[c];
        }
    }
    if constexpr (EPI == 3) {
      // BatchNorm statistics of the stored (rounded) output for the BN that consumes C
      // (1x1 conv forward): per column, sum(v - s) and sum((v - s)^2) over the tile's
      // rows.  Column block q at a time (16 live sums, not 64): rows i in-lane, the 16
      // lanes fr by DPP row reductions (fixed order), the two wm waves through LDS; one
      // channel-major slab entry per (column, M-tile), as conv_tap_k's epilogue writes.
      float* red3 = reinterpret_cast<float*>(lds + 2 * kW4Slot);  // [sum][wm][256]
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float sh[8], s1[8], s2[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sh[e] = p.shift ? p.shift[n0 + ccol + q * 32 + e] : 0.f;
          s1[e] = s2[e] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = wm * 128 + i * 16 + fr;
          const bool in = m0 + row < p.M;
          v8 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = (TT)acc[i][2 * q][e];
            v[4 + e] = (TT)acc[i][2 * q + 1][e];
          }
          const uint32_t off = ((uint32_t)row * (uint32_t)p.ldc + (uint32_t)(n0 + ccol + q * 32)) * sizeof(TT);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, v), rC, off, 0, 0);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = in ? (float)v[e] - sh[e] : 0.f;
            s1[e] += d;
            s2[e] = fmaf(d, d, s2[e]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float a = s1[e], b = s2[e];
#define W4_ROWSUM(v_)                                                                                  \
  v_ += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v_), 0xB1, 0xf, 0xf, true)); \
  v_ += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v_), 0x4E, 0xf, 0xf, true)); \
  v_ += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v_), 0x141, 0xf, 0xf, true)); \
  v_ += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v_), 0x140, 0xf, 0xf, true));
          W4_ROWSUM(a)
          W4_ROWSUM(b)
#undef W4_ROWSUM
          if (fr == 0) {
            red3[wm * 256 + ccol + q * 32 + e] = a;
            red3[512 + wm * 256 + ccol + q * 32 + e] = b;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      w4_barrier();
      const int S = (p.M + 255) >> 8, tm = m0 >> 8;
      p.slab[(int64_t)(n0 + tid) * S + tm] = red3[tid] + red3[256 + tid];
      p.slab[(int64_t)(p.N + n0 + tid) * S + tm] = red3[512 + tid] + red3[768 + tid];
      return;
    }
    float colsum[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) colsum[q][e] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wm * 128 + i * 16 + fr;
      const bool in = m0 + row < p.M;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float x[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = acc[i][2 * q][e];
          x[4 + e] = acc[i][2 * q + 1][e];
        }
        const uint32_t off = ((uint32_t)row * (uint32_t)p.ldc + (uint32_t)(n0 + ccol + q * 32)) * sizeof(TT);
        v8 v;
        if constexpr (EPI == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (TT)(x[e] + bias[q][e]);  // one rounding
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (TT)x[e];
        }
        if constexpr (EPI == 0) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, v), rC, off, 0, 0);
        } else if constexpr (EPI == 1) {
          // pre = acc + bias rounded once (kept as aux); h = gelu(pre) of the rounded pre
          v8 h;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float pf = (float)v[e];
            h[e] = (TT)(TANH ? w4_gelu_t(pf) : w4_gelu_erf(pf));
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, v), rX, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, h), rC, off, 0, 0);
        } else {
          // dpre = dh * gelu'(pre), dh = this GEMM's output rounded; column sums of the
          // rounded dpre for the bias gradient (rows past M read 0 and add 0)
          const v8 pre = __builtin_bit_cast(v8, __builtin_amdgcn_raw_buffer_load_b128(rX, off, 0, 0));
          v8 d;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float pf = (float)pre[e];
            const TT db = (TT)((float)v[e] * (TANH ? w4_dgelu_t(pf) : w4_dgelu_erf(pf)));
            d[e] = db;
            colsum[q][e] += in ? (float)db : 0.f;
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, d), rC, off, 0, 0);
        }
      }
      // one row block at a time: the next tile's F0 fragments are live across the
      // epilogue, so the accumulator reads must not all be hoisted
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (EPI == 2) {
      if (p.colsum) {
        // sum over the 16 lanes fr of each column (DPP: quad swaps, half-row and row
        // mirrors; a fixed order), then the two wm waves through 2 KB of LDS
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float v = colsum[q][e];
            v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, true));
            v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, true));
            v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xf, 0xf, true));
            v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xf, 0xf, true));
            colsum[q][e] = v;
          }
        if (fr == 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) red[wm * 256 + ccol + q * 32 + e] = colsum[q][e];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        w4_barrier();
        const int tm = m0 >> 8;
        p.colsum[(int64_t)tm * p.N + n0 + tid] = red[tid] + red[256 + tid];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        w4_barrier();  // red is rewritten by the next tile's epilogue
      }
    }
  };

  // prologue: K-tiles 0 and 1 in flight, wait for K-tile 0, read its k-step-0 fragments
#pragma unroll
  for (int q = 0; q < 16; ++q) piece(0, q);
  ld_next();
#pragma unroll
  for (int q = 0; q < 16; ++q) piece(1, q);
  ld_next();  // the cursor now names K-tile 2 (issued by k-step 1 of K-tile 0)
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  w4_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) rd(0, 0, rd_order(r), fa0, fb0);

  // MFMA group g of a k-step: rows i = g / 2, columns j = (g & 1) * 4 .. +3
#define W4_GROUP(FA, FB, g)                                                  \
  _Pragma("unroll") for (int jj = 0; jj < 4; ++jj) {                         \
    const int i_ = (g) >> 1, j_ = ((g) & 1) * 4 + jj;                        \
    W4T<TT>::mma(FA[i_], FB[j_], acc[i_][j_]);                               \
  }
#define W4_GROUP0(FA, FB, g)                                                 \
  _Pragma("unroll") for (int jj = 0; jj < 4; ++jj) {                         \
    const int i_ = (g) >> 1, j_ = ((g) & 1) * 4 + jj;                        \
    W4T<TT>::mma0(FA[i_], FB[j_], acc[i_][j_]);                              \
  }

  // one flattened K-tile t: k-step 0 (FIRST: a tile's first K-tile starts the
  // accumulators from zero) reading F1, then k-step 1 reading the next K-tile's F0 and
  // issuing K-tile t+2's DMA
  auto ktile = [&](int t, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    const int slot = t & 1;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if constexpr (FIRST) {
        W4_GROUP0(fa0, fb0, g);
      } else {
        W4_GROUP(fa0, fb0, g);
      }
      __builtin_amdgcn_sched_barrier(0);
      rd(slot, 1, rd_order(g), fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // k-step 1: K-tile t+1 must have landed (every wave's DMA: vmcnt + barrier), and every
    // wave's reads of this slot are retired before K-tile t+2's DMA overwrites it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    w4_barrier();
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      W4_GROUP(fa1, fb1, g);
      __builtin_amdgcn_sched_barrier(0);
      rd(slot ^ 1, 0, rd_order(g), fa0, fb0);
      piece(t + 2, g);
      __builtin_amdgcn_sched_barrier(0);
    }
    ld_next();  // K-tile t+3, for the next K-tile's k-step 1
  };

  ktile(0, std::true_type{});
  for (int kt = 1; kt < KT; ++kt) ktile(kt, std::false_type{});
  w4_mfma_drain();
  epilogue(tm0, tn0);
#undef W4_GROUP
#undef W4_GROUP0
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool gemm4w_supported(int M, int N, int K) {
  return M > 0 && N > 0 && N % 256 == 0 && K >= 64 && K % 64 == 0;
}

void gemm4w(const GemmArgs& a0, int epi, hipStream_t st) {
  GemmArgs a = a0;
  a.group_m = 4;  // XCD-grouped tile order: 4 m-tiles per group (measured best, round 5)
  const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
  auto launch = [&](auto t0, auto tanh_c) {
    using TT = decltype(t0);
    constexpr bool TH = decltype(tanh_c)::value;
    if (epi == 0)
      hipLaunchKernelGGL((gemm4w_k<TT, 0, false>), dim3(ntiles), dim3(kW4T), 0, st, a);
    else if (epi == 3)
      hipLaunchKernelGGL((gemm4w_k<TT, 3, false>), dim3(ntiles), dim3(kW4T), 0, st, a);
    else if (epi == 1)
      hipLaunchKernelGGL((gemm4w_k<TT, 1, TH>), dim3(ntiles), dim3(kW4T), 0, st, a);
    else
      hipLaunchKernelGGL((gemm4w_k<TT, 2, TH>), dim3(ntiles), dim3(kW4T), 0, st, a);
  };
  auto go = [&](auto t0) {
    if (a.tanh) launch(t0, std::true_type{});
    else launch(t0, std::false_type{});
  };
  if (a.fp16) go(half_t{});
  else go(bf16_t{});
}

}  // namespace amd
