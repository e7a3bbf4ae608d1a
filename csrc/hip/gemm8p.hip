// C[M, N] = A[M, K] . B[N, K]^T on the gfx950 matrix cores: a 256 x 256 workgroup tile,
// 8 wave64s (2 x 4, 128 x 64 accumulators each = 128 VGPRs), bf16 in / fp32 accumulate,
// with the K loop as 8 PHASES per two 64-deep K-tiles:
//
//   phase = { DMA one half-tile (2 glds per wave) | [counted vmcnt] | s_barrier |
//             ds_read the NEXT phase's fragments | 16 MFMAs (one 64 x 32 quadrant of the
//             wave's tile, K = 64) at raised priority | s_barrier }
//
// A tile's A and B operands live in LDS as four 16 KB half-tile regions - A_q0 / A_q1 (the
// wave rows of quadrant row 0 / 1) and B_n0 / B_n1 (quadrant column 0 / 1) - in two
// buffers (even / odd K-tiles): 128 KB.  Each region is read in exactly one phase (one
// phase ahead of the MFMAs that use it), so it can be refilled two phases later: the DMA
// of every region is issued >= 2 phases after its read, one region per phase, and only
// phases 4 and 8 wait - vmcnt(6): the three youngest regions stay in flight across the
// barrier.  Every region has ~4 phases (~2000 cycles of MFMA work at two waves per SIMD)
// to arrive, and no wave waits for vmcnt(0) inside the loop (the 2-barrier 128 x 128
// conv kernel's ceiling).
//
// LDS rows are 64 bf16 (128 B) with the 16-byte chunks XOR-swizzled by (row >> 1) & 7 on
// the DMA's SOURCE side (the DMA writes lane-linearly), so the 16 rows a ds_read_b128 lane
// group touches hit distinct bank slots.  Workgroups are remapped so the tiles of one
// A row panel run on one XCD (its 4 MB L2 then serves the panel to all of them).
//
// bf16 or fp16 operands (v_mfma_f32_16x16x32_bf16 / _f16).  Epilogues: plain store; bias + GELU with the pre-activation kept (the FFN
// input projection); dGELU from the saved pre-activation + the bias gradient's per-tile
// column sums (the FFN data gradient).  M may be ragged (zero-page rows); N % 256 == 0,
// K % 128 == 0.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kG8T = 512;       // threads
constexpr int kG8Half = 16384;  // one half-tile region: 128 rows x 128 B

// swizzle: logical 16-byte chunk c of region row r sits at physical chunk c ^ ((r >> 1) & 7)
__device__ __forceinline__ void g8_glds(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// s_barrier that the compiler may not move memory operations across (the raw builtin is
// not a memory barrier to it) and that waits for nothing: DMAs stay in flight
__device__ __forceinline__ void g8_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int g8_xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

__device__ __forceinline__ float g8_gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}
__device__ __forceinline__ float g8_gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float g8_dgelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
}
__device__ __forceinline__ float g8_dgelu_erf(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

template <typename T> struct G8T;
template <> struct G8T<bf16_t> {
  typedef bf16x8 v8;
  static __device__ __forceinline__ f32x4_t mma(v8 a, v8 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct G8T<half_t> {
  typedef f16x8 v8;
  static __device__ __forceinline__ f32x4_t mma(v8 a, v8 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <typename TT, int EPI, int SCHED>
__global__ void __launch_bounds__(kG8T, 1) gemm8p_k(G8Args p) {
  typedef typename G8T<TT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[8 * kG8Half];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR math
  const int wm = wid >> 2, wn = wid & 3;
  const int ntn = p.N >> 8;
  // XCD x runs a contiguous range of tile ids; within it the ids go down groups of
  // group_m m-tiles first, so the ~32 tiles an XCD runs at once form a group_m x 8 block
  // (group_m A panels + 8 B panels through its L2 per K-step instead of 1 + 32)
  const int bid = g8_xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  if (p.group_m > 1) {
    const int mt = gridDim.x / ntn, gsz = p.group_m * ntn, g = bid / gsz;
    const int first = g * p.group_m, rows = min(p.group_m, mt - first), r = bid - g * gsz;
    tm = first + r % rows;
    tn = r / rows;
  } else {
    tm = bid / ntn;
    tn = bid - tm * ntn;
  }
  const int m0 = tm * 256, n0 = tn * 256;
  const int KT = p.K >> 6;

  // DMA geometry: half-tile wave-instruction j = wid * 2 + i fills region rows j*8 .. j*8+7,
  // lane -> (row j*8 + lane/8, physical chunk lane%8) fetching the logical chunk that the
  // swizzle stores there.  Row rr = wid*16 + i*8 + lane/8 stays in one 64-row (A) / 32-row
  // (B) block for both i, so the region q / instruction i rows are the lane's base row plus
  // a uniform q*64 + i*8 (A) / q*32 + i*8 (B); the chunk of i = 1 is i = 0's ^ 4.  Only
  // the base rows and chunk offsets live in VGPRs - the fragments and accumulators need
  // 224 of the 256.  A rows past M re-read row M-1 (their outputs are never stored).
  const int lrow = lane >> 3, pch = lane & 7;
  const int rr0 = wid * 16 + lrow;
  const int ch0 = pch ^ ((rr0 >> 1) & 7);
  const int arow0 = m0 + (rr0 >> 6) * 128 + (rr0 & 63);
  const TT* __restrict__ Ab = static_cast<const TT*>(p.A);
  const TT* __restrict__ pB0 =
      static_cast<const TT*>(p.B) + (int64_t)(n0 + (rr0 >> 5) * 64 + (rr0 & 31)) * p.ldb;
  const int mlast = p.M - 1;

  // region r of buffer (T & 1): 0 = A_q0, 1 = A_q1, 2 = B_n0, 3 = B_n1.  Tiles past the end
  // re-fetch the last tile (into regions no longer read) so every phase issues the same
  // number of DMAs and the counted waits stay exact.
  auto stage = [&](int r, int T) {
    unsigned char* dst = lds + ((T & 1) * 4 + r) * kG8Half + wid * 2048;
    const int koff = (T < KT ? T : KT - 1) * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ch = (ch0 ^ (i * 4)) * 8 + koff;
      const TT* src;
      if (r < 2) {
        const int row = min(arow0 + r * 64 + i * 8, mlast);
        src = Ab + (int64_t)row * p.lda + ch;
      } else {
        src = pB0 + (int64_t)((r - 2) * 32 + i * 8) * p.ldb + ch;
      }
      g8_glds(src, dst + i * 1024);
    }
  };
  // one of stage()'s two wave-instructions, to place between MFMAs
  auto piece = [&](int r, int T, int i) {
    unsigned char* dst = lds + ((T & 1) * 4 + r) * kG8Half + wid * 2048;
    const int koff = (T < KT ? T : KT - 1) * 64;
    const int ch = (ch0 ^ (i * 4)) * 8 + koff;
    const TT* src;
    if (r < 2) src = Ab + (int64_t)min(arow0 + r * 64 + i * 8, mlast) * p.lda + ch;
    else src = pB0 + (int64_t)((r - 2) * 32 + i * 8) * p.ldb + ch;
    g8_glds(src, dst + i * 1024);
  };

  // fragment reads: row wm*64 + i*16 + fr (A) has swizzle key (fr >> 1) & 7 for every i,
  // so each (operand, k-step) needs one lane offset and the rest are immediates
  const int fr = lane & 15, fg = lane >> 4, fx = (fr >> 1) & 7;
  const int offA0 = (wm * 64 + fr) * 128 + ((fg ^ fx) << 4);
  const int offA1 = (wm * 64 + fr) * 128 + (((4 + fg) ^ fx) << 4);
  const int offB0 = (wn * 32 + fr) * 128 + ((fg ^ fx) << 4);
  const int offB1 = (wn * 32 + fr) * 128 + (((4 + fg) ^ fx) << 4);
  v8 a0[4][2], a1[4][2], b0[2][2], b1[2][2];
  auto readA = [&](int buf, int q, v8 (&a)[4][2]) {
    const unsigned char* R = lds + (buf * 4 + q) * kG8Half;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i][0] = *reinterpret_cast<const v8*>(R + offA0 + i * 2048);
      a[i][1] = *reinterpret_cast<const v8*>(R + offA1 + i * 2048);
    }
  };
  auto readB = [&](int buf, int q, v8 (&b)[2][2]) {
    const unsigned char* R = lds + (buf * 4 + 2 + q) * kG8Half;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b[j][0] = *reinterpret_cast<const v8*>(R + offB0 + j * 2048);
      b[j][1] = *reinterpret_cast<const v8*>(R + offB1 + j * 2048);
    }
  };

  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#define G8_MMA_K(QM, QN, AR, BR, KS)                                                    \
  {                                                                                     \
    __builtin_amdgcn_s_setprio(1);                                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                       \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                       \
      acc[QM][QN][i][j] = G8T<TT>::mma(AR[i][KS], BR[j][KS], acc[QM][QN][i][j]);         \
    __builtin_amdgcn_s_setprio(0);                                                      \
  }
#define G8_MMA(QM, QN, AR, BR) \
  G8_MMA_K(QM, QN, AR, BR, 0)  \
  G8_MMA_K(QM, QN, AR, BR, 1)

  if constexpr (SCHED == 1) {
    // Barrier every second phase ("pair schedule"): each barrier is preceded by
    // lgkmcnt(0) (the previous phases' fragment reads retired) and vmcnt(8), and followed
    // by two regions' DMA.  Reads: A_q0 / B_n0 of a tile in the last phase of the tile
    // before, B_n1 in its first, A_q1 in its second phase.  A region read in the phase
    // pair before barrier k is restaged right after barrier k; every region has three
    // phase pairs (~6 x 512 MFMA cycles per SIMD) to land before the barrier that
    // precedes its read.
    stage(0, 0);
    stage(2, 0);
    stage(3, 0);
    stage(1, 0);
    stage(0, 1);
    stage(2, 1);
    stage(3, 1);
    stage(1, 1);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    g8_barrier();
    readA(0, 0, a0);
    readB(0, 0, b0);
#define G8_SYNC()                                           \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");          \
  g8_barrier();
// one quadrant in four 4-MFMA chunks; P0 / P1 after chunks 0 / 1 (a DMA piece each, which
// costs ~60 issue cycles on its own: placed between MFMAs the partner wave's MFMAs hide
// it), READS after chunk 1 (fragments for the next quadrant)
#define G8_QUAD(QM, QN, AR, BR, P0, P1, READS)                                           \
  _Pragma("unroll") for (int c = 0; c < 4; ++c) {                                       \
    __builtin_amdgcn_s_setprio(1);                                                      \
    _Pragma("unroll") for (int ii = 0; ii < 2; ++ii)                                    \
    _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                     \
      const int i = (c & 1) * 2 + ii, ks = c >> 1;                                      \
      acc[QM][QN][i][j] = G8T<TT>::mma(AR[i][ks], BR[j][ks], acc[QM][QN][i][j]);         \
    }                                                                                   \
    __builtin_amdgcn_s_setprio(0);                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    if (c == 0) { P0; }                                                                 \
    if (c == 1) { P1; READS; }                                                          \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  }
    for (int t = 0; t < KT; t += 2) {
      G8_SYNC();
      G8_QUAD(0, 0, a0, b0, piece(0, t + 2, 0), piece(0, t + 2, 1), readB(0, 1, b1));
      G8_QUAD(0, 1, a0, b1, piece(2, t + 2, 0), piece(2, t + 2, 1), readA(0, 1, a1));
      G8_SYNC();
      G8_QUAD(1, 0, a1, b0, piece(3, t + 2, 0), piece(3, t + 2, 1), (void)0);
      G8_QUAD(1, 1, a1, b1, piece(1, t + 2, 0), piece(1, t + 2, 1),
              (readA(1, 0, a0), readB(1, 0, b0)));
      G8_SYNC();
      G8_QUAD(0, 0, a0, b0, piece(0, t + 3, 0), piece(0, t + 3, 1), readB(1, 1, b1));
      G8_QUAD(0, 1, a0, b1, piece(2, t + 3, 0), piece(2, t + 3, 1), readA(1, 1, a1));
      G8_SYNC();
      G8_QUAD(1, 0, a1, b0, piece(3, t + 3, 0), piece(3, t + 3, 1), (void)0);
      G8_QUAD(1, 1, a1, b1, piece(1, t + 3, 0), piece(1, t + 3, 1),
              (readA(0, 0, a0), readB(0, 0, b0)));
    }
#undef G8_SYNC
#undef G8_QUAD
  } else {
    // Each phase reads the fragments of the NEXT phase, so their LDS latency runs under
    // MFMAs; per tile the quadrants go (0,0),
    // (0,1), (1,0), (1,1), which lets phase 4 / 8 fetch the next tile's A_q0 / B_n0 into
    // the registers phases 1-3 are done with.  Region reads (r = tile's buffer): A_q0, B_n0
    // in the phase before the tile, B_n1 in its phase 1, A_q1 in phase 2.  Each region is
    // re-staged >= 2 phases after its read (retired by the next phase's lgkmcnt wait before
    // that phase's closing barrier); a tile's four regions are issued four consecutive
    // phases, and the waits at phases 4 / 8 leave the 3 youngest regions (6 glds) in flight.
    // The reads go between a phase's two K-steps: the compiler then waits (lgkmcnt(0)) only
    // for the previous phase's reads before the first MFMA, never for the new ones.
    // prologue: tile 0 complete, tile 1's A_q0 / B_n0 / B_n1 in flight
    stage(0, 0);
    stage(2, 0);
    stage(3, 0);
    stage(1, 0);
    stage(0, 1);
    stage(2, 1);
    stage(3, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    g8_barrier();
    readA(0, 0, a0);
    readB(0, 0, b0);

    for (int t = 0; t < KT; t += 2) {
      // ---------------- tile t (buffer 0)
      stage(1, t + 1);  // phase 1
      g8_barrier();
      G8_MMA_K(0, 0, a0, b0, 0);
      __builtin_amdgcn_sched_barrier(0);
      readB(0, 1, b1);
      __builtin_amdgcn_sched_barrier(0);
      G8_MMA_K(0, 0, a0, b0, 1);
      g8_barrier();
      stage(0, t + 2);  // phase 2
      g8_barrier();
      G8_MMA_K(0, 1, a0, b1, 0);
      __builtin_amdgcn_sched_barrier(0);
      readA(0, 1, a1);
      __builtin_amdgcn_sched_barrier(0);
      G8_MMA_K(0, 1, a0, b1, 1);
      g8_barrier();
      stage(2, t + 2);  // phase 3
      g8_barrier();
      G8_MMA(1, 0, a1, b0);
      g8_barrier();
      stage(3, t + 2);  // phase 4: retire tile t+1, fetch its first fragments
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      g8_barrier();
      G8_MMA_K(1, 1, a1, b1, 0);
      __builtin_amdgcn_sched_barrier(0);
      readA(1, 0, a0);
      readB(1, 0, b0);
      __builtin_amdgcn_sched_barrier(0);
      G8_MMA_K(1, 1, a1, b1, 1);
      g8_barrier();
      // ---------------- tile t+1 (buffer 1)
      stage(1, t + 2);  // phase 5
      g8_barrier();
      G8_MMA_K(0, 0, a0, b0, 0);
      __builtin_amdgcn_sched_barrier(0);
      readB(1, 1, b1);
      __builtin_amdgcn_sched_barrier(0);
      G8_MMA_K(0, 0, a0, b0, 1);
      g8_barrier();
      stage(0, t + 3);  // phase 6
      g8_barrier();
      G8_MMA_K(0, 1, a0, b1, 0);
      __builtin_amdgcn_sched_barrier(0);
      readA(1, 1, a1);
      __builtin_amdgcn_sched_barrier(0);
      G8_MMA_K(0, 1, a0, b1, 1);
      g8_barrier();
      stage(2, t + 3);  // phase 7
      g8_barrier();
      G8_MMA(1, 0, a1, b0);
      g8_barrier();
      stage(3, t + 3);  // phase 8: retire tile t+2, fetch its first fragments
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      g8_barrier();
      G8_MMA_K(1, 1, a1, b1, 0);
      __builtin_amdgcn_sched_barrier(0);
      readA(0, 0, a0);
      readB(0, 0, b0);
      __builtin_amdgcn_sched_barrier(0);
      G8_MMA_K(1, 1, a1, b1, 1);
      g8_barrier();
    }
  }
#undef G8_MMA
#undef G8_MMA_K
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: accumulators -> bf16 tile in LDS (the whole 128 KB) -> 16-byte row stores
  TT* T = reinterpret_cast<TT*>(lds);
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = wm * 128 + qm * 64 + i * 16 + fg * 4 + e;
            const int col = wn * 64 + qn * 32 + j * 16 + fr;
            float v = acc[qm][qn][i][j][e];
            if constexpr (EPI == 1) {  // bias before the one rounding, as addmm does
              if (p.bias)
                v += p.bias_f32 ? static_cast<const float*>(p.bias)[n0 + col]
                                : (float)static_cast<const TT*>(p.bias)[n0 + col];
            }
            T[row * 256 + col] = (TT)v;
          }
  __syncthreads();
  // each thread: one 8-column chunk (fixed for all its rows: 512 % 32 == 0) of 16 rows
  const int cc = tid & 31, rg = tid >> 5;
  TT* Cp = static_cast<TT*>(p.C);
  TT* auxp = static_cast<TT*>(p.aux);
  const int col0 = n0 + cc * 8;
  float colsum[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) colsum[k] = 0.f;
  // all 16 LDS rows first (one lgkmcnt wait), then the stores / epilogue math
  v8 rv[256 / (kG8T / 32)];
#pragma unroll
  for (int q = 0; q < 256 / (kG8T / 32); ++q)
    rv[q] = *reinterpret_cast<const v8*>(T + (rg + q * (kG8T / 32)) * 256 + cc * 8);
#pragma unroll
  for (int q = 0; q < 256 / (kG8T / 32); ++q) {
    const int row = rg + q * (kG8T / 32);
    const int gm = m0 + row;
    if (gm >= p.M) continue;
    const v8 v = rv[q];
    if constexpr (EPI == 0) {
      *reinterpret_cast<v8*>(Cp + (int64_t)gm * p.ldc + col0) = v;
    } else {
      float x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (float)v[k];
      if constexpr (EPI == 1) {
        // pre = acc + bias (one rounding, as the unfused addmm), h = gelu(pre)
        v8 h;
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = (TT)(p.tanh ? g8_gelu_tanh(x[k]) : g8_gelu_erf(x[k]));
        if (auxp) *reinterpret_cast<v8*>(auxp + (int64_t)gm * p.ldc + col0) = v;
        *reinterpret_cast<v8*>(Cp + (int64_t)gm * p.ldc + col0) = h;
      } else {
        // dpre = dh * gelu'(pre), dh = this GEMM's output rounded to bf16; bias gradient
        // partial sums of the bf16-rounded dpre
        const v8 pre = *reinterpret_cast<const v8*>(auxp + (int64_t)gm * p.ldc + col0);
        v8 d;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float pf = (float)pre[k];
          const TT db = (TT)(x[k] * (p.tanh ? g8_dgelu_tanh(pf) : g8_dgelu_erf(pf)));
          d[k] = db;
          colsum[k] += (float)db;
        }
        *reinterpret_cast<v8*>(Cp + (int64_t)gm * p.ldc + col0) = d;
      }
    }
  }
  if constexpr (EPI == 2) {
    if (p.colsum) {
      // the 16 row groups of each column chunk through LDS, one row of the [Mtiles][N]
      // partial-sum slab per workgroup (fixed order: deterministic)
      __syncthreads();
      float* red = reinterpret_cast<float*>(lds);
#pragma unroll
      for (int k = 0; k < 8; ++k) red[rg * 256 + cc * 8 + k] = colsum[k];
      __syncthreads();
      if (tid < 256) {
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < kG8T / 32; ++g) s += red[g * 256 + tid];
        p.colsum[(int64_t)tm * p.N + n0 + tid] = s;
      }
    }
  }
}

}  // namespace

bool gemm8p_supported(int M, int N, int K) {
  return M > 0 && N > 0 && N % 256 == 0 && K >= 128 && K % 128 == 0;
}

int gemm8p_mtiles(int M) { return (M + 255) / 256; }

// APEX_AMD_G8_SCHED: 1 = barrier every second phase (default), 0 = two barriers per phase
static int g8_sched() {
  static const int v = [] {
    const char* e = std::getenv("APEX_AMD_G8_SCHED");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

// APEX_AMD_G8_GROUPM: m-tiles per tile-order group (default 4; 1 = row-major tile order)
static int g8_group_m() {
  static const int v = [] {
    const char* e = std::getenv("APEX_AMD_G8_GROUPM");
    return e ? std::max(1, std::atoi(e)) : 4;
  }();
  return v;
}

void gemm8p(const G8Args& a0, int epi, hipStream_t st) {
  G8Args a = a0;
  a.group_m = g8_group_m();
  const int grid = gemm8p_mtiles(a.M) * (a.N / 256);
  auto launch = [&](auto t0, auto s0) {
    using TT = decltype(t0);
    constexpr int S = decltype(s0)::value;
    if (epi == 1)
      hipLaunchKernelGGL((gemm8p_k<TT, 1, S>), dim3(grid), dim3(kG8T), 0, st, a);
    else if (epi == 2)
      hipLaunchKernelGGL((gemm8p_k<TT, 2, S>), dim3(grid), dim3(kG8T), 0, st, a);
    else
      hipLaunchKernelGGL((gemm8p_k<TT, 0, S>), dim3(grid), dim3(kG8T), 0, st, a);
  };
  auto go = [&](auto t0) {
    if (g8_sched() == 1) launch(t0, std::integral_constant<int, 1>{});
    else launch(t0, std::integral_constant<int, 0>{});
  };
  if (a.fp16) go(half_t{});
  else go(bf16_t{});
}

}  // namespace amd
