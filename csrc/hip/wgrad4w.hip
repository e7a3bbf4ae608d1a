// Weight gradients of the dense layers on the gfx950 matrix cores, one wave per SIMD:
//
//   P[s][m][n] = sum over rows k of split s of  A[k][m] * B[k][n]
//
// with A = dY [T, M] and B = X [T, N] both stored ROW-major over the token dimension T
// (dW = dY^T X, the reduction runs down the columns of both operands).  fp32 partials per
// split s, summed by the slab reduction (splitk_reduce) that also writes the weight dtype.
//
// Why: hipBLASLt's split-K batched GEMM tops out near 1.0 PF on these shapes (BERT-large
// 4096 x 1024 x 16384: 137 us at its best split, TunableOp's online search included,
// profiles/r5/wgrad_dense.md), while the same tile / K structure in the TN layout runs at
// 1.43 PF on gemm4w.hip.  This kernel is gemm4w's K loop (256 x 256 workgroup tile, 4
// waves of 128 x 128 fp32 accumulators, 64-deep K-tiles on a 2-deep LDS ring, buffer-
// descriptor LDS DMA, fragments of the next k-step read under the current MFMAs, one
// barrier per k-step) with operands that arrive K-major: the MFMA fragments (8
// consecutive k of one column per lane) come from ds_read_b64_tr_b16 transposed reads.
//
// LDS image of one operand K-tile (64 rows k x 256 columns, 32 KB): 32 blocks of 1 KB,
// block (row group r >> 4, chunk group c >> 2) holds 16 rows x 4 16-byte chunks, row-major
// inside the block with the chunk index XORed by 2 on odd 8-row halves:
//
//   byte(r, c) = ((r >> 4) * 8 + (c >> 2)) * 1024 + ((r & 15) * 4 + ((c & 3) ^ (((r >> 3) & 1) << 1))) * 16
//
// One DMA wave-instruction fills one block (lanes 4 i .. 4 i + 3 read 64 contiguous bytes
// of row i: coalesced), and every 32-lane half of a transposed fragment read (rows
// kb .. kb+3 and kb+8 .. kb+11 of two chunks) lands on 16 distinct 16-byte bank slots:
// conflict-free (MI355X_MICROARCH.md LDS table: ds_read_b64_tr_b16 banks per 32 lanes).
//
// The MFMA takes the X fragment as its first operand, so the accumulator lane (fr, fg)
// holds 4 CONSECUTIVE n of one m: one 16-byte fp32 store each.
//
// Measured and removed in round 6 (round-5 A/Bs, all bitwise equal to this layout): 8-row x
// 128-byte and whole-row DMA blocks (within 1-5 %), and the slot released per HALF K-tile
// so a DMA piece gets 1.5 K-tiles to land (within -3..+2 % on every BERT / GPT-2 shape,
// profiles/r5/wgrad_dense/variant3_sweep.txt: the load slack was not the limit).
//
// Status (round 5, profiles/r5/wgrad_dense.md): BERT-large FFN weight gradient 114.5 us
// (1.20 PF, reduction included) vs 136.8 us for hipBLASLt's best split; one workgroup runs
// a K-tile in 1.15 us against 0.85 us of MFMA issue.  The first build ran 3.3 us per K-tile
// whatever the load: with the LDS-DMA as a builtin the compiler put an s_waitcnt vmcnt(0)
// in front of every transposed read (the DMA writes LDS, the tr-read builtin carries no
// alias information), i.e. the loop waited out the full memory latency of the next
// K-tile's DMA at every MFMA group.  The DMA is inline asm now (ww_dma).
//
// M % 256 == 0, N % 256 == 0, rows per split % 64 == 0.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int uint4_t __attribute__((ext_vector_type(4)));
typedef short v4s_t __attribute__((ext_vector_type(4)));

constexpr int kWwT = 256;            // threads: 4 waves, one per SIMD
constexpr int kWwOp = 32768;         // one operand of one K-tile
constexpr int kWwSlot = 2 * kWwOp;   // A + B

__device__ __forceinline__ void ww_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int ww_xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ww_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// tied-accumulator MFMA (see gemm4w.hip: the builtin lets the allocator shuffle the 256
// accumulator registers); first operand X (n), second dY (m): acc = P^T per 16 x 16 tile
template <typename T> struct WwT;
template <> struct WwT<bf16_t> {
  typedef bf16x8 v8;
  static __device__ __forceinline__ void mma(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  }
  static __device__ __forceinline__ void mma0(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  }
};
template <> struct WwT<half_t> {
  typedef f16x8 v8;
  static __device__ __forceinline__ void mma(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  }
  static __device__ __forceinline__ void mma0(v8 a, v8 b, f32x4_t& c) {
    asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  }
};

__device__ __forceinline__ void ww_mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

// One LDS-DMA wave-instruction (16 bytes per lane into M0 + 16 * lane) as inline asm: the
// compiler does not see it write LDS, so it does not wait for every outstanding DMA piece
// (vmcnt(0)) in front of each ds_read_b64_tr_b16 - with the builtin form it did, which
// serialised the K loop on the full memory latency (3.3 us per K-tile for ONE workgroup).
// The loop orders DMA and fragment reads itself: explicit vmcnt(0) + s_barrier before a
// slot is read, lgkmcnt(0) + s_barrier before it is overwritten.
__device__ __forceinline__ void ww_dma(__amdgpu_buffer_rsrc_t r, uint32_t lds_addr, uint32_t voff,
                                       uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(r), "s"(soff), "{m0}"(lds_addr)
               : "memory");
}

// 8 consecutive k of one column: the two transposed 4-row reads at byte offsets lo, lo+HI
template <typename V8, int HI>
__device__ __forceinline__ V8 ww_frag(const unsigned char* p) {
  const v4s_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)p);
  const v4s_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(p + HI));
  V8 f;
  v4s_t* fp = reinterpret_cast<v4s_t*>(&f);
  fp[0] = a;
  fp[1] = b;
  return f;
}

// column sums of A from the dY fragments (variant 4, p.colsum: the dense layer's bias
// gradient without a separate pass over dY): lane l holds 8 k of column l & 15 of
// fragment i; one v_dot2 with (1, 1) per bf16 / f16 pair adds it exactly in fp32.  The pairs
// are taken with __builtin_shufflevector: a bit_cast of the fragment to a dword vector
// indexed inside the unrolled loop made this compiler read the same register three times
template <typename TT, typename V8>
__device__ __forceinline__ float ww_sum8(V8 f, float acc) {
  if constexpr (std::is_same<TT, half_t>::value) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 one = {(_Float16)1.0f, (_Float16)1.0f};
    acc = __builtin_amdgcn_fdot2(__builtin_shufflevector(f, f, 0, 1), one, acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_shufflevector(f, f, 2, 3), one, acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_shufflevector(f, f, 4, 5), one, acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_shufflevector(f, f, 6, 7), one, acc, false);
  } else {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    const b2 one = {(__bf16)1.0f, (__bf16)1.0f};
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 0, 1), one, acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 2, 3), one, acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 4, 5), one, acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(f, f, 6, 7), one, acc, false);
  }
  return acc;
}

// CS: with the column sums of A (p.colsum)
template <typename TT, bool CS>
__global__ void __launch_bounds__(kWwT, 1) wgrad4w_k(WgradArgs p) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass only needs the launch stub)
  typedef typename WwT<TT>::v8 v8;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * kWwSlot];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int mt = p.M >> 8, nt = p.N >> 8, per_split = mt * nt;
  const int b = ww_xcd_remap(blockIdx.x, gridDim.x);
  const int s = b / per_split;
  int r = b - s * per_split;
  // grouped order inside a split: group_m m-tiles x all n-tiles
  int tm, tn;
  {
    const int gm = p.group_m, gsz = gm * nt, g = r / gsz;
    const int first = g * gm, rows = min(gm, mt - first), rr = r - g * gsz;
    tm = first + rr % rows;
    tn = rr / rows;
  }
  const int m0 = tm * 256, n0 = tn * 256;
  const int KT = p.rows >> 6;
  const int64_t k0 = (int64_t)s * p.rows;

  // DMA: wave w fills blocks (row group w, chunk group cg = 0..7) of each operand; lane
  // (i = lane >> 2, j = lane & 3) reads row 16 w + i, chunk cg*4 + (j ^ 2 (i >> 3 & 1)).
  // The K-tile and the chunk group go into the (scalar) soffset.
  const int drow = wid * 16 + (lane >> 2);
  const int dch = (lane & 3) ^ (((lane >> 5) & 1) << 1);
  const uint32_t offA = (uint32_t)drow * (uint32_t)p.lda * (uint32_t)sizeof(TT) + (uint32_t)dch * 16u;
  const uint32_t offB = (uint32_t)drow * (uint32_t)p.ldb * (uint32_t)sizeof(TT) + (uint32_t)dch * 16u;
  const __amdgpu_buffer_rsrc_t rA =
      ww_rsrc(static_cast<const TT*>(p.A) + k0 * p.lda + m0, 0xffffffffu);
  const __amdgpu_buffer_rsrc_t rB =
      ww_rsrc(static_cast<const TT*>(p.B) + k0 * p.ldb + n0, 0xffffffffu);
  const uint32_t strideA = 64u * (uint32_t)p.lda * (uint32_t)sizeof(TT);  // one K-tile
  const uint32_t strideB = 64u * (uint32_t)p.ldb * (uint32_t)sizeof(TT);
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;
  // piece q (0..7 A, 8..15 B) of K-tile T (clamped: past the end the last K-tile is
  // re-fetched into the free slot, so every K-tile issues the same stream)
  auto piece = [&](int T, int q) {
    const int Tc = T < KT ? T : KT - 1;
    const int qq = q & 7;
    const uint32_t cgo = (uint32_t)qq * 64u;
    const uint32_t dst = lds_base + (uint32_t)((T & 1) * kWwSlot + (q >> 3) * kWwOp + (wid * 8 + qq) * 1024);
    if (q < 8) {
      ww_dma(rA, dst, offA, (uint32_t)Tc * strideA + cgo);
    } else {
      ww_dma(rB, dst, offB, (uint32_t)Tc * strideB + cgo);
    }
  };

  // transposed fragment reads: lane (q = (lane & 15) >> 2, p1 = lane >> 1 & 1, p0 = lane & 1,
  // fg = lane >> 4) of fragment i (columns 16 i .. of the wave's 128) at k-step ks: rows
  // ks*32 + fg*8 + q (+4 for the second read), chunk 2 i + p1, byte 8 p0: a lane base
  // per parity of i
  const int fq = (lane & 15) >> 2, fp1 = (lane >> 1) & 1, fp0 = lane & 1, fg = lane >> 4;
  constexpr int HI = 256;  // byte distance of rows +4
  int lb[2];
#pragma unroll
  for (int ip = 0; ip < 2; ++ip)
    lb[ip] = (fg >> 1) * 8 * 1024 + ((fg & 1) * 8 + fq) * 64 +
             (((2 * ip + fp1) ^ ((fg & 1) << 1)) << 4) + 8 * fp0;
  v8 fa0[8], fb0[8], fa1[8], fb1[8];
  // n-th read of a k-step in the order the next k-step's groups consume them (group g:
  // A[g / 2] with B[(g & 1) * 4 .. +3]): B0-3, A0, B4-7, A1 .. A7
  auto rd_order = [](int n) { return n < 4 ? 8 + n : n == 4 ? 0 : n < 9 ? 7 + n : n - 8; };
  auto frag_off = [&](int i, int w) { return lb[i & 1] + w * 4096 + (i >> 1) * 1024; };
  auto rd = [&](int slot, int ks, int n, v8(&fa)[8], v8(&fb)[8]) {
    const unsigned char* base = lds + slot * kWwSlot + ks * 16384;
    if (n < 8) {
      fa[n] = ww_frag<v8, HI>(base + frag_off(n, wm));
    } else {
      const int j = n - 8;
      fb[j] = ww_frag<v8, HI>(base + kWwOp + frag_off(j, wn));
    }
  };

  f32x4_t acc[8][8];
  float csum[CS ? 8 : 1];
  if constexpr (CS) {
#pragma unroll
    for (int i = 0; i < 8; ++i) csum[i] = 0.f;
  }

  // prologue: K-tiles 0 and 1 in flight, K-tile 0 landed, its k-step-0 fragments read
#pragma unroll
  for (int q = 0; q < 16; ++q) piece(0, q);
#pragma unroll
  for (int q = 0; q < 16; ++q) piece(1, q);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  ww_barrier();
#pragma unroll
  for (int n = 0; n < 16; ++n) rd(0, 0, rd_order(n), fa0, fb0);

#define WW_GROUP(FA, FB, g, OP)                                              \
  _Pragma("unroll") for (int jj = 0; jj < 4; ++jj) {                         \
    const int i_ = (g) >> 1, j_ = ((g) & 1) * 4 + jj;                        \
    WwT<TT>::OP(FA[i_], FB[j_], acc[i_][j_]);                                \
  }

  // one K-tile: k-step 0 on F0 while F1 (k 32..63 of this K-tile) is read; then K-tile
  // t+1 must have landed (its DMA went out during k-step 1 of K-tile t-1) and every wave's
  // reads of this slot retired, so K-tile t+2 may overwrite it; k-step 1 on F1 while F0 of
  // K-tile t+1 is read and K-tile t+2's DMA goes out
  auto ktile = [&](int t, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    const int slot = t & 1;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if constexpr (FIRST) {
        WW_GROUP(fa0, fb0, g, mma0);
      } else {
        WW_GROUP(fa0, fb0, g, mma);
      }
      if constexpr (CS) {
        if ((g & 1) == 0) csum[g >> 1] = ww_sum8<TT>(fa0[g >> 1], csum[g >> 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      rd(slot, 1, rd_order(g), fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ww_barrier();
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      WW_GROUP(fa1, fb1, g, mma);
      if constexpr (CS) {
        if ((g & 1) == 0) csum[g >> 1] = ww_sum8<TT>(fa1[g >> 1], csum[g >> 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      rd(slot ^ 1, 0, rd_order(g), fa0, fb0);
      piece(t + 2, g);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  ktile(0, std::true_type{});
  for (int t = 1; t < KT; ++t) ktile(t, std::false_type{});
#undef WW_GROUP
  ww_mfma_drain();

  // epilogue: lane (fr, fg) of acc[i][j] holds P[m0 + wm*128 + 16 i + fr][n0 + wn*128 +
  // 16 j + 4 fg .. +3]: one 16-byte store per (i, j)
  const int fr = lane & 15;
  float* P = p.P + (int64_t)s * p.M * p.N;
  const __amdgpu_buffer_rsrc_t rP = ww_rsrc(P + (int64_t)m0 * p.N + n0,
                                            (uint32_t)(255 * p.N + 256) * 4u);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t row = (uint32_t)(wm * 128 + i * 16 + fr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t off = (row * (uint32_t)p.N + (uint32_t)(wn * 128 + j * 16 + fg * 4)) * 4u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_t, acc[i][j]), rP, off, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (CS) {
    // the 4 k-groups of a column sit in lanes l, l ^ 16, l ^ 32, l ^ 48; the n-tile 0
    // workgroup's wn == 0 waves write their 128 columns (every n-tile forms the same sums)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = csum[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      csum[i] = v;
    }
    if (tn == 0 && wn == 0 && lane < 16) {
      float* cp = p.colsum + (int64_t)s * p.M + m0 + wm * 128 + lane;
#pragma unroll
      for (int i = 0; i < 8; ++i) cp[i * 16] = csum[i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
  (void)p;
#endif
}

}  // namespace

bool wgrad4w_supported(int64_t T, int M, int N, int S) {
  return M > 0 && N > 0 && M % 256 == 0 && N % 256 == 0 && S >= 1 && T % ((int64_t)S * 64) == 0 &&
         T / S >= 64 && T / S < (1 << 24) &&
         (int64_t)T * std::max(M, N) * 2 < ((int64_t)1 << 32) &&
         (int64_t)M * N * 4 < ((int64_t)1 << 32);
}

void wgrad4w(const WgradArgs& a0, hipStream_t st) {
  WgradArgs a = a0;
  // XCD-grouped tile order, 4 m-tiles per group (1 to 16 measured within 3 %, round 5)
  if (a.group_m <= 0) a.group_m = 4;
  const int grid = (a.M / 256) * (a.N / 256) * a.S;
  auto go = [&](auto t0) {
    using TT = decltype(t0);
    if (a.colsum)
      hipLaunchKernelGGL((wgrad4w_k<TT, true>), dim3(grid), dim3(kWwT), 0, st, a);
    else
      hipLaunchKernelGGL((wgrad4w_k<TT, false>), dim3(grid), dim3(kWwT), 0, st, a);
  };
  if (a.fp16) go(half_t{});
  else go(bf16_t{});
}

}  // namespace amd
