// 3x3 / stride-1 / pad-1 convolution on channels-last bf16 as an implicit GEMM
// on the gfx950 matrix cores (v_mfma_f32_16x16x32_bf16).
//
//   y[m, co] = sum_{r,s,ci} x[n, h+r-1, w+s-1, ci] * W[co, r, s, ci]
//   GEMM: M = N*H*W output pixels, N = Cout, K = 9*Cin; A = im2col(x) built on
//   the fly (zero rows for the padding), B = W in KRSC order (= PyTorch's
//   channels_last weight layout).  The data gradient of the same conv is the
//   same kernel on dY with the weights rotated by 180 degrees and Cin/Cout
//   swapped (ops/conv.py).
//
// Tiling (MI355X-first, not a CUDA warp tiling): a 256-thread workgroup = 4
// wave64s computes a BM=128 pixel x BN (64|128) output tile; each K-tile is one
// filter tap x 64 input channels (BK = 64 = one 128-byte row per pixel).
// Operands go HBM -> LDS directly with global_load_lds (16 B per lane, one
// 1 KiB wave-instruction = 8 tile rows), through a ring of NB LDS buffers:
// the DMA of tile t+NB-1 is in flight while tile t is multiplied, retired by a
// counted `s_waitcnt vmcnt` + raw s_barrier (never vmcnt(0) in the loop).  The
// padding halo is a lane whose source address points at a zeroed 16-byte
// global, so no lane ever branches.  LDS rows carry a (row>>1)&7 XOR swizzle of
// their 16-byte chunks (applied on the SOURCE side of the DMA, since the DMA
// writes lane-linearly), so the 16 rows a ds_read_b128 lane group touches land
// in distinct bank slots.  Workgroups are remapped so consecutive M tiles
// (which share input rows through the 3x3 halo) run on one XCD's L2.
#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kCT = 256;  // threads
constexpr int kBM = 128;
constexpr int kBK = 64;
constexpr int kRowBytes = kBK * 2;  // 128

__device__ uint4 g_zero16[4];  // zero source for the padding halo (static storage: zeroed)

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * kRowBytes + ((chunk ^ ((row >> 1) & 7)) << 4);
}

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// bijective blockIdx -> tile remap keeping consecutive tiles on one XCD
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

template <int BN, int WM, int WN, int NB>
__global__ void __launch_bounds__(kCT, 2)
    conv3x3_fwd_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wt,
                  bf16_t* __restrict__ y, int N, int H, int W, int Cin, int Cout, int M) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = kBM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = kBM * kRowBytes, B_BYTES = BN * kRowBytes;
  constexpr int BUF = A_BYTES + B_BYTES;
  constexpr int AI = kBM / 32;      // A wave-instructions (8 rows each) per wave per tile
  constexpr int BI = BN / 32;       // B wave-instructions per wave per tile
  constexpr int G = AI + BI;        // glds per wave per tile (vmcnt units)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NB * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int mt = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = mt * kBM, n0 = blockIdx.y * BN;
  const int HW = H * W;

  // DMA lane geometry: wave `wid` fills A rows [wid*32, wid*32+32) as AI
  // instructions of 8 rows; lane -> (row = base + lane/8, physical chunk lane%8)
  // fetching the logical chunk that the swizzle stores at that position.
  const int lrow = lane >> 3, pchunk = lane & 7;
  int an[AI], ah[AI], aw[AI], ach[AI];
  bool aval[AI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    const int row = wid * (kBM / 4) + q * 8 + lrow;
    ach[q] = pchunk ^ ((row >> 1) & 7);
    const int m = m0 + row;
    aval[q] = m < M;
    const int mm = aval[q] ? m : 0;
    an[q] = mm / HW;
    const int rem = mm - an[q] * HW;
    ah[q] = rem / W;
    aw[q] = rem - ah[q] * W;
  }
  int bco[BI], bch[BI];
#pragma unroll
  for (int q = 0; q < BI; ++q) {
    const int row = wid * (BN / 4) + q * 8 + lrow;
    bch[q] = pchunk ^ ((row >> 1) & 7);
    bco[q] = n0 + row;
  }
  const int kc_per_tap = Cin / kBK;
  const int KT = 9 * kc_per_tap;

#define CONV_ISSUE(kt_)                                                                     \
  {                                                                                         \
    const int tap_ = (kt_) / kc_per_tap;                                                    \
    const int c0_ = ((kt_) - tap_ * kc_per_tap) * kBK;                                      \
    const int dr_ = tap_ / 3 - 1, ds_ = tap_ % 3 - 1;                                       \
    unsigned char* A_ = lds + ((kt_) % NB) * BUF;                                           \
    unsigned char* B_ = A_ + A_BYTES;                                                       \
    _Pragma("unroll") for (int q = 0; q < AI; ++q) {                                        \
      const int hh = ah[q] + dr_, ww = aw[q] + ds_;                                         \
      const bool ok = aval[q] && hh >= 0 && hh < H && ww >= 0 && ww < W;                    \
      const bf16_t* src = x + (((int64_t)an[q] * H + hh) * W + ww) * Cin + c0_ + ach[q] * 8; \
      glds16(ok ? (const void*)src : (const void*)g_zero16,                                 \
             A_ + (wid * (kBM / 4) + q * 8) * kRowBytes);                                   \
    }                                                                                       \
    _Pragma("unroll") for (int q = 0; q < BI; ++q) {                                        \
      const bf16_t* src = wt + ((int64_t)bco[q] * 9 + tap_) * Cin + c0_ + bch[q] * 8;       \
      glds16(src, B_ + (wid * (BN / 4) + q * 8) * kRowBytes);                               \
    }                                                                                       \
  }

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;

  // prologue: NB-1 tiles in flight
#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < KT) CONV_ISSUE(p);

  for (int kt = 0; kt < KT; ++kt) {
    // retire tile kt: leave the (NB-2) younger tiles' DMAs in flight
    if (kt + NB - 2 < KT) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (NB - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    // the buffer of tile kt+NB-1 was last read at iteration kt-1: every wave has
    // passed this barrier, so it is free
    if (kt + NB - 1 < KT) CONV_ISSUE(kt + NB - 1);
    const unsigned char* A = lds + (kt % NB) * BUF;
    const unsigned char* B = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fg;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + swz(wm * TM + i * 16 + fr, ch));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(B + swz(wn * TN + j * 16 + fr, ch));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
#undef CONV_ISSUE
  __syncthreads();

  // epilogue: accumulators -> bf16 tile in LDS -> coalesced 16-byte row stores
  bf16_t* T = reinterpret_cast<bf16_t*>(lds);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * TM + i * 16 + fg * 4 + e;
        const int col = wn * TN + j * 16 + fr;
        T[row * BN + col] = (bf16_t)acc[i][j][e];
      }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-byte chunks per output row
  for (int c = tid; c < kBM * CPR; c += kCT) {
    const int row = c / CPR, cc = c - row * CPR;
    const int m = m0 + row;
    if (m < M)
      *reinterpret_cast<uint4*>(y + (int64_t)m * Cout + n0 + cc * 8) =
          *reinterpret_cast<const uint4*>(T + row * BN + cc * 8);
  }
}

}  // namespace

bool conv3x3_nhwc_supported(int Cin, int Cout) { return Cin % 64 == 0 && Cout % 64 == 0; }

void conv3x3_nhwc_fwd(const void* x, const void* w, void* y, int N, int H, int W, int Cin,
                      int Cout, hipStream_t st) {
  const int M = N * H * W;
  if (M == 0) return;
  const int mtiles = (M + kBM - 1) / kBM;
  const auto* xp = static_cast<const bf16_t*>(x);
  const auto* wp = static_cast<const bf16_t*>(w);
  auto* yp = static_cast<bf16_t*>(y);
  if (Cout % 128 == 0) {
    hipLaunchKernelGGL((conv3x3_fwd_k<128, 2, 2, 2>), dim3(mtiles, Cout / 128), dim3(kCT), 0, st,
                       xp, wp, yp, N, H, W, Cin, Cout, M);
  } else {
    hipLaunchKernelGGL((conv3x3_fwd_k<64, 4, 1, 3>), dim3(mtiles, Cout / 64), dim3(kCT), 0, st,
                       xp, wp, yp, N, H, W, Cin, Cout, M);
  }
}

}  // namespace amd
