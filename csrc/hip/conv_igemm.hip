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


// ============================================================================
// Weight gradient: dW[co, r, s, ci] = sum_p dY[p, co] * x[shift_rs(p), ci].
// Per tap (r, s) a GEMM with rows = co, cols = ci and K = output pixels, split
// over pixel ranges (grid.y) for parallelism; fp32 partials [split][tap][co][ci]
// are summed by wgrad_reduce_k.  Both operands arrive pixel-major ([k][col]), so
// the MFMA fragments (8 consecutive k per lane) are read with ds_read_b64_tr_b16
// transposed reads from LDS images whose 16-byte chunks carry a row swizzle that
// keeps each 32-lane half of a transposed read conflict-free (8 rows apart,
// 2 chunks each -> 16 distinct bank slots).
typedef short v4s_t __attribute__((ext_vector_type(4)));

template <int RB>  // row bytes: 128 or 256
__device__ __forceinline__ int tr_swz(int row, int chunk) {
  if constexpr (RB == 256) {
    return row * 256 + ((chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
  } else {
    return row * 128 + ((chunk ^ ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1)) << 4);
  }
}

// 8 consecutive k (rows kb..kb+7) of column (c0 + lane&15) as an MFMA fragment
template <int RB>
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* T, int kb, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;               // element column of this lane's 4-wide piece
  const int chunk = col >> 3, half = (col >> 2) & 1;
  const unsigned char* a0 = T + tr_swz<RB>(kb + q, chunk) + 8 * half;
  const unsigned char* a1 = T + tr_swz<RB>(kb + 4 + q, chunk) + 8 * half;
  v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)a0);
  v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)a1);
  bf16x8 f;
  v4s_t* fp = reinterpret_cast<v4s_t*>(&f);
  fp[0] = lo;
  fp[1] = hi;
  return f;
}

__device__ __forceinline__ int fdiv(int a, int b, float inv) {
  int q = (int)((float)a * inv);
  int r = a - q * b;
  if (r < 0) --q;
  else if (r >= b) ++q;
  return q;
}

template <int BM, int BN, int NB>
__global__ void __launch_bounds__(kCT, 2)
    conv3x3_wgrad_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                    float* __restrict__ part, int H, int W, int Cin, int Cout, int M, int pps) {
  constexpr int BK = 64;                         // pixels per K-tile
  constexpr int RA = BM * 2, RBb = BN * 2;       // row bytes of the A / B images
  constexpr int A_BYTES = BK * RA, B_BYTES = BK * RBb, BUF = A_BYTES + B_BYTES;
  constexpr int CA = RA / 16, CB = RBb / 16;     // 16-byte chunks per row
  constexpr int AI = A_BYTES / 1024 / 4, BI = B_BYTES / 1024 / 4;  // glds per wave
  constexpr int G = AI + BI;
  constexpr int TM = BM / 2, TN = BN / 2;        // 2x2 waves
  constexpr int FM = TM / 16, FN = TN / 16;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NB * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ci_tiles = Cin / BN, co_tiles = Cout / BM;
  int t = blockIdx.x;
  const int tap = t % 9;
  t /= 9;
  const int cit = t % ci_tiles, cot = t / ci_tiles;
  const int co0 = cot * BM, ci0 = cit * BN;
  const int dr = tap / 3 - 1, ds = tap % 3 - 1;
  const int p_begin = blockIdx.y * pps;
  int p_end = p_begin + pps;
  if (p_end > M) p_end = M;
  const int KT = (p_end - p_begin + BK - 1) / BK;
  const float invW = 1.f / (float)W, invH = 1.f / (float)H;
  const int shift = dr * W + ds;

  // glds lane geometry (per 1 KiB wave-instruction: 1024/RA rows of the A image)
  constexpr int ARPI = 1024 / RA, BRPI = 1024 / RBb;  // rows per instruction
  const int arow_l = lane / CA, apch = lane % CA;
  const int brow_l = lane / CB, bpch = lane % CB;

#define WG_ISSUE(kt_)                                                                        \
  {                                                                                          \
    unsigned char* A_ = lds + ((kt_) % NB) * BUF;                                            \
    unsigned char* B_ = A_ + A_BYTES;                                                        \
    const int pk_ = p_begin + (kt_) * BK;                                                    \
    _Pragma("unroll") for (int q = 0; q < AI; ++q) {                                         \
      const int row = (wid * AI + q) * ARPI + arow_l;                                        \
      const int chunk = (tr_swz<RA>(row, apch) - row * RA) >> 4; /* = apch ^ f(row) */      \
      const int pix = pk_ + row;                                                             \
      const void* src = pix < p_end ? (const void*)(dy + (int64_t)pix * Cout + co0 + chunk * 8) \
                                     : (const void*)g_zero16;                                \
      glds16(src, A_ + (wid * AI + q) * 1024);                                               \
    }                                                                                        \
    _Pragma("unroll") for (int q = 0; q < BI; ++q) {                                         \
      const int row = (wid * BI + q) * BRPI + brow_l;                                        \
      const int chunk = (tr_swz<RBb>(row, bpch) - row * RBb) >> 4;                           \
      const int pix = pk_ + row;                                                             \
      const int tq = fdiv(pix, W, invW);                                                     \
      const int w_ = pix - tq * W;                                                           \
      const int h_ = tq - fdiv(tq, H, invH) * H;                                             \
      const int hh = h_ + dr, ww = w_ + ds;                                                  \
      const bool ok = pix < p_end && hh >= 0 && hh < H && ww >= 0 && ww < W;                 \
      const void* src = ok ? (const void*)(x + (int64_t)(pix + shift) * Cin + ci0 + chunk * 8) \
                           : (const void*)g_zero16;                                          \
      glds16(src, B_ + (wid * BI + q) * 1024);                                               \
    }                                                                                        \
  }

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < KT) WG_ISSUE(p);

  for (int kt = 0; kt < KT; ++kt) {
    if (kt + NB - 2 < KT) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (NB - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + NB - 1 < KT) WG_ISSUE(kt + NB - 1);
    const unsigned char* A = lds + (kt % NB) * BUF;
    const unsigned char* B = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kb = ks * 32 + (lane >> 4) * 8;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = tr_frag<RA>(A, kb, wm * TM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = tr_frag<RBb>(B, kb, wn * TN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
#undef WG_ISSUE

  // partial tile: rows = co (4 per lane group), cols = ci (lane & 15)
  float* out = part + ((int64_t)blockIdx.y * 9 + tap) * Cout * Cin;
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * TM + i * 16 + fg * 4 + e;
        const int ci = ci0 + wn * TN + j * 16 + fr;
        out[(int64_t)co * Cin + ci] = acc[i][j][e];
      }
}

// dW[co][tap][ci] (KRSC) = sum over splits of part[split][tap][co][ci]
template <typename TO>
__global__ void __launch_bounds__(256)
    wgrad_reduce_k(const float* __restrict__ part, int S, int Cout, int Cin, TO* __restrict__ dw) {
  const int64_t total = (int64_t)9 * Cout * Cin;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(e % Cin);
    const int64_t r = e / Cin;
    const int co = (int)(r % Cout);
    const int tap = (int)(r / Cout);
    float sum = 0.f;
    for (int s = 0; s < S; ++s) sum += part[(int64_t)s * total + e];
    dw[((int64_t)co * 9 + tap) * Cin + ci] = from_f32<TO>(sum);
  }
}
}  // namespace

bool conv3x3_nhwc_supported(int Cin, int Cout) { return Cin % 64 == 0 && Cout % 64 == 0; }

int conv3x3_wgrad_splits(int N, int H, int W, int Cin, int Cout) {
  const int M = N * H * W;
  const int bm = (Cout % 128 == 0 && Cin % 128 == 0) ? 128 : 64;
  const int tiles = (Cout / bm) * (Cin / bm) * 9;
  int S = (1536 + tiles - 1) / tiles;
  const int max_s = M / (64 * 4);  // >= 4 K-tiles per split
  if (S > max_s) S = max_s;
  return S < 1 ? 1 : S;
}

void conv3x3_nhwc_wgrad(const void* dy, const void* x, float* part, void* dw, bool dw_fp32,
                        int N, int H, int W, int Cin, int Cout, int S, hipStream_t st) {
  const int M = N * H * W;
  int pps = (M + S - 1) / S;
  pps = (pps + 63) / 64 * 64;
  const auto* dyp = static_cast<const bf16_t*>(dy);
  const auto* xp = static_cast<const bf16_t*>(x);
  if (Cout % 128 == 0 && Cin % 128 == 0) {
    const int tiles = (Cout / 128) * (Cin / 128) * 9;
    hipLaunchKernelGGL((conv3x3_wgrad_k<128, 128, 2>), dim3(tiles, S), dim3(kCT), 0, st, dyp, xp,
                       part, H, W, Cin, Cout, M, pps);
  } else {
    const int tiles = (Cout / 64) * (Cin / 64) * 9;
    hipLaunchKernelGGL((conv3x3_wgrad_k<64, 64, 3>), dim3(tiles, S), dim3(kCT), 0, st, dyp, xp,
                       part, H, W, Cin, Cout, M, pps);
  }
  const int64_t total = (int64_t)9 * Cout * Cin;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  if (dw_fp32)
    hipLaunchKernelGGL((wgrad_reduce_k<float>), dim3(blocks), dim3(256), 0, st, part, S, Cout, Cin,
                       static_cast<float*>(dw));
  else
    hipLaunchKernelGGL((wgrad_reduce_k<bf16_t>), dim3(blocks), dim3(256), 0, st, part, S, Cout,
                       Cin, static_cast<bf16_t*>(dw));
}

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
