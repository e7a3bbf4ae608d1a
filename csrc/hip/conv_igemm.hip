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
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

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

// LDS image of a K-tile of RB-byte rows (RB = 2 * BK): 16-byte chunks XOR-swizzled so the
// 16 rows a ds_read_b128 lane group reads (rows fr = lane & 15, chunk lane >> 4 (+4 k))
// hit distinct bank slots.  128-byte rows: key (row >> 1) & 7.  64-byte rows (four rows per
// 256-byte bank line, so bank slot = 4 (row & 3) + chunk): key ((row >> 2) & 1) << 1 -
// each group's rows {0-3, 12-15} x chunk c and {4-11} x chunk c ^ 1 land on 16 distinct
// slots.
template <int RB>
__device__ __forceinline__ int swz_key(int row) {
  if constexpr (RB == 128) return (row >> 1) & 7;
  else return ((row >> 2) & 1) << 1;
}
template <int RB>
__device__ __forceinline__ int swzr(int row, int chunk) {
  return row * RB + ((chunk ^ swz_key<RB>(row)) << 4);
}

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// The same DMA as inline asm, for the weight-gradient kernels: there the compiler, unable
// to tell which LDS bytes a pending builtin DMA writes, put an s_waitcnt vmcnt(0) in front
// of the first transposed read of the CURRENT K-tile, right after the NEXT K-tile's issue -
// every K-tile waited out its own prefetch (ISA of the round-5 build, one per kernel).
// These loops order the ring themselves (explicit vmcnt wait + barrier before a stage is
// read), so the compiler need not see the writes.  (conv_tap_k keeps the builtin: its
// ISA has no such wait.)
__device__ __forceinline__ void glds16a(const void* g, unsigned char* l) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)l;
  asm volatile("global_load_lds_dwordx4 %0, off" : : "v"(g), "{m0}"(la) : "memory");
#endif
}

// workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not wait for
// outstanding global loads / stores (vmcnt), so prefetches and output stores stay in
// flight; the empty asm statements keep the compiler from moving memory operations
// across it
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// bijective blockIdx -> tile remap keeping consecutive tiles on one XCD
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

// Tap sets of the implicit-GEMM launches (all wave-uniform integer arithmetic, so
// the K loop's per-tile offsets stay in scalar registers):
//   kFwd3 / kFwd1   - 3x3 pad-1 / 1x1 conv forward (stride via ConvGeom::as)
//   kDgrad3 / kDgrad1 - data gradient of a stride-2 conv, blockIdx.z = input-pixel
//                       parity class (ph, pw): class pixel (2a+ph, 2b+pw) receives
//                       dY at (a + dh, b + dw) through the taps of matching parity
//                       only (3x3: 1, 2, 2 or 4 taps; 1x1: one tap for the even-even
//                       class, none - a zero store - for the others)
enum ConvMode { kFwd3 = 0, kFwd1 = 1, kDgrad3 = 2, kDgrad1 = 3 };

template <int MODE>
__device__ __forceinline__ int conv_ntaps(int z) {
  if constexpr (MODE == kFwd3) return 9;
  else if constexpr (MODE == kFwd1) return 1;
  else if constexpr (MODE == kDgrad3) return ((z >> 1) ? 2 : 1) * ((z & 1) ? 2 : 1);
  else return z == 0 ? 1 : 0;
}

// tap t of class z: A-pixel offset (dh, dw) from the row's centre pixel and the
// filter tap index wt into the B rows
template <int MODE>
__device__ __forceinline__ void conv_tap(int z, int t, int& dh, int& dw, int& wt) {
  if constexpr (MODE == kFwd3) {
    const int r = t / 3, s = t - r * 3;
    dh = r - 1; dw = s - 1; wt = t;
  } else if constexpr (MODE == kDgrad3) {
    const int ph = z >> 1, pw = z & 1, ns = pw ? 2 : 1;
    const int ri = t / ns, si = t - ri * ns;
    const int r = ph ? 2 * ri : 1, s = pw ? 2 * si : 1;
    dh = (ph + 1 - r) >> 1; dw = (pw + 1 - s) >> 1;
    wt = 8 - (3 * r + s);  // B = rotated filter: wrot[ci][8-t][co] = W[co][t][ci]
  } else {
    dh = 0; dw = 0; wt = 0;
  }
}

// GEMM row m -> (img, gh, gw) on a GH x GW grid; A centre pixel (gh*as, gw*as) of an
// AH x AW image with KC channels; output pixel (gh*ys + yoh, gw*ys + yow) of a
// YH x YW image with NC channels (dgrad: ys = 2, (yoh, yow) = the parity class);
// B rows ([NC][taps][KC]) are kb_stride elements long
struct ConvGeom {
  int GH, GW, AH, AW, as, YH, YW, ys, KC, NC, M, kb_stride;
};

// BN-backward epilogue (conv_tap_k EPI == 1, ConvBnEpi).  Each thread owns one 8-channel
// column group of the BM x BN output tile and visits ROWS of its rows.  bnbwd_prefetch
// issues every global load the epilogue needs (residual gradient, BN input x, ReLU
// bitmask byte, the channel constants) BEFORE the accumulators go to LDS, so their
// latency hides under the tile write and barrier - the pass is otherwise a chain of
// dependent loads with few waves per CU.  bnbwd_store then forms, per row chunk,
// o = T (+ add), g = relu_mask ? o : 0 rounded to bf16, stores g in place of o and
// accumulates the BN's backward sums of exactly those values: sum(g), sum(g*(x-mean)).
template <int BM, int BN, int CT = kCT>
struct BnPre {
  static constexpr int CPR = BN / 8;
  static constexpr int RGS = CT / CPR;  // row groups; a thread visits rows rg, rg + RGS, ...
  static constexpr int ROWS = BM / RGS;
  uint4 av[ROWS], xv[ROWS];
  unsigned mk[ROWS];
  float mu[8], iv[8], wv[8], bv[8];  // raw per-channel constants (combined after the wait)
};

template <int MODE>
__device__ __forceinline__ int64_t out_pix(const ConvGeom& g, int m, int z) {
  if constexpr (MODE == kFwd3 || MODE == kFwd1) {
    return m;
  } else {
    const int GHW = g.GH * g.GW;
    const int n = m / GHW;
    const int rem = m - n * GHW;
    const int gh = rem / g.GW, gw = rem - gh * g.GW;
    return (int64_t)(n * g.YH + gh * g.ys + (z >> 1)) * g.YW + gw * g.ys + (z & 1);
  }
}

// constant sources for the branch-free epilogue loads below (absent tensors)
__device__ const float g_one8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
__device__ const uint8_t g_ff16[16] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                       0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};

// Branch-free: every load is issued unconditionally through a selected pointer (a
// constant array when the tensor is absent), the per-channel constants first.  With the
// former conditional loads (`addp ? load : 0`, `ep.w ? ep.w[c] : 1`) the compiler put an
// s_waitcnt vmcnt(0) at each control-flow join (a register written by a load on one path
// and by a move on the other) and before the constants' arithmetic - which also drained
// every row load issued before it: the prefetch ran as ~10 serial memory round trips per
// workgroup (ISA of the round-5 build).
template <int MODE, int BM, int BN, int CT>
__device__ __forceinline__ void bnbwd_prefetch(const ConvGeom& g, const ConvBnEpi& ep, int m0,
                                               int n0, int z, BnPre<BM, BN, CT>& P) {
  using PT = BnPre<BM, BN, CT>;
  const int tid = threadIdx.x;
  const int cc = tid % PT::CPR, rg = tid / PT::CPR;
  const int c0 = n0 + cc * 8;
  const int NC = g.NC;
  const bool rm2 = ep.relu_mode == 2, rm1 = ep.relu_mode == 1;
  const float* zf = reinterpret_cast<const float*>(g_zero16);
  {
    const float* wp = rm2 && ep.w ? ep.w + c0 : g_one8;
    const float* bp = rm2 && ep.b ? ep.b + c0 : zf;
    const float* ip = rm2 ? ep.invstd + c0 : zf;
    const float* mp = ep.mean + c0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      P.mu[i] = mp[i];
      P.iv[i] = ip[i];
      P.wv[i] = wp[i];
      P.bv[i] = bp[i];
    }
  }
  const bf16_t* addp = static_cast<const bf16_t*>(ep.add);
  const bf16_t* xp = static_cast<const bf16_t*>(ep.xbn);
  const bf16_t* zb = reinterpret_cast<const bf16_t*>(g_zero16);
  const bool x_on = true, s2 = ep.add_s2 && addp;
#pragma unroll
  for (int q = 0; q < PT::ROWS; ++q) {
    const int m = m0 + q * PT::RGS + rg;
    const int mm = m < g.M ? m : 0;
    const int64_t opix = out_pix<MODE>(g, mm, z);
    const int64_t off = opix * NC + c0;
    int64_t aoff = off;
    bool a_on = addp != nullptr;
    if (s2) {
      // compact stride-2 residual gradient: pixel (n, h, w) receives add[n][h/2][w/2] when
      // h and w are even (dense output pixels: opix = m on a GH x GW grid)
      const int GHW = g.GH * g.GW;
      const int n = mm / GHW, rem = mm - n * GHW;
      const int h = rem / g.GW, w = rem - h * g.GW;
      aoff = ((int64_t)(n * (g.GH >> 1) + (h >> 1)) * (g.GW >> 1) + (w >> 1)) * NC + c0;
      a_on = ((h | w) & 1) == 0;
    }
    P.av[q] = *reinterpret_cast<const uint4*>(a_on ? addp + aoff : zb);
    P.xv[q] = *reinterpret_cast<const uint4*>(x_on ? xp + off : zb);
    P.mk[q] = *(rm1 ? ep.rmask + opix * (NC >> 3) + (c0 >> 3) : g_ff16);
  }
}

// one specialisation per (ReLU-mask mode, residual add): the per-element mode tests are
// compile-time, so the unrolled store loop is straight-line code (runtime tests there
// made the compiler branch around every element: +30-60 us per ResNet-50 layer)
template <int MODE, int BM, int BN, int CT, int RM, bool ADD, int TS>
__device__ __forceinline__ void bnbwd_store_t(const bf16_t* T, bf16_t* __restrict__ y,
                                              const ConvGeom& g, int m0, int n0, int z,
                                              const BnPre<BM, BN, CT>& P, float (&s1)[8],
                                              float (&s2)[8]) {
  using PT = BnPre<BM, BN, CT>;
  const int tid = threadIdx.x;
  const int cc = tid % PT::CPR, rg = tid / PT::CPR;
  const int c0 = n0 + cc * 8;
  // every prefetched load has landed (they flew under the accumulator -> LDS tile
  // write): one vmcnt(0) the compiler sees (the builtin, not asm), so the row loop below
  // issues its stores without a wait per row - the compiler cannot count loads past the
  // guarded stores and waited vmcnt(0), i.e. for the previous row's store, in front of
  // every row
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt untouched
  // the BN affine of the ReLU recompute, from the raw constants (arithmetic on them before
  // this point made the compiler wait for every prefetched row in the prefetch itself)
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = P.iv[i] * P.wv[i];
    sh[i] = P.bv[i] - P.mu[i] * sc[i];
  }
#pragma unroll
  for (int q = 0; q < PT::ROWS; ++q) {
    const int row = q * PT::RGS + rg;
    const int m = m0 + row;
    if (m >= g.M) continue;
    const uint4 tv = *reinterpret_cast<const uint4*>(T + row * TS + cc * 8);
    const unsigned tw[4] = {tv.x, tv.y, tv.z, tv.w};
    const unsigned aw[4] = {P.av[q].x, P.av[q].y, P.av[q].z, P.av[q].w};
    const unsigned xw[4] = {P.xv[q].x, P.xv[q].y, P.xv[q].z, P.xv[q].w};
    unsigned ow[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float o[2], xx[2];
      o[0] = __uint_as_float(tw[k] << 16);
      o[1] = __uint_as_float(tw[k] & 0xffff0000u);
      if constexpr (ADD) {  // the residual gradient (rounded once more, as a separate add would)
        o[0] += __uint_as_float(aw[k] << 16);
        o[1] += __uint_as_float(aw[k] & 0xffff0000u);
      }
      xx[0] = __uint_as_float(xw[k] << 16);
      xx[1] = __uint_as_float(xw[k] & 0xffff0000u);
      unsigned short hb[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = 2 * k + h;
        bool keep = true;
        if constexpr (RM == 1) keep = (P.mk[q] >> i) & 1u;
        else if constexpr (RM == 2) keep = fmaf(xx[h], sc[i], sh[i]) > 0.f;
        const bf16_t gb = (bf16_t)(keep ? o[h] : 0.f);
        const float gv = (float)gb;
        s1[i] += gv;
        s2[i] = fmaf(gv, xx[h] - P.mu[i], s2[i]);
        hb[h] = __builtin_bit_cast(unsigned short, gb);
      }
      ow[k] = (unsigned)hb[0] | ((unsigned)hb[1] << 16);
    }
    *reinterpret_cast<uint4*>(y + out_pix<MODE>(g, m, z) * g.NC + c0) =
        make_uint4(ow[0], ow[1], ow[2], ow[3]);
  }
}

template <int MODE, int BM, int BN, int CT, int TS>
__device__ __forceinline__ void bnbwd_store(const bf16_t* T, bf16_t* __restrict__ y,
                                            const ConvGeom& g, const ConvBnEpi& ep, int m0,
                                            int n0, int z, const BnPre<BM, BN, CT>& P,
                                            float (&s1)[8], float (&s2)[8]) {
  const bool add = ep.add != nullptr;
  switch (ep.relu_mode * 2 + (add ? 1 : 0)) {
    case 0: bnbwd_store_t<MODE, BM, BN, CT, 0, false, TS>(T, y, g, m0, n0, z, P, s1, s2); break;
    case 1: bnbwd_store_t<MODE, BM, BN, CT, 0, true, TS>(T, y, g, m0, n0, z, P, s1, s2); break;
    case 2: bnbwd_store_t<MODE, BM, BN, CT, 1, false, TS>(T, y, g, m0, n0, z, P, s1, s2); break;
    case 3: bnbwd_store_t<MODE, BM, BN, CT, 1, true, TS>(T, y, g, m0, n0, z, P, s1, s2); break;
    case 4: bnbwd_store_t<MODE, BM, BN, CT, 2, false, TS>(T, y, g, m0, n0, z, P, s1, s2); break;
    default: bnbwd_store_t<MODE, BM, BN, CT, 2, true, TS>(T, y, g, m0, n0, z, P, s1, s2); break;
  }
}

// NB = 1 (no DMA ring): for 1x1 convs with one or two K-tiles (K = 64 / 128: the
// ResNet layer1-2 channel-expanding convs) - nothing to overlap inside a workgroup, so
// the LDS goes to more resident workgroups instead (3 per CU: one's loads overlap
// another's MFMAs and stores; 4 would cap the registers at 128 and spill the epilogue
// statistics).
// BK = 32: 64-byte K-tile rows - half the LDS per ring stage, so a 3-deep ring keeps two
// stages (32 KB at 128 x 128) in flight with up to 3 workgroups per CU.
template <int MODE, int BM, int BN, int WM, int WN, int NB, int EPI = 0, int CT = kCT,
          int BK = kBK, bool EARLY = false>
__global__ void __launch_bounds__(CT, (NB * (BM + BN) * BK * 2 > 80 * 1024)
                                          ? 1 : (NB == 1 && EPI == 0 ? 3 : 2))
    conv_tap_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wt,
               bf16_t* __restrict__ y, ConvGeom g, float* __restrict__ slab,
               const float* __restrict__ shift, ConvBnEpi ep) {
  constexpr int NW = CT / 64;
  static_assert(WM * WN == NW, "one wave per output sub-tile");
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int RB = BK * 2;        // bytes per K-tile row
  constexpr int LPR = RB / 16;      // DMA lanes per row
  constexpr int RPI = 64 / LPR;     // rows per DMA wave-instruction
  constexpr int KS = BK / 32;       // MFMA k-steps per K-tile
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB;
  constexpr int BUF = A_BYTES + B_BYTES;
  constexpr int AI = BM / (RPI * NW);  // A wave-instructions (RPI rows each) per wave per tile
  constexpr int BI = BN / (RPI * NW);  // B wave-instructions per wave per tile
  static_assert(AI >= 1 && BI >= 1, "tile rows per wave");
  constexpr int G = AI + BI;        // glds per wave per tile (vmcnt units)
  // the ring, or the epilogue's bf16 tile / statistics exchange if larger
  // epilogue tile rows padded by 16 bytes: the 16 lanes of a ds_write_b64 group (16 rows,
  // one 4-column slice) then hit 16 distinct bank pairs
  constexpr int TS = BN + 8;
  constexpr int EPI_BYTES = BM * TS * 2 > 2 * CT * 8 * 4 ? BM * TS * 2 : 2 * CT * 8 * 4;
  constexpr int LDS_BYTES = NB * BUF > EPI_BYTES ? NB * BUF : EPI_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // tile order: with gridDim.y == 1 the N tiles are folded into x, N fastest (a launch
  // with N tiles > 1 on y walks every M tile per N tile): consecutive tiles on one XCD
  // then share the A rows (one L2 fill per M tile instead of one per N tile)
  const int NTf = gridDim.y == 1 ? g.NC / BN : 1;
  const int lt = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lt / NTf, MTn = (int)gridDim.x / NTf;
  const int m0 = mt * BM, n0 = (gridDim.y == 1 ? lt - mt * NTf : (int)blockIdx.y) * BN;
  // parity classes of a stride-2 3x3 dgrad in longest-first order: blockIdx.z is
  // dispatched slowest, so the 4-tap class (z = 3) goes out first and the 1-tap class
  // fills the tail (ResNet-50 shapes 118 -> 107, 103 -> 90, 93 -> 82 us,
  // tools/dgrad_s2_bench.py; the 1x1 form's only real class, z = 0, is already first)
  const int z = MODE == kDgrad3 ? (int)gridDim.z - 1 - (int)blockIdx.z : (int)blockIdx.z;
  const int ntaps = conv_ntaps<MODE>(z);
  const int KC = g.KC, M = g.M, GHW = g.GH * g.GW;

  // DMA lane geometry: wave `wid` fills A rows [wid*32, wid*32+32) as AI
  // instructions of 8 rows; lane -> (row = base + lane/8, physical chunk lane%8)
  // fetching the logical chunk that the swizzle stores at that position.
  const int lrow = lane / LPR, pchunk = lane % LPR;
  // per DMA row: source pointer at the centre pixel / channel chunk, and a bit
  // mask of the taps whose pixel is inside the A image (so the K loop only adds a
  // wave-uniform offset and tests one bit per row)
  const bf16_t* abase[AI];
  unsigned amask[AI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    const int row = wid * (BM / NW) + q * RPI + lrow;
    const int ch = pchunk ^ swz_key<RB>(row);
    const int m = m0 + row;
    const int mm = m < M ? m : 0;
    const int n = mm / GHW;
    const int rem = mm - n * GHW;
    const int gh = rem / g.GW, gw = rem - gh * g.GW;
    const int h = gh * g.as, w = gw * g.as;
    abase[q] = x + ((int64_t)(n * g.AH + h) * g.AW + w) * KC + ch * 8;
    unsigned mk = 0;
    constexpr int TMAX = MODE == kFwd3 ? 9 : (MODE == kDgrad3 ? 4 : 1);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      int dh, dw, wti;
      conv_tap<MODE>(z, t, dh, dw, wti);
      const int hh = h + dh, ww = w + dw;
      if (t < ntaps && m < M && hh >= 0 && hh < g.AH && ww >= 0 && ww < g.AW) mk |= 1u << t;
    }
    amask[q] = mk;
  }
  const bf16_t* bbase[BI];
#pragma unroll
  for (int q = 0; q < BI; ++q) {
    const int row = wid * (BN / NW) + q * RPI + lrow;
    bbase[q] = wt + (int64_t)(n0 + row) * g.kb_stride + (pchunk ^ swz_key<RB>(row)) * 8;
  }
  const int kc_per_tap = KC / BK;
  const int KT = ntaps * kc_per_tap;

#define CONV_ISSUE(kt_)                                                                     \
  {                                                                                         \
    /* 1x1 modes have one tap: no per-K-tile scalar division */                             \
    const int tap_ = (MODE == kFwd1 || MODE == kDgrad1) ? 0 : (kt_) / kc_per_tap;           \
    const int c0_ = ((kt_) - tap_ * kc_per_tap) * BK;                                       \
    int dh_, dw_, wt_;                                                                      \
    conv_tap<MODE>(z, tap_, dh_, dw_, wt_);                                                 \
    const int64_t aoff_ = (int64_t)(dh_ * g.AW + dw_) * KC + c0_;                           \
    const int boff_ = wt_ * KC + c0_;                                                       \
    unsigned char* A_ = lds + ((kt_) % NB) * BUF;                                           \
    unsigned char* B_ = A_ + A_BYTES;                                                       \
    _Pragma("unroll") for (int q = 0; q < AI; ++q) {                                        \
      const bool ok = (amask[q] >> tap_) & 1u;                                              \
      glds16(ok ? (const void*)(abase[q] + aoff_) : (const void*)g_zero16,                  \
             A_ + (wid * (BM / NW) + q * RPI) * RB);                                       \
    }                                                                                       \
    _Pragma("unroll") for (int q = 0; q < BI; ++q)                                          \
      glds16(bbase[q] + boff_, B_ + (wid * (BN / NW) + q * RPI) * RB);                      \
  }

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // epilogue BN statistics (see the store loop): this thread's 8 channels' shift,
  // loaded now so the latency hides under the K loop
  constexpr int CPR = BN / 8;  // 16-byte chunks per output row
  // EPI == 1 (BN-backward epilogue, ConvBnEpi): slab gets sum(g), sum(g * (x - mean))
  const bool want_stats = EPI == 1 ? slab != nullptr
                                   : (MODE == kFwd3 || MODE == kFwd1) && slab != nullptr;
  const int scc = tid % CPR;
  float shv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    shv[i] = (EPI == 0 && want_stats && shift) ? shift[n0 + scc * 8 + i] : 0.f;

  // BN-backward epilogue operands (EPI == 1): issued after the K loop - issued earlier
  // they would sit at the head of the in-order vmcnt queue and every counted wait of the
  // loop would stall on them (measured: no gain from a prefetch at kernel start) - and
  // consumed after barriers that wait for LDS only, so they fly under the accumulator ->
  // LDS tile write instead of being waited for at a __syncthreads()
  BnPre<BM, BN, CT> pre;
  if constexpr (EPI == 1 && EARLY) bnbwd_prefetch<MODE, BM, BN, CT>(g, ep, m0, n0, z, pre);

  {
    // prologue: NB-1 tiles in flight
  #pragma unroll
    for (int p = 0; p < NB - 1; ++p)
      if (p < KT) CONV_ISSUE(p);

    for (int kt = 0; kt < KT; ++kt) {
      if constexpr (NB == 1) {
        if (kt > 0) __syncthreads();  // every wave is done reading the single buffer
        CONV_ISSUE(kt);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      } else {
        // retire tile kt: leave the (NB-2) younger tiles' DMAs in flight
        if (kt + NB - 2 < KT) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (NB > 2 ? NB - 2 : 0)) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + NB - 1 < KT) CONV_ISSUE(kt + NB - 1);
      }
      const unsigned char* A = lds + (kt % NB) * BUF;
      const unsigned char* B = A + A_BYTES;
  #pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = ks * 4 + fg;
        bf16x8 af[FM], bfr[FN];
  #pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(A + swzr<RB>(wm * TM + i * 16 + fr, ch));
  #pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(B + swzr<RB>(wn * TN + j * 16 + fr, ch));
  #pragma unroll
        for (int i = 0; i < FM; ++i)
  #pragma unroll
          for (int j = 0; j < FN; ++j)  // (B, A): accumulator = C^T, 4 columns per lane
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  }
#undef CONV_ISSUE
  // (the K loop ended on a vmcnt(0) wait: no tile DMA is in flight; an LDS-only barrier
  // leaves the epilogue prefetch of EPI == 1 outstanding)
  if constexpr (EPI == 1) {
    if constexpr (!EARLY) bnbwd_prefetch<MODE, BM, BN, CT>(g, ep, m0, n0, z, pre);
    lds_barrier();
  } else {
    __syncthreads();
  }

  // epilogue: accumulators -> bf16 tile in LDS -> coalesced 16-byte row stores.  The
  // accumulators hold C^T (B was the first MFMA operand): lane (fr, fg) of block (i, j)
  // has the 4 consecutive columns j*16 + fg*4 .. +3 of row i*16 + fr - one 8-byte LDS
  // store instead of four 2-byte ones
  bf16_t* T = reinterpret_cast<bf16_t*>(lds);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wm * TM + i * 16 + fr;
      const int col = wn * TN + j * 16 + fg * 4;
      const unsigned lo = (unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][0]) |
                          ((unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][1]) << 16);
      const unsigned hi = (unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][2]) |
                          ((unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][3]) << 16);
      *reinterpret_cast<uint2*>(T + row * TS + col) = make_uint2(lo, hi);
    }
  if constexpr (EPI == 1) {
    lds_barrier();
  } else {
    __syncthreads();
  }
  constexpr bool dense = MODE == kFwd3 || MODE == kFwd1;
  // BatchNorm statistics of this output tile for the BN that consumes y (its stats
  // pass over y disappears): a thread's 16-byte chunks all lie in ONE 8-channel
  // column group (kCT % CPR == 0), so the bf16-ROUNDED values it stores (exactly what
  // y holds) also feed its per-channel shifted sums sum(v - s), sum((v - s)^2) with
  // s = that BN's running mean; the row groups are combined through LDS and written
  // channel-major, slab[0|1][c][m-tile]: the finalize kernel then reads each channel's
  // S tile sums as one contiguous row (one coalesced pass, no fold kernel; fixed order).
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s2[i] = 0.f;
  if constexpr (EPI == 1) {
    bnbwd_store<MODE, BM, BN, CT, TS>(T, y, g, ep, m0, n0, z, pre, s1, s2);
  } else
  for (int c = tid; c < BM * CPR; c += CT) {
    const int row = c / CPR, cc = c - row * CPR;
    const int m = m0 + row;
    if (m >= M) continue;
    int64_t opix = m;
    if (!dense) {
      const int n = m / GHW;
      const int rem = m - n * GHW;
      const int gh = rem / g.GW, gw = rem - gh * g.GW;
      opix = (int64_t)(n * g.YH + gh * g.ys + (z >> 1)) * g.YW + gw * g.ys + (z & 1);
    }
    const uint4 v = *reinterpret_cast<const uint4*>(T + row * TS + cc * 8);
    *reinterpret_cast<uint4*>(y + opix * g.NC + n0 + cc * 8) = v;
    if (want_stats) {
      const unsigned wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = __uint_as_float(wv[q] << 16) - shv[2 * q];
        const float hi = __uint_as_float(wv[q] & 0xffff0000u) - shv[2 * q + 1];
        s1[2 * q] += lo;
        s2[2 * q] = fmaf(lo, lo, s2[2 * q]);
        s1[2 * q + 1] += hi;
        s2[2 * q + 1] = fmaf(hi, hi, s2[2 * q + 1]);
      }
    }
  }
  if (want_stats) {
    constexpr int RGS = CT / CPR;  // row groups (threads sharing a column group)
    // every thread is done reading the bf16 tile (an LDS-only barrier: the output
    // stores just issued need not complete before the statistics exchange)
    lds_barrier();
    float* red = reinterpret_cast<float*>(lds);
    const int rg = tid / CPR;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[rg * BN + scc * 8 + i] = s1[i];
      red[RGS * BN + rg * BN + scc * 8 + i] = s2[i];
    }
    lds_barrier();
    if (tid < BN) {
      float a = 0.f, b = 0.f;
#pragma unroll 4
      for (int q = 0; q < RGS; ++q) {
        a += red[q * BN + tid];
        b += red[RGS * BN + q * BN + tid];
      }
      // channel-major [2][C][S] (S = M tiles x parity classes, blockIdx.z after the M
      // tiles): consecutive M tiles run on one XCD, so its L2 merges the 4-byte stores of
      // neighbouring workgroups into whole lines
      const int64_t S = (int64_t)MTn * gridDim.z, s = (int64_t)z * MTn + mt;
      slab[(int64_t)(n0 + tid) * S + s] = a;
      slab[(int64_t)(g.NC + n0 + tid) * S + s] = b;
    }
  }
}

// Tile choice per launch (measured per shape, docs/PERF.md rounds 3-5; the losing A/B
// variants - 256-row tiles with 4 or 8 waves, the 4-deep pipelined 32-deep ring, the
// burst-free interleaved 64-deep loop, 64-row tiles for the large 1x1 forwards - were
// removed in round 6):
//  * 1x1 data gradients with the BN-backward epilogue over >= 50,176 output pixels and
//    K < 256 (ResNet-50 layers 1-3; 2.8-3.5 TB/s of epilogue traffic): 64-row M tiles, up
//    to 4 workgroups per CU (11,373 -> 11,430 img/s, profiles/r5/ab_r50_bm64/); from
//    K = 256 the 128-row tiles win (8 MFMAs per wave per barrier were too few: round 6,
//    1024->256 @ 14 68 -> 53 us, 512->128 @ 28 91 -> 82, 256->1024 @ 14 113 -> 107,
//    profiles/r6/bnbwd1x1_k256.md);
//  * 1x1 forwards with one 64-channel K-tile (the layer-1/2 channel-expanding convs): no
//    DMA ring (NB = 1), 3 workgroups per CU;
//  * 128-wide output tiles: 32-deep K-tiles on a 3-deep ring where the grid has >= 1024
//    workgroups (48 KB in flight, up to 3 workgroups per CU; 3x3 128@28 94.8 -> 86.3 us),
//    64-deep K-tiles on a 2-deep ring on the smaller grids (twice the barriers per K
//    cost more there: 3x3 256@14 82 -> 96 us);
//  * 64-wide output tiles: 32-deep K-tiles on a 3-deep ring (layer-1 3x3 64@56 fwd
//    111 -> 106 us, dgrad 103 -> 99 us).
int g_bnbwd_early = 1;  // BN-backward epilogue prefetch at kernel start for small K (A/B switch)
// (the 64-row tile rule below depends on K too: conv_bnbwd_mtiles mirrors it)

// N-fastest tile order (N tiles folded into grid x, see conv_tap_k): 0 off, 1 by shape
// (default), 2 every conv_tap_k launch (A/B switch).  Per call, same box
// (profiles/r6/nfast/bench*.md, tools/diag/nfast_bench.py): 512 -> 2048 @ 7 51.2 -> 47.6 us,
// 2048 -> 512 @ 7 43.0 -> 37.4, 256 -> 1024 @ 14 58.0 -> 54.9, the BN-backward 1x1 dgrads
// 65.2 -> 58.6 / 52.8 -> 45.5 / 82.3 -> 77.2, 64 -> 256 @ 56 172.6 -> 161.7 - but the
// 4-N-tile launches over >= 1024 M tiles (the @ 28 expansions, 128 -> 512 and the stride-2
// 256 -> 512 projection) lose (78.0 -> 89.4, 113.4 -> 125.8): those keep M fastest.
// ResNet-50 (folding every 1x1 launch): 12,367 / 12,228 vs 12,174 / 12,060 img/s.
int g_conv_nfast = 1;

inline dim3 conv_grid(int mtiles, int ntiles, int nclasses, bool one_by_one) {
  (void)one_by_one;
  const bool fold = ntiles > 1 && (g_conv_nfast == 2 ||
                                   (g_conv_nfast == 1 && !(ntiles == 4 && mtiles >= 1024)));
  return fold ? dim3((unsigned)(mtiles * ntiles), 1, nclasses)
              : dim3((unsigned)mtiles, (unsigned)ntiles, nclasses);
}

template <int MODE, int EPI = 0>
void launch_conv_tap(const bf16_t* a, const bf16_t* w, bf16_t* y, const ConvGeom& g,
                     hipStream_t st, float* slab = nullptr, const float* shift = nullptr,
                     const ConvBnEpi& ep = ConvBnEpi{}) {
  if (g.M == 0) return;
  const int nclasses = MODE == kDgrad3 || MODE == kDgrad1 ? 4 : 1;
  constexpr bool k1 = MODE == kFwd1 || MODE == kDgrad1;
  if (EPI == 1 && MODE == kFwd1 && g.NC % 128 == 0 && g.M >= 50176 && g.KC < 256) {
    const dim3 grid = conv_grid((g.M + 63) / 64, g.NC / 128, nclasses, k1);
    // K <= 128 (two to four 32-deep K-tiles): the epilogue's loads go out at kernel start
    // and fly under the K loop's DMA (64 -> 256 @ 56 +skip: 324 -> 307 us, 128 -> 512
    // @ 28: 176 -> 171; at K = 256 the held registers cost a wave per SIMD: 110 -> 115)
    if (g_bnbwd_early && g.KC <= 128)
      hipLaunchKernelGGL((conv_tap_k<MODE, 64, 128, 2, 2, 3, EPI, kCT, 32, true>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
    else
      hipLaunchKernelGGL((conv_tap_k<MODE, 64, 128, 2, 2, 3, EPI, kCT, 32>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
  } else if (MODE == kFwd1 && g.NC % 128 == 0 && g.KC / kBK <= 1) {
    const dim3 grid = conv_grid((g.M + kBM - 1) / kBM, g.NC / 128, nclasses, k1);
    hipLaunchKernelGGL((conv_tap_k<MODE, 128, 128, 2, 2, 1, EPI>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
  } else if (g.NC % 128 == 0) {
    const dim3 grid = conv_grid((g.M + kBM - 1) / kBM, g.NC / 128, nclasses, k1);
    if (grid.x * grid.y * grid.z >= 1024)
      hipLaunchKernelGGL((conv_tap_k<MODE, 128, 128, 2, 2, 3, EPI, kCT, 32>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
    else
      hipLaunchKernelGGL((conv_tap_k<MODE, 128, 128, 2, 2, 2, EPI>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
  } else {
    const dim3 grid = conv_grid((g.M + kBM - 1) / kBM, g.NC / 64, nclasses, k1);
    hipLaunchKernelGGL((conv_tap_k<MODE, 128, 64, 4, 1, 3, EPI, kCT, 32>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
  }
}

// ============================================================================
// 3x3 / stride-1 / pad-1 forward with the input HALO resident in LDS (conv3h_k).
//
// conv_tap_k loads a fresh 128-pixel A tile for every (tap, channel slice): 9 loads of
// nearly the same pixels per slice, one 1 KiB LDS-DMA piece per 8 rows - and a DMA piece
// costs ~60 issue cycles among the MFMAs (MI355X_MICROARCH.md), so at 128 x 128 tiles the
// piece stream alone is about as long as the MFMA stream (PMC: 23-28 % MFMA busy, 41 % of
// wave cycles waiting to issue, profiles/r6/conv_pmc).  Here a workgroup's 256 output
// pixels are consecutive in raster order, and in the zero-PADDED raster (row width
// Wp = W + 2, two zero rows between images) the input a tap (r, s) needs for output pixel
// p is at padded position P(p) + (r - 1) Wp + (s - 1): every tap reads one contiguous
// window of R = P(last) - P(first) + 2 Wp + 3 padded rows.  That window (<= 448 rows x
// 32 channels) is DMA'd ONCE per 32-channel slice and the nine taps read their A
// fragments from it at a wave-uniform row shift; only the weights stream per tap.  Pieces
// per MFMA drop ~3x (128@28: 9 x 32 pieces per slice per 128 x 128 tile -> 28 + 9 x 8 per
// 256 x 128 tile).
//
// LDS images are row-major, 64 bytes (32 channels) per row, with the (row >> 2) & 1 chunk
// swizzle of conv_tap_k's 64-byte rows - conflict-free for 16 consecutive rows at ANY
// alignment, which the tap shifts need (the row jumps at image-row ends still cost some
// 2-way conflicts: 5.7 LDS cycles per fragment read at W = 28 vs 4 ideal, 8 at W <= 14).
// A DMA wave-instruction fills 16 rows x 4 chunks, so it touches 16 cache lines (a
// planar layout - lane l -> row l of one chunk plane - touched 64, and ran no faster
// than conv_tap_k: the address/tag work, not the piece count, bounded it).  Halo rows
// that are padding or past the window carry an out-of-range buffer offset, which the
// buffer load returns as zeros.
//
// Pipeline (per 32-channel slice c, taps t = 0..8 = K-steps k = 9 c + t): the weights of
// step k go to ring slot k % 3 two steps ahead; the next slice's halo goes to the other
// halo buffer in piece pairs during taps 0-3.  One counted vmcnt wait + one barrier per
// step.  80 KiB of LDS: two workgroups per CU, so one's barrier / DMA issue hides under
// the other's MFMAs.  Tile 256 x BN (4 waves of 128 x 64 for BN = 128, 64 x 64 for 64).
constexpr int kHBM = 256;                  // output pixels per workgroup (224: a variant)
// halo rows per buffer: 448 (7 DMA row blocks, 28 KiB) next to the 128-wide weight ring,
// 512 (32 KiB) next to the 64-wide one - either way 80 KiB in all
constexpr int halo_rows(int BN) { return BN == 128 ? 448 : 512; }
constexpr uint32_t kHZero = 0x80000000u;   // out-of-range offset: the DMA writes zeros

__device__ __forceinline__ int halo_ppos(int p, int H, int W, int HW) {
  const int n = p / HW, r = p - n * HW;
  const int h = r / W, w = r - h * W;
  return (n * (H + 2) + h + 1) * (W + 2) + w + 1;
}

// buffer load of 16 bytes per lane straight into LDS (lane l -> l * 16 from dst).  A
// __device__ wrapper: with the builtin called in the kernel body on per-lane offsets the
// HIP host pass dropped the kernel's launch stub without a diagnostic (link error)
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, unsigned char* dst,
                                          uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16,
                                           voff, soff, 0, 0);
}

// halo pieces of the NEXT slice issued at tap t of a slice (two per tap over taps 0-3)
constexpr int conv3h_hcount(int t, int nhp) {
  return t < 0 || t >= 4 ? 0 : (nhp - 2 * t < 2 ? nhp - 2 * t : 2);
}

template <int N>
__device__ __forceinline__ void vm_wait_c() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BN, int EPI, int BM_ = kHBM>
__global__ void __launch_bounds__(kCT, 2)
    conv3h_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wt,
             bf16_t* __restrict__ y, ConvGeom g, float* __restrict__ slab,
             const float* __restrict__ shift, ConvBnEpi ep) {
  constexpr int BM = BM_, CT = kCT, WM = BN == 128 ? 2 : 4, WN = 4 / WM;
  static_assert(BM % (16 * WM) == 0, "16-row fragments per wave");
  constexpr int kHRows = halo_rows(BN), kHBuf = kHRows * 64;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int BSLOT = BN * 64;           // BN weight rows x 32 channels
  constexpr int BPW = BN / 64;             // weight pieces (16 rows each) per wave per step
  constexpr int NHP = kHRows / 64;         // halo pieces per wave per slice (7 | 8)
  constexpr int RING = 2 * kHBuf + 3 * BSLOT;
  constexpr int TS = BN + 8;               // padded epilogue tile rows (as conv_tap_k)
  constexpr int EPI_BYTES = BM * TS * 2;
  constexpr int LDS_BYTES = RING > EPI_BYTES ? RING : EPI_BYTES;
  static_assert(LDS_BYTES <= 80 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];
  unsigned char* const hbuf = lds;
  unsigned char* const bring = lds + 2 * kHBuf;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  // N tiles folded into grid x when gridDim.y == 1 (N fastest, as conv_tap_k)
  const int NTf = gridDim.y == 1 ? g.NC / BN : 1;
  const int lt = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lt / NTf, MTn = (int)gridDim.x / NTf;
  const int m0 = mt * BM, n0 = (gridDim.y == 1 ? lt - mt * NTf : (int)blockIdx.y) * BN;
  const int H = g.GH, W = g.GW, HW = H * W, Wp = W + 2, HpWp = (H + 2) * Wp;
  const int M = g.M, KC = g.KC;
  const int p1 = min(m0 + BM, M) - 1;
  const int base = halo_ppos(m0, H, W, HW) - Wp - 1;   // padded position of halo row 0
  const int pend = halo_ppos(p1, H, W, HW) + Wp + 1;   // of the last halo row (host-checked)
  const int lrow = lane >> 2, pch = lane & 3;          // DMA: row in the piece, stored chunk

  // halo DMA: wave w fills row blocks w, w + 4, ... (16 rows each); the descriptor starts
  // at the window's first image so the 32-bit offsets stay small
  const int64_t pix0 = (int64_t)(base / HpWp) * HW;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(x + pix0 * KC), 0, 0x7fffffff, 0x00020000);
  uint32_t hoff[NHP];
#pragma unroll
  for (int u = 0; u < NHP; ++u) {
    const int row = (wid + 4 * u) * 16 + lrow;
    const int q = base + row;
    const int n = q / HpWp, rr = q - n * HpWp;
    const int hp = rr / Wp, wp = rr - hp * Wp;
    const bool ok = q <= pend && hp >= 1 && hp <= H && wp >= 1 && wp <= W;
    const int64_t pix = (int64_t)(n * H + hp - 1) * W + wp - 1 - pix0;
    hoff[u] = ok ? (uint32_t)(pix * KC * 2) + (uint32_t)((pch ^ swz_key<64>(row)) * 16) : kHZero;
  }
  // weight DMA: wave w fills weight row blocks w * BPW .. + BPW - 1
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(wt + (int64_t)n0 * g.kb_stride), 0, 0x7fffffff, 0x00020000);
  uint32_t woff[BPW];
#pragma unroll
  for (int u = 0; u < BPW; ++u) {
    const int row = (wid * BPW + u) * 16 + lrow;
    woff[u] = (uint32_t)(row * g.kb_stride * 2) + (uint32_t)((pch ^ swz_key<64>(row)) * 16);
  }

  const int nch = KC / 32;
  // halo pieces 2t, 2t + 1 of slice c, with constant register indices (a runtime index
  // put hoff in scratch)
#define HALO_PIECE(c_, u_) \
  buf_lds16(rx, hbuf + ((c_) & 1) * kHBuf + (wid + 4 * (u_)) * 1024, hoff[u_], (c_) * 64)
#define HALO_PIECES(c_, t_)                                                                 \
  switch (t_) {                                                                             \
    case 0: HALO_PIECE(c_, 0); HALO_PIECE(c_, 1); break;                                    \
    case 1: HALO_PIECE(c_, 2); HALO_PIECE(c_, 3); break;                                    \
    case 2: HALO_PIECE(c_, 4); HALO_PIECE(c_, 5); break;                                    \
    default: HALO_PIECE(c_, 6); if (NHP > 7) HALO_PIECE(c_, NHP - 1); break;                \
  }
#define W_PIECES(k_)                                                                        \
  {                                                                                         \
    const int c_ = (k_) / 9, t_ = (k_) - c_ * 9;                                            \
    _Pragma("unroll") for (int u = 0; u < BPW; ++u)                                         \
      buf_lds16(rw, bring + ((k_) % 3) * BSLOT + (wid * BPW + u) * 1024, woff[u],           \
                (t_ * KC + c_ * 32) * 2);                                                   \
  }
  // halo pieces of the NEXT slice issued in step k (taps 0-3 of a slice, two per tap)
  // fragment reads: A row of output pixel m0 + wm*TM + 16 i + fr (past M: the last pixel)
  // shifted by the tap; B row wn*TN + 16 j + fr; logical chunk fg
  const int fr = lane & 15, fg = lane >> 4;
  int arow[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int p = min(m0 + wm * TM + i * 16 + fr, p1);
    arow[i] = halo_ppos(p, H, W, HW) - base;
  }
  const int boff = swzr<64>(wn * TN + fr, fg);

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: slice 0's halo, the weights of steps 0 and 1
#pragma unroll
  for (int t = 0; t < 4; ++t) HALO_PIECES(0, t);
  W_PIECES(0);
  W_PIECES(1);
  // The nine taps of a slice are unrolled (tap index T a compile-time constant): ring slot
  // (9c + T) % 3 = T % 3, the DMA schedule and every vmcnt count are constants, so a step
  // carries no scalar bookkeeping or branches beyond `more` (the first build computed
  // k / 9, k % 3 and the counts per step: 154 SALU + 27 branch instructions per 32 MFMAs).
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;  // a next slice: its halo goes out during taps 0-3
    const unsigned char* A = hbuf + (c & 1) * kHBuf;
    auto step = [&](auto tc) {
      constexpr int T = decltype(tc)::value;
      // retire this step's weights (and at T = 0 the slice's halo, issued before them):
      // younger pieces are the halo pieces of steps T-2 and T-1 and the weights of T+1
      constexpr int HP = conv3h_hcount(T - 2, NHP) + conv3h_hcount(T - 1, NHP);
      if (more) vm_wait_c<HP + BPW>();
      else if (T < 8) vm_wait_c<BPW>();
      else vm_wait_c<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (more || T < 7) {
        constexpr int T2 = (T + 2) % 9, C2 = (T + 2) / 9;
#pragma unroll
        for (int u = 0; u < BPW; ++u)
          buf_lds16(rw, bring + ((T + 2) % 3) * BSLOT + (wid * BPW + u) * 1024, woff[u],
                    (T2 * KC + (c + C2) * 32) * 2);
      }
      if constexpr (T < 4) {
        if (more) HALO_PIECES(c + 1, T);
      }
      int toff = (T / 3 - 1) * Wp + (T % 3) - 1;
      // opaque per step: else the compiler hoists all 9 x FM tap addresses out of the slice
      // loop (72 live VGPRs, spills)
      asm volatile("" : "+s"(toff));
      const unsigned char* B = bring + (T % 3) * BSLOT + boff;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(B + j * 1024);
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + swzr<64>(arow[i] + toff, fg));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)  // (B, A): accumulator = C^T (see the epilogue)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
    step(std::integral_constant<int, 6>{});
    step(std::integral_constant<int, 7>{});
    step(std::integral_constant<int, 8>{});
  }
#undef HALO_PIECE
#undef HALO_PIECES
#undef W_PIECES
  // the last step waited vmcnt(0): no DMA in flight
  __syncthreads();
  // the statistics shift, loaded only now (held across the loop it cost the registers
  // the fragment double buffer needs)
  constexpr int CPR = BN / 8;
  const bool want_stats = slab != nullptr;
  const int scc = tid % CPR;
  float shv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) shv[i] = (EPI == 0 && want_stats && shift) ? shift[n0 + scc * 8 + i] : 0.f;

  // epilogue (as conv_tap_k): C^T accumulators -> bf16 tile in LDS (8-byte stores of 4
  // consecutive columns, padded rows) -> coalesced row stores
  bf16_t* T = reinterpret_cast<bf16_t*>(lds);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wm * TM + i * 16 + fr;
      const int col = wn * TN + j * 16 + fg * 4;
      const unsigned lo = (unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][0]) |
                          ((unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][1]) << 16);
      const unsigned hi = (unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][2]) |
                          ((unsigned)__builtin_bit_cast(unsigned short, (bf16_t)acc[i][j][3]) << 16);
      *reinterpret_cast<uint2*>(T + row * TS + col) = make_uint2(lo, hi);
    }
  __syncthreads();
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s2[i] = 0.f;
  if constexpr (EPI == 1) {
    // the BN-backward operands are fetched after the accumulators are dead (a 256-row
    // prefetch held across the tile write would exceed the 2-workgroups-per-CU registers)
    BnPre<BM, BN, CT> pre;
    bnbwd_prefetch<kFwd3, BM, BN, CT>(g, ep, m0, n0, 0, pre);
    bnbwd_store<kFwd3, BM, BN, CT, TS>(T, y, g, ep, m0, n0, 0, pre, s1, s2);
  } else {
    for (int q = tid; q < BM * CPR; q += CT) {
      const int row = q / CPR, cc = q - row * CPR;
      const int m = m0 + row;
      if (m >= M) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(T + row * TS + cc * 8);
      *reinterpret_cast<uint4*>(y + (int64_t)m * g.NC + n0 + cc * 8) = v;
      if (want_stats) {
        const unsigned wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float lo = __uint_as_float(wv[u] << 16) - shv[2 * u];
          const float hi = __uint_as_float(wv[u] & 0xffff0000u) - shv[2 * u + 1];
          s1[2 * u] += lo;
          s2[2 * u] = fmaf(lo, lo, s2[2 * u]);
          s1[2 * u + 1] += hi;
          s2[2 * u + 1] = fmaf(hi, hi, s2[2 * u + 1]);
        }
      }
    }
  }
  if (want_stats) {
    constexpr int RGS = CT / CPR;
    lds_barrier();
    float* red = reinterpret_cast<float*>(lds);
    const int rg = tid / CPR;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[rg * BN + scc * 8 + i] = s1[i];
      red[RGS * BN + rg * BN + scc * 8 + i] = s2[i];
    }
    lds_barrier();
    if (tid < BN) {
      float a = 0.f, b = 0.f;
#pragma unroll 4
      for (int q = 0; q < RGS; ++q) {
        a += red[q * BN + tid];
        b += red[RGS * BN + q * BN + tid];
      }
      const int64_t S = MTn;
      slab[(int64_t)(n0 + tid) * S + mt] = a;
      slab[(int64_t)(g.NC + n0 + tid) * S + mt] = b;
    }
  }
}

// Largest halo window (rows) of any BM-pixel tile of an N x H x W raster, cached per
// shape (the launch path asks once per conv call).
int halo_rows_max(int N, int H, int W, int BM) {
  struct Ent { int n, h, w, bm, r; };
  static Ent cache[32];
  static int filled = 0;
  for (int i = 0; i < filled; ++i)
    if (cache[i].n == N && cache[i].h == H && cache[i].w == W && cache[i].bm == BM)
      return cache[i].r;
  const int64_t M = (int64_t)N * H * W;
  const int HW = H * W, Wp = W + 2;
  auto pp = [&](int64_t p) {
    const int64_t n = p / HW, r = p - n * HW, h = r / W, w = r - h * W;
    return (n * (H + 2) + h + 1) * Wp + w + 1;
  };
  int64_t r = 0;
  for (int64_t m0 = 0; m0 < M; m0 += BM) {
    const int64_t p1 = std::min<int64_t>(m0 + BM, M) - 1;
    r = std::max<int64_t>(r, pp(p1) - pp(m0) + 2 * Wp + 3);
  }
  const int res = (int)std::min<int64_t>(r, 1 << 30);
  if (filled < 32) cache[filled++] = Ent{N, H, W, BM, res};
  return res;
}

// 0: off, 1: automatic tile width, 64 / 128: that width wherever it is possible (A/B)
int g_conv_halo = 1;
// pixel tile: 0 automatic, 224 / 256 forced (A/B)
int g_conv_halo_bm = 0;

// Tile of the halo kernel for a 3x3 conv, {0, 0} = not eligible.  Width 128 where Cout
// allows and the window fits 448 rows, else 64 (512-row window).  Measured (profiles/r6/
// conv_halo.md, batch 256, vs conv_tap_k): 128@28 fwd / +stats / +BN-bwd 93 / 97 / 110 ->
// 85 / 78 / 87 us, 256@14 79 / 82 / 81 -> 63 / 64 / 69, 512@7 (64 wide) 75 / 77 / 72 ->
// 66 / 67 / 69, 64@56 (64 wide) 102 / 110 / 147 -> 79 / 93 / 120.  Pixel tile 256 or 224:
// the one with the smaller (rounds of 512 workgroup slots - two per CU) x tile work, so a
// grid that would leave a mostly empty last round, or fill one round only partly, takes
// the 12.5 % shorter tiles (128 wide only).  (Cin % 64 == 0 is conv3x3_nhwc_supported's.)
struct Conv3hCfg {
  int bn, bm;
};
Conv3hCfg conv3h_cfg(int N, int H, int W, int Cout, int stride) {
  if (g_conv_halo == 0 || stride != 1 || N <= 0 || Cout % 64 != 0) return {0, 0};
  const int64_t M = (int64_t)N * H * W;
  Conv3hCfg best{0, 0};
  double best_cost = 1e300;
  for (int bm : {256, 224}) {
    if (g_conv_halo_bm != 0 && bm != g_conv_halo_bm) continue;
    const int r = halo_rows_max(N, H, W, bm);
    for (int bn : {128, 64}) {
      if (bn == 128 && (Cout % 128 != 0 || g_conv_halo == 64)) continue;
      if (bn == 64 && bm != 256) continue;  // 4 x 1 waves: 56-row wave tiles don't exist
      if (r > halo_rows(bn)) continue;
      const int64_t tiles = (M + bm - 1) / bm * (Cout / bn);
      const int64_t rounds = (tiles + 511) / 512;
      // 64-wide tiles do 64 x 64 per wave (vs 128 x 64): ~5 % less efficient per FLOP
      const double cost = (double)rounds * bm * bn * (bn == 64 ? 1.05 : 1.0);
      if (cost < best_cost * 0.999) {
        best_cost = cost;
        best = {bn, bm};
      }
    }
  }
  return best;
}
int conv3h_bn(int N, int H, int W, int Cout, int stride) {
  return conv3h_cfg(N, H, W, Cout, stride).bn;
}
bool conv3h_ok(int N, int H, int W, int Cout, int stride) {
  return conv3h_bn(N, H, W, Cout, stride) != 0;
}
int conv3h_mtile(int N, int H, int W, int Cout) { return conv3h_cfg(N, H, W, Cout, 1).bm; }

// halo kernel tile order: N tiles folded into grid x, N fastest (1) or on grid y (0).
// Neutral per call (its M tiles' windows are small next to the weights re-read per tap)
// and ResNet-50 12,136 / 12,140 vs 12,220 / 12,214 img/s same box (profiles/r6/nfast/halo/):
// off by default (A/B switch)
int g_conv3h_nfast = 0;

template <int EPI>
void launch_conv3h(const bf16_t* a, const bf16_t* w, bf16_t* y, const ConvGeom& g, int N,
                   hipStream_t st, float* slab, const float* shift, const ConvBnEpi& ep) {
  const Conv3hCfg c = conv3h_cfg(N, g.GH, g.GW, g.NC, 1);
  const int mtiles = (g.M + c.bm - 1) / c.bm, ntiles = g.NC / c.bn;
  const dim3 grid = g_conv3h_nfast && ntiles > 1 ? dim3((unsigned)(mtiles * ntiles), 1, 1)
                                                 : dim3((unsigned)mtiles, (unsigned)ntiles, 1);
  if (c.bn == 128 && c.bm == 256)
    hipLaunchKernelGGL((conv3h_k<128, EPI, 256>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
  else if (c.bn == 128)
    hipLaunchKernelGGL((conv3h_k<128, EPI, 224>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
  else
    hipLaunchKernelGGL((conv3h_k<64, EPI, 256>), grid, dim3(kCT), 0, st, a, w, y, g, slab, shift, ep);
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

__device__ __forceinline__ bf16x8 tr_pair(const unsigned char* T, unsigned lo, unsigned hi) {
  v4s_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(T + lo));
  v4s_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(T + hi));
  bf16x8 f;
  v4s_t* fp = reinterpret_cast<v4s_t*>(&f);
  fp[0] = a;
  fp[1] = b;
  return f;
}

// byte offsets of the two transposed reads (k rows kb..kb+3 / kb+4..kb+7) of column
// block c0 for this lane; column block c0+16 is the same with bit 5 flipped
// (its chunk index differs by 2 with no carry)
template <int RB>
__device__ __forceinline__ void tr_offsets(int kb, int c0, int lane, unsigned& lo, unsigned& hi) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  const int chunk = col >> 3, half = (col >> 2) & 1;
  lo = (unsigned)(tr_swz<RB>(kb + q, chunk) + 8 * half);
  hi = (unsigned)(tr_swz<RB>(kb + 4 + q, chunk) + 8 * half);
}

__device__ __forceinline__ int fdiv(int a, int b, float inv) {
  int q = (int)((float)a * inv);
  int r = a - q * b;
  if (r < 0) --q;
  else if (r >= b) ++q;
  return q;
}

// All 9 taps per workgroup.  The GEMM K index runs over output pixels laid out
// in the zero-PADDED row width Wp = W + 2 (q = h*Wp + w', the 2 extra columns
// per row are dummy K rows whose dY is zero), because then the input a tap
// (r, s) needs is x_padded[q + r*Wp + s]: for a K-tile of BK consecutive q all
// 9 taps read ONE contiguous strip of the padded input (BK + 2*Wp + 2 rows),
// loaded once, instead of 9 separate shifted tiles.  Padding = zero-page lanes.
constexpr int kWgBK = 64, kWgMaxW = 56;
constexpr int kWgStrip = kWgBK + 2 * (kWgMaxW + 2) + 2;   // 182 rows max
constexpr int kWgStripI = (kWgStrip + 31) / 32;            // glds per wave (8 rows each)

template <int NB>
__global__ void __launch_bounds__(kCT, 1)
    conv3x3_wgrad9_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                     float* __restrict__ part, int H, int W, int Cin, int Cout, int kpi,
                     int kps, int total_kt) {
  constexpr int BM = 64, BN = 64, BK = kWgBK, RB = 128;
  constexpr int A_BYTES = BK * RB;                       // 8 KiB
  constexpr int S_BYTES = kWgStripI * 4 * 1024;          // strip rows, 1 KiB per instruction
  constexpr int BUF = A_BYTES + S_BYTES;
  constexpr int AI = A_BYTES / 1024 / 4;                 // 2 glds per wave
  constexpr int G = AI + kWgStripI;
  constexpr int FM = 2, FN = 2;                          // 2x2 waves of 32x32 per tap
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NB * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ci_tiles = Cin / BN;
  const int cit = blockIdx.x % ci_tiles, cot = blockIdx.x / ci_tiles;
  const int co0 = cot * BM, ci0 = cit * BN;
  const int kt_begin = blockIdx.y * kps;
  int kt_end = kt_begin + kps;
  if (kt_end > total_kt) kt_end = total_kt;
  const int KT = kt_end - kt_begin;
  const int Wp = W + 2, HWp = H * Wp;
  const float invWp = 1.f / (float)Wp;
  const int lrow = lane >> 3, pch = lane & 7;

#define WG9_ISSUE(i_)                                                                          \
  {                                                                                            \
    const int gkt = kt_begin + (i_);                                                           \
    const int n_ = gkt / kpi;                                                                  \
    const int q0 = (gkt - n_ * kpi) * BK;                                                      \
    unsigned char* A_ = lds + ((i_) % NB) * BUF;                                               \
    unsigned char* S_ = A_ + A_BYTES;                                                          \
    _Pragma("unroll") for (int q = 0; q < AI; ++q) {                                           \
      const int row = (wid * AI + q) * 8 + lrow;                                               \
      const int chunk = (tr_swz<RB>(row, pch) - row * RB) >> 4;                                \
      const int qq = q0 + row;                                                                 \
      const int h_ = fdiv(qq, Wp, invWp), w_ = qq - h_ * Wp;                                   \
      const bool ok = qq < HWp && w_ < W;                                                      \
      const void* src = ok ? (const void*)(dy + (((int64_t)n_ * H + h_) * W + w_) * Cout + co0 + chunk * 8) \
                           : (const void*)g_zero16;                                            \
      glds16(src, A_ + (wid * AI + q) * 1024);                                                 \
    }                                                                                          \
    _Pragma("unroll") for (int q = 0; q < kWgStripI; ++q) {                                    \
      const int row = (q * 4 + wid) * 8 + lrow;                                                \
      const int chunk = (tr_swz<RB>(row, pch) - row * RB) >> 4;                                \
      const int P = q0 + row;                                                                  \
      const int hp = fdiv(P, Wp, invWp), wp = P - hp * Wp;                                     \
      const bool ok = hp >= 1 && hp <= H && wp >= 1 && wp <= W;                                \
      const void* src = ok ? (const void*)(x + (((int64_t)n_ * H + hp - 1) * W + wp - 1) * Cin + ci0 + chunk * 8) \
                           : (const void*)g_zero16;                                            \
      glds16(src, S_ + (q * 4 + wid) * 1024);                                                  \
    }                                                                                          \
  }

  f32x4_t acc[9][FM][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // loop-invariant transposed-read offsets: A (2 ks) and the strip (2 ks x 9 taps)
  unsigned alo[2], ahi[2], slo[2][9], shi[2][9];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int kb = ks * 32 + (lane >> 4) * 8;
    tr_offsets<RB>(kb, wm * 32, lane, alo[ks], ahi[ks]);
#pragma unroll
    for (int t = 0; t < 9; ++t)
      tr_offsets<RB>(kb + (t / 3) * Wp + (t % 3), wn * 32, lane, slo[ks][t], shi[ks][t]);
  }

#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < KT) WG9_ISSUE(p);

  for (int kt = 0; kt < KT; ++kt) {
    if (kt + NB - 2 < KT) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (NB - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + NB - 1 < KT) WG9_ISSUE(kt + NB - 1);
    const unsigned char* A = lds + (kt % NB) * BUF;
    const unsigned char* S = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM];
      af[0] = tr_pair(A, alo[ks], ahi[ks]);
      af[1] = tr_pair(A, alo[ks] ^ 32u, ahi[ks] ^ 32u);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        bf16x8 bfr[FN];
        bfr[0] = tr_pair(S, slo[ks][t], shi[ks][t]);
        bfr[1] = tr_pair(S, slo[ks][t] ^ 32u, shi[ks][t] ^ 32u);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[t][i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[t][i][j], 0, 0, 0);
      }
    }
  }
#undef WG9_ISSUE

  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    float* out = part + ((int64_t)blockIdx.y * 9 + t) * Cout * Cin;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + wm * 32 + i * 16 + fg * 4 + e;
          const int ci = ci0 + wn * 32 + j * 16 + fr;
          out[(int64_t)co * Cin + ci] = acc[t][i][j][e];
        }
  }
}

// ----------------------------------------------------------------------------
// 3x3 stride-1 weight gradient for 64 -> 64 channels (ResNet layer 1), all 9 taps per
// workgroup on a strip RING.  The per-tap kernel below reads each dY / X pixel row once
// per tap for a 64 x 64 output tile - for 64 channels that is 9x the operand traffic per
// MFMA and the kernel ends up L2 / LDS bound (357 TF standalone, 128 TF beside the
// side-stream work).  Here one workgroup owns the whole [64 co] x [9 taps x 64 ci] output
// and a contiguous range of K-tiles (64 padded-row pixels, q = h*(W+2) + w: the two pad
// columns are dummy K rows whose dY is zero, so tap (r, s) of pixel q reads the padded
// input at q + r*(W+2) + s - one contiguous strip of 64 + 2*(W+2) + 2 rows serves all 9
// taps).  Consecutive K-tiles' strips overlap by all but 64 rows, so the strip lives in
// a 256-row LDS ring: each K-tile DMAs only its 64 dY rows and the 64 strip rows past the
// current frontier (16 KB instead of 31), the first K-tile of an image the whole strip.
// The ring's 16-byte chunks carry tr_swz<128>'s row swizzle, which depends on row bits 1
// and 3 only, so a read offset moves with the ring base by a plain add + wrap mask.
// 8 waves: (k half of the K-tile) x (a quarter of the 576 output columns, 9 MFMA column
// blocks = 64 x 144 per wave); the two k halves are summed through LDS at the end and
// the workgroup writes one fp32 partial [tap][co][ci] slab for wgrad_reduce*_k.
constexpr int kW64Ring = 256;                     // strip ring rows (x 128 B = 32 KB)
constexpr int kW64BK = 64;                        // pixels per K-tile

__global__ void __launch_bounds__(512, 1)
    conv3x3_wgrad_c64_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                        float* __restrict__ part, int H, int W, int kpi, int kps, int total_kt,
                        int Cin, int Cout) {
  constexpr int RB = 128;                                   // 64 channels x bf16
  constexpr int A_BYTES = kW64BK * RB;                      // 8 KB per dY K-tile
  constexpr int RING_BYTES = kW64Ring * RB;                 // 32 KB
  constexpr int NFB = 9;                                    // column blocks per wave
  constexpr int EX_BYTES = 4 * 64 * NFB * 16 * 4;           // k-half exchange, 147,456 B
  constexpr int LOOP_BYTES = RING_BYTES + 2 * A_BYTES;
  constexpr int LDSB = EX_BYTES > LOOP_BYTES ? EX_BYTES : LOOP_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDSB];
  unsigned char* ring = lds;
  unsigned char* abuf = lds + RING_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid >> 2, wn = wid & 3;
  const int Wp = W + 2, HWp = H * Wp;
  const int SR = (kW64BK + 2 * Wp + 2 + 7) & ~7;            // strip rows (8-row aligned)
  // 64 x 64 channel tile blockIdx.y of a Cout x Cin layer (round 6: the kernel was
  // 64 -> 64 only)
  const int ci_tiles = Cin >> 6;
  const int co0 = ((int)blockIdx.y / ci_tiles) * 64, ci0 = ((int)blockIdx.y % ci_tiles) * 64;
  const float invWp = 1.f / (float)Wp;
  const int kt_begin = blockIdx.x * kps;
  const int kt_end = kt_begin + kps < total_kt ? kt_begin + kps : total_kt;
  const int lrow = lane >> 3, pch = lane & 7;

  // one 8-row DMA group of strip rows [P, P + 8) of image n into the ring (P % 8 == 0)
  auto strip_group = [&](int n, int P) {
    const int row = P + lrow;
    const int pos = row & (kW64Ring - 1);
    const int chunk = (tr_swz<RB>(pos, pch) - pos * RB) >> 4;
    const int hp = fdiv(row, Wp, invWp), wp = row - hp * Wp;
    const bool ok = hp >= 1 && hp <= H && wp >= 1 && wp <= W;
    const void* src = ok ? (const void*)(x + (((int64_t)n * H + hp - 1) * W + wp - 1) * Cin + ci0 + chunk * 8)
                         : (const void*)g_zero16;
    glds16a(src, ring + (P & (kW64Ring - 1)) * RB);
  };
  // the 8 dY row groups of K-tile (n, q0)
  auto a_tile = [&](int n, int q0, int buf) {  // 8 row groups: one per wave
    const int row = wid * 8 + lrow;
    const int chunk = (tr_swz<RB>(row, pch) - row * RB) >> 4;
    const int qq = q0 + row;
    const int h_ = fdiv(qq, Wp, invWp), w_ = qq - h_ * Wp;
    const bool ok = qq < HWp && w_ < W;
    const void* src = ok ? (const void*)(dy + (((int64_t)n * H + h_) * W + w_) * Cout + co0 + chunk * 8)
                         : (const void*)g_zero16;
    glds16a(src, abuf + buf * A_BYTES + wid * 1024);
  };

  // loop-invariant transposed-read offsets.  A (dY image, 64 co): k rows wk*32 + ...
  unsigned alo[2], ahi[2];
  {
    const int kb = wk * 32 + (lane >> 4) * 8;
    tr_offsets<RB>(kb, 0, lane, alo[0], ahi[0]);
    tr_offsets<RB>(kb, 32, lane, alo[1], ahi[1]);
  }
  // B (strip ring): column block cb = wn * 9 + j -> tap = cb / 4, ci block cb % 4; the
  // offsets at ring base 0 - a K-tile adds base * 128 and wraps at 32 KB
  unsigned blo[NFB], bhi[NFB];
#pragma unroll
  for (int j = 0; j < NFB; ++j) {
    const int cb = wn * NFB + j, tap = cb >> 2, cib = cb & 3;
    const int kb = wk * 32 + (lane >> 4) * 8 + (tap / 3) * Wp + (tap % 3);
    tr_offsets<RB>(kb, cib * 16, lane, blo[j], bhi[j]);
  }

  f32x4_t acc[4][NFB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NFB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  int t = kt_begin;
  while (t < kt_end) {
    const int n = t / kpi;
    const int seg_end = (n + 1) * kpi < kt_end ? (n + 1) * kpi : kt_end;
    int q0 = (t - n * kpi) * kW64BK;
    // segment prologue: the whole strip [q0, q0 + SR) and the first dY tile
    for (int grp = wid; grp * 8 < SR; grp += 8) strip_group(n, q0 + grp * 8);
    a_tile(n, q0, t & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (; t < seg_end; ++t, q0 += kW64BK) {
      if (t + 1 < seg_end) {
        // next K-tile: its dY rows + the 64 strip rows past the frontier q0 + SR
        a_tile(n, q0 + kW64BK, (t + 1) & 1);
        strip_group(n, q0 + SR + wid * 8);
      }
      const unsigned char* A = abuf + (t & 1) * A_BYTES;
      const unsigned base = (unsigned)(q0 & (kW64Ring - 1)) * RB;
      bf16x8 af[4];
      af[0] = tr_pair(A, alo[0], ahi[0]);
      af[1] = tr_pair(A, alo[0] ^ 32u, ahi[0] ^ 32u);
      af[2] = tr_pair(A, alo[1], ahi[1]);
      af[3] = tr_pair(A, alo[1] ^ 32u, ahi[1] ^ 32u);
#pragma unroll
      for (int j = 0; j < NFB; ++j) {
        const bf16x8 bf = tr_pair(ring, (blo[j] + base) & (RING_BYTES - 1),
                                  (bhi[j] + base) & (RING_BYTES - 1));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[i][j], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

  // k halves: waves wk = 1 hand their accumulators to wk = 0 through LDS
  float* E = reinterpret_cast<float*>(lds);
  const int fr = lane & 15, fg = lane >> 4;
  __syncthreads();
  if (wk == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NFB; ++j)
        *reinterpret_cast<f32x4_t*>(E + (((wn * 4 + i) * NFB + j) * 64 + lane) * 4) = acc[i][j];
  }
  __syncthreads();
  if (wk == 0) {
    float* out = part + (int64_t)blockIdx.x * 9 * Cout * Cin;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NFB; ++j) {
        const f32x4_t o = *reinterpret_cast<const f32x4_t*>(E + (((wn * 4 + i) * NFB + j) * 64 + lane) * 4);
        const int cb = wn * NFB + j, tap = cb >> 2, ci = (cb & 3) * 16 + fr;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = i * 16 + fg * 4 + e;
          out[((int64_t)tap * Cout + co0 + co) * Cin + ci0 + ci] = acc[i][j][e] + o[e];
        }
      }
  }
}

// ----------------------------------------------------------------------------
// Per-tap weight gradient (the default path): one workgroup = one filter tap
// (r, s) x a BM(co) x BN(ci) output tile x one pixel range (split-K), so the
// wave tiles are 64 x 64 (16 MFMA 16x16x32 accumulators per wave, two
// workgroups per CU) instead of the 9-tap kernel's 32 x 32 x 9:
//   dW[co, tap, ci] += sum_{p in range} dY[p, co] * X[p + (r-1)*W + (s-1), ci]
// with the shifted pixel zeroed outside the image.  Both LDS images are pixel
// rows ([k][channel], 16-byte chunks XOR-swizzled on the DMA source side) read
// as MFMA fragments with ds_read_b64_tr_b16.  128 x 128 tiles use 2 x 2 waves on
// BK = 64 pixels; 64-channel layers use 64 x 64 tiles with the 4 waves splitting
// BK = 128 pixels (an in-workgroup split-K summed in the epilogue), so the LDS
// bytes per MFMA stay the same.  Workgroups of one pixel range (all taps and
// tiles: the same dY rows and nearly the same X rows) are packed onto one XCD.
// Output: fp32 partials [split][tap][co][ci] for wgrad_reduce{1,2}_k.
template <int BM, int BN, int WM, int WN, int WK, int BK, int NB, bool S1>
__global__ void __launch_bounds__(kCT, 2)
    conv3x3_wgrad_tap_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                        float* __restrict__ part, int H, int W, int Ho, int Wo, int stride,
                        int T, int Cin, int Cout, int M, int kps, int total_kt, int gx) {
  static_assert(WM * WN * WK == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN;
  static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tiles of 32-column blocks");
  constexpr int FM = TM / 16, FN = TN / 16, HM = TM / 32, HN = TN / 32;
  constexpr int RBA = BM * 2, RBB = BN * 2;        // LDS row bytes (128 | 256)
  constexpr int A_BYTES = BK * RBA, B_BYTES = BK * RBB, BUF = A_BYTES + B_BYTES;
  constexpr int AI = A_BYTES / 4096, BI = B_BYTES / 4096;  // 1 KiB glds per wave per tile
  constexpr int G = AI + BI;
  constexpr int LPRA = RBA / 16, LPRB = RBB / 16;  // lanes per LDS row
  constexpr int KW = BK / WK, KS = KW / 32;        // k rows per wave, 32-k MFMA steps
  static_assert(AI >= 1 && BI >= 1 && KS >= 1, "tile too small");
  constexpr int ES = BN + 4;                       // epilogue fp32 row stride
  constexpr int EPI = WK * BM * ES * 4;
  constexpr int LDSB = NB * BUF > EPI ? NB * BUF : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDSB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid % WK, wn = (wid / WK) % WN, wm = wid / (WK * WN);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / gx, tt = lid - split * gx;
  const int tap = tt % T, tile = tt / T;
  const int ci_tiles = Cin / BN;
  const int co0 = (tile / ci_tiles) * BM, ci0 = (tile % ci_tiles) * BN;
  const int kt_begin = split * kps;
  const int kt_end = kt_begin + kps < total_kt ? kt_begin + kps : total_kt;
  const int KT = kt_end - kt_begin;
  const int dr = T == 9 ? tap / 3 - 1 : 0, dc = T == 9 ? tap % 3 - 1 : 0;
  const float invWo = 1.f / (float)Wo, invHo = 1.f / (float)Ho;

  // per DMA row: logical chunk fetched by this lane (source-side swizzle)
  int achunk[AI], bchunk[BI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    const int row = (wid * AI + q) * (1024 / RBA) + lane / LPRA;
    achunk[q] = (tr_swz<RBA>(row, lane % LPRA) - row * RBA) >> 4;
  }
#pragma unroll
  for (int q = 0; q < BI; ++q) {
    const int row = (wid * BI + q) * (1024 / RBB) + lane / LPRB;
    bchunk[q] = (tr_swz<RBB>(row, lane % LPRB) - row * RBB) >> 4;
  }

#define WGT_ISSUE(i_)                                                                          \
  {                                                                                            \
    const int p0_ = (kt_begin + (i_)) * BK;                                                    \
    unsigned char* A_ = lds + ((i_) % NB) * BUF;                                               \
    unsigned char* B_ = A_ + A_BYTES;                                                          \
    _Pragma("unroll") for (int q = 0; q < AI; ++q) {                                           \
      const int p_ = p0_ + (wid * AI + q) * (1024 / RBA) + lane / LPRA;                        \
      const void* src_ = p_ < M ? (const void*)(dy + (int64_t)p_ * Cout + co0 + achunk[q] * 8) \
                                : (const void*)g_zero16;                                       \
      glds16a(src_, A_ + (wid * AI + q) * 1024);                                               \
    }                                                                                          \
    _Pragma("unroll") for (int q = 0; q < BI; ++q) {                                           \
      const int p_ = p0_ + (wid * BI + q) * (1024 / RBB) + lane / LPRB;                        \
      const int hq_ = fdiv(p_, Wo, invWo);                                                     \
      const int n_ = fdiv(hq_, Ho, invHo);                                                     \
      const int hi_ = (hq_ - n_ * Ho) * (S1 ? 1 : stride) + dr;                                \
      const int wi_ = (p_ - hq_ * Wo) * (S1 ? 1 : stride) + dc;                                \
      const bool ok_ = p_ < M && (unsigned)hi_ < (unsigned)H && (unsigned)wi_ < (unsigned)W;   \
      /* stride 1: the input pixel is the output pixel shifted by (dr, dc) */                  \
      const int64_t xpix_ = S1 ? (int64_t)p_ + dr * W + dc                                     \
                               : (int64_t)(n_ * H + hi_) * W + wi_;                            \
      const void* src_ = ok_ ? (const void*)(x + xpix_ * Cin + ci0 + bchunk[q] * 8)            \
                             : (const void*)g_zero16;                                          \
      glds16a(src_, B_ + (wid * BI + q) * 1024);                                               \
    }                                                                                          \
  }

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // loop-invariant transposed-read offsets: per k-step, column blocks c0 and c0+32
  // (c0+16 / c0+48 are the same offsets with bit 5 flipped)
  unsigned alo[KS][HM], ahi[KS][HM], blo[KS][HN], bhi[KS][HN];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int kb = wk * KW + ks * 32 + (lane >> 4) * 8;
#pragma unroll
    for (int h2 = 0; h2 < HM; ++h2)
      tr_offsets<RBA>(kb, wm * TM + 32 * h2, lane, alo[ks][h2], ahi[ks][h2]);
#pragma unroll
    for (int h2 = 0; h2 < HN; ++h2)
      tr_offsets<RBB>(kb, wn * TN + 32 * h2, lane, blo[ks][h2], bhi[ks][h2]);
  }

#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < KT) WGT_ISSUE(p);

  for (int kt = 0; kt < KT; ++kt) {
    if (kt + NB - 2 < KT) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (NB - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + NB - 1 < KT) WGT_ISSUE(kt + NB - 1);
    const unsigned char* A = lds + (kt % NB) * BUF;
    const unsigned char* B = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int h2 = 0; h2 < HM; ++h2) {
        af[2 * h2] = tr_pair(A, alo[ks][h2], ahi[ks][h2]);
        af[2 * h2 + 1] = tr_pair(A, alo[ks][h2] ^ 32u, ahi[ks][h2] ^ 32u);
      }
#pragma unroll
      for (int h2 = 0; h2 < HN; ++h2) {
        bfr[2 * h2] = tr_pair(B, blo[ks][h2], bhi[ks][h2]);
        bfr[2 * h2 + 1] = tr_pair(B, blo[ks][h2] ^ 32u, bhi[ks][h2] ^ 32u);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
#undef WGT_ISSUE
  __syncthreads();

  // epilogue: accumulators -> fp32 LDS image [wk][BM][BN] -> (sum over wk) -> float4 rows
  float* E = reinterpret_cast<float*>(lds);
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        E[(wk * BM + wm * TM + i * 16 + fg * 4 + e) * ES + wn * TN + j * 16 + fr] = acc[i][j][e];
  __syncthreads();
  float* out = part + ((int64_t)split * T + tap) * Cout * Cin;
  constexpr int C4 = BN / 4;
  for (int c = tid; c < BM * C4; c += kCT) {
    const int row = c / C4, c4 = c - row * C4;
    float4 v = *reinterpret_cast<const float4*>(E + row * ES + c4 * 4);
#pragma unroll
    for (int k = 1; k < WK; ++k) {
      const float4 u = *reinterpret_cast<const float4*>(E + (k * BM + row) * ES + c4 * 4);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    *reinterpret_cast<float4*>(out + (int64_t)(co0 + row) * Cin + ci0 + c4 * 4) = v;
  }
}

// Split-K partial reduction, two stages so that thousands of threads each keep
// several independent 16-byte loads in flight: stage 1 sums groups of splits
// (grid.y = group), stage 2 sums the groups and writes dW (KRSC, bf16 / fp32).
constexpr int kRedGroup = 16;  // splits per stage-1 group

__global__ void __launch_bounds__(256)
    wgrad_reduce1_k(const float4* __restrict__ part, int S, int64_t total4,
                    float4* __restrict__ stage) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total4) return;
  const int s0 = blockIdx.y * kRedGroup;
  int s1 = s0 + kRedGroup;
  if (s1 > S) s1 = S;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int s = s0;
  for (; s + 1 < s1; s += 2) {
    const float4 u = part[(int64_t)s * total4 + e], v = part[(int64_t)(s + 1) * total4 + e];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  if (s < s1) {
    const float4 u = part[(int64_t)s * total4 + e];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  stage[(int64_t)blockIdx.y * total4 + e] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// dW[co][tap][ci] (KRSC) = sum over groups of stage[group][tap][co][ci]
template <typename TO>
__global__ void __launch_bounds__(256)
    wgrad_reduce2_k(const float* __restrict__ stage, int Gn, int Cout, int Cin, TO* __restrict__ dw,
                    int taps, int accum) {
  const int64_t total = (int64_t)taps * Cout * Cin;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int ci = (int)(e % Cin);
  const int64_t r = e / Cin;
  const int co = (int)(r % Cout);
  const int tap = (int)(r / Cout);
  float sum = 0.f;
  for (int g = 0; g < Gn; ++g) sum += stage[(int64_t)g * total + e];
  TO* o = dw + ((int64_t)co * taps + tap) * Cin + ci;
  *o = from_f32<TO>(accum ? to_f32(*o) + sum : sum);
}

// Single-pass form for <= kRedGroup splits: sum the S slabs of 4 consecutive ci and
// write the final dtype / KRSC layout directly (no stage slab, one launch less).
template <typename TO>
__global__ void __launch_bounds__(256)
    wgrad_reduce_one_k(const float4* __restrict__ part, int S, int64_t total4, int Cout, int Cin,
                       int taps, TO* __restrict__ dw, int accum) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total4) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  int s = 0;
  for (; s + 1 < S; s += 2) {
    const float4 u = part[(int64_t)s * total4 + e], v = part[(int64_t)(s + 1) * total4 + e];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  if (s < S) {
    const float4 u = part[(int64_t)s * total4 + e];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  const int64_t el = e * 4;  // element index in [tap][co][ci]
  const int ci = (int)(el % Cin);
  const int64_t r = el / Cin;
  const int co = (int)(r % Cout);
  const int tap = (int)(r / Cout);
  TO* o = dw + ((int64_t)co * taps + tap) * Cin + ci;
  float v[4] = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
  if (accum) {  // accumulate into an existing gradient (a DDP bucket view): one rounding
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += to_f32(o[i]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = from_f32<TO>(v[i]);
}

// W'[ci][T-1-t][co] = W[co][t][ci]: the 180-degree-rotated, in/out-swapped 3x3
// filter of the data gradient (T = 9), or the plain transpose W^T of a 1x1 filter
// (T = 1), as a 64x64 LDS-tiled transpose per tap
__global__ void __launch_bounds__(256)
    rot_weight_k(const uint16_t* __restrict__ w, uint16_t* __restrict__ out, int Cout, int Cin,
                 int T) {
  __shared__ uint16_t tile[64][66];
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64, t = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  for (int r = ty; r < 64; r += 4) {
    const int co = co0 + r, ci = ci0 + tx;
    tile[r][tx] = (co < Cout && ci < Cin) ? w[((int64_t)co * T + t) * Cin + ci] : 0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < Cin && co < Cout) out[((int64_t)ci * T + (T - 1 - t)) * Cout + co] = tile[tx][r];
  }
}

// Every backward-pass weight layout of a model in ONE launch: the descriptors of up to
// kPrepMax filters travel in the kernel arguments; workgroup b finds its filter by the
// running tile offsets and does one 64x64 tap tile of rot_weight_k's transpose.
constexpr int kPrepMax = 48;
struct PrepDesc {
  const uint16_t* w;
  uint16_t* out;
  int Cout, Cin, T, tile0;
};
struct PrepArgs {
  int n, pad;
  PrepDesc d[kPrepMax];
};

__global__ void __launch_bounds__(256) prep_weights_k(PrepArgs a) {
  __shared__ uint16_t tile[64][66];
  int i = 0;
  while (i + 1 < a.n && (int)blockIdx.x >= a.d[i + 1].tile0) ++i;
  const PrepDesc d = a.d[i];
  const int local = (int)blockIdx.x - d.tile0;
  const int cot_n = (d.Cout + 63) / 64, cit_n = (d.Cin + 63) / 64;
  const int t = local / (cot_n * cit_n), rem = local - t * cot_n * cit_n;
  const int co0 = (rem / cit_n) * 64, ci0 = (rem % cit_n) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int co = co0 + r, ci = ci0 + tx;
    tile[r][tx] = (co < d.Cout && ci < d.Cin) ? d.w[((int64_t)co * d.T + t) * d.Cin + ci] : 0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < d.Cin && co < d.Cout)
      d.out[((int64_t)ci * d.T + (d.T - 1 - t)) * d.Cout + co] = tile[tx][r];
  }
}

// per-tap kernel tiling: 128 x 128 when both channel counts allow it, else 64 x 64
// (algo 2/3: tuning variants - deeper DMA ring with a shorter or equal K-tile)
struct WgTapCfg {
  int BM, BN, BK, NB;
};
WgTapCfg wg_tap_cfg(int Cin, int Cout, int algo) {
  if (Cin % 128 == 0 && Cout % 128 == 0) {
    if (algo == 2) return {128, 128, 32, 4};
    if (algo == 5) return {128, 128, 32, 3};
    if (algo == 3) return {128, 128, 64, 3};
    return {128, 128, 64, 2};
  }
  if (algo == 2) return {64, 64, 64, 3};
  if (algo == 3) return {64, 64, 128, 3};
  return {64, 64, 128, 2};
}

}  // namespace

bool conv3x3_nhwc_supported(int Cin, int Cout) { return Cin % 64 == 0 && Cout % 64 == 0; }

int conv_wgrad_splits(int N, int H, int W, int Cin, int Cout, int ksize, int stride, int algo) {
  if (algo == 4) {
    // one 8-wave workgroup per CU over (splits x 64 x 64 channel tiles); K-tile ranges of
    // whole images where possible (each image boundary costs a full strip load)
    const int kpi = (H * (W + 2) + kW64BK - 1) / kW64BK;
    const int total = N * kpi;
    const int tiles = (Cout / 64) * (Cin / 64);
    int S = 256 / tiles;
    if (S > N) S = N;
    if (S < 1) S = 1;
    return S > total ? total : S;
  }
  if (algo == 1) {
    const int kpi = (H * (W + 2) + kWgBK - 1) / kWgBK;  // K-tiles per image
    const int total = N * kpi;
    const int tiles = (Cout / 64) * (Cin / 64);
    int S = (512 + tiles - 1) / tiles;                  // ~2 workgroups per CU
    const int max_s = total / 8;                         // >= 8 K-tiles per workgroup
    if (S > max_s) S = max_s;
    return S < 1 ? 1 : S;
  }
  // per-tap kernel: pick the split count minimising (rounds of 512 workgroup slots =
  // 2 per CU) x (K-tiles per workgroup) x tile time + the fp32 partial traffic
  const int T = ksize * ksize;
  const WgTapCfg c = wg_tap_cfg(Cin, Cout, algo);
  const int64_t M = (int64_t)N * ((H - 1) / stride + 1) * ((W - 1) / stride + 1);
  const int total_kt = (int)((M + c.BK - 1) / c.BK);
  const int gx = T * (Cout / c.BM) * (Cin / c.BN);
  const int slots = c.BK * c.NB * (c.BM + c.BN) * 2 > 80 * 1024 ? 256 : 512;  // WGs per CU
  const double t_tile = 2.0 * c.BM * c.BN * c.BK / (4096.0 * 2400.0 * 0.5 / (slots / 256));  // us
  const double t_split = (double)T * Cout * Cin * 8.0 / 5.0e6;                     // us
  int best = 1;
  double best_cost = 1e30;
  const int smax = total_kt < 2048 ? total_kt : 2048;
  for (int S = 1; S <= smax; ++S) {
    const int kps = (total_kt + S - 1) / S;
    if (kps < 4 && S > 1) break;
    const int se = (total_kt + kps - 1) / kps;
    const int64_t rounds = ((int64_t)gx * se + slots - 1) / slots;
    const double cost = (double)rounds * kps * t_tile + se * t_split;
    if (cost < best_cost) {
      best_cost = cost;
      best = se;
    }
  }
  return best;
}

bool conv3x3_wgrad_supported(int W, int algo) { return (algo != 1 && algo != 4) || W <= kWgMaxW; }

// the strip-ring kernel's shapes: 3x3 stride 1, channels % 64 (64 x 64 tiles), W <= 56
bool conv3x3_wgrad_c64_ok(int W, int Cin, int Cout, int ksize, int stride) {
  return ksize == 3 && stride == 1 && Cin % 64 == 0 && Cout % 64 == 0 && W <= kWgMaxW;
}

int64_t conv_wgrad_workspace(int S, int Cin, int Cout, int ksize) {
  return (int64_t)(S + (S + kRedGroup - 1) / kRedGroup) * ksize * ksize * Cout * Cin;
}

void conv_nhwc_wgrad(const void* dy, const void* x, float* part, void* dw, bool dw_fp32, int N,
                     int H, int W, int Cin, int Cout, int ksize, int stride, int S, int algo,
                     hipStream_t st, bool accum) {
  const auto* dyp = static_cast<const bf16_t*>(dy);
  const auto* xp = static_cast<const bf16_t*>(x);
  const int T = ksize * ksize;
  if (algo == 4) {
    const int kpi = (H * (W + 2) + kW64BK - 1) / kW64BK;
    const int total = N * kpi;
    const int kps = (total + S - 1) / S;
    const unsigned tiles = (unsigned)((Cout / 64) * (Cin / 64));
    hipLaunchKernelGGL(conv3x3_wgrad_c64_k, dim3((unsigned)S, tiles), dim3(512), 0, st, dyp, xp,
                       part, H, W, kpi, kps, total, Cin, Cout);
  } else if (algo == 1) {
    const int kpi = (H * (W + 2) + kWgBK - 1) / kWgBK;
    const int total = N * kpi;
    const int kps = (total + S - 1) / S;
    const int tiles = (Cout / 64) * (Cin / 64);
    hipLaunchKernelGGL((conv3x3_wgrad9_k<3>), dim3(tiles, S), dim3(kCT), 0, st, dyp, xp, part,
                       H, W, Cin, Cout, kpi, kps, total);
  } else {
    const WgTapCfg c = wg_tap_cfg(Cin, Cout, algo);
    const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
    const int M = N * Ho * Wo;
    const int total_kt = (M + c.BK - 1) / c.BK;
    const int kps = (total_kt + S - 1) / S;
    const int gx = T * (Cout / c.BM) * (Cin / c.BN);
    const dim3 grid((unsigned)(gx * S));
#define WGT_LAUNCH(...)                                                                       \
  hipLaunchKernelGGL((conv3x3_wgrad_tap_k<__VA_ARGS__>), grid, dim3(kCT), 0, st, dyp, xp, part, \
                     H, W, Ho, Wo, stride, T, Cin, Cout, M, kps, total_kt, gx)
    const bool s1 = stride == 1;
    if (c.BM == 128) {
      if (c.BK == 32 && c.NB == 3 && s1) WGT_LAUNCH(128, 128, 2, 2, 1, 32, 3, true);
      else if (c.BK == 32 && c.NB == 3) WGT_LAUNCH(128, 128, 2, 2, 1, 32, 3, false);
      else if (c.BK == 32) WGT_LAUNCH(128, 128, 2, 2, 1, 32, 4, false);
      else if (c.NB == 3) WGT_LAUNCH(128, 128, 2, 2, 1, 64, 3, false);
      else if (s1) WGT_LAUNCH(128, 128, 2, 2, 1, 64, 2, true);
      else WGT_LAUNCH(128, 128, 2, 2, 1, 64, 2, false);
    } else {
      if (c.BK == 64) WGT_LAUNCH(64, 64, 1, 2, 2, 64, 3, false);
      else if (c.NB == 3) WGT_LAUNCH(64, 64, 1, 1, 4, 128, 3, false);
      else if (s1) WGT_LAUNCH(64, 64, 1, 1, 4, 128, 2, true);
      else WGT_LAUNCH(64, 64, 1, 1, 4, 128, 2, false);
    }
#undef WGT_LAUNCH
  }
  // two-stage reduction; `part` holds S partial slabs followed by ceil(S/16)
  // stage-1 slabs (conv_wgrad_workspace); one pass when S <= 16 (Cin % 4 == 0)
  const int64_t nout = (int64_t)T * Cout * Cin;
  const int Gn = (S + kRedGroup - 1) / kRedGroup;
  if (Gn == 1 && Cin % 4 == 0) {
    const int64_t n4 = nout / 4;
    const unsigned blocks = (unsigned)((n4 + 255) / 256);
    if (dw_fp32)
      hipLaunchKernelGGL((wgrad_reduce_one_k<float>), dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(part), S, n4, Cout, Cin, T,
                         static_cast<float*>(dw), accum ? 1 : 0);
    else
      hipLaunchKernelGGL((wgrad_reduce_one_k<bf16_t>), dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(part), S, n4, Cout, Cin, T,
                         static_cast<bf16_t*>(dw), accum ? 1 : 0);
    return;
  }
  float* stage = part + (int64_t)S * nout;
  const int64_t n4 = nout / 4;
  hipLaunchKernelGGL(wgrad_reduce1_k, dim3((unsigned)((n4 + 255) / 256), Gn), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(part), S, n4, reinterpret_cast<float4*>(stage));
  const unsigned blocks = (unsigned)((nout + 255) / 256);
  if (dw_fp32)
    hipLaunchKernelGGL((wgrad_reduce2_k<float>), dim3(blocks), dim3(256), 0, st, stage, Gn, Cout,
                       Cin, static_cast<float*>(dw), T, accum ? 1 : 0);
  else
    hipLaunchKernelGGL((wgrad_reduce2_k<bf16_t>), dim3(blocks), dim3(256), 0, st, stage, Gn, Cout,
                       Cin, static_cast<bf16_t*>(dw), T, accum ? 1 : 0);
}

int64_t splitk_reduce_workspace(int S, int64_t n) {
  return (int64_t)((S + kRedGroup - 1) / kRedGroup) * n;
}

void splitk_reduce(const float* part, int S, int Cout, int Cin, float* stage, void* out,
                   bool out_fp32, hipStream_t st, bool accum) {
  const int64_t n = (int64_t)Cout * Cin;
  const int Gn = (S + kRedGroup - 1) / kRedGroup;
  if (Gn == 1 && Cin % 4 == 0) {
    const int64_t n4 = n / 4;
    const unsigned blocks = (unsigned)((n4 + 255) / 256);
    if (out_fp32)
      hipLaunchKernelGGL((wgrad_reduce_one_k<float>), dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(part), S, n4, Cout, Cin, 1,
                         static_cast<float*>(out), accum ? 1 : 0);
    else
      hipLaunchKernelGGL((wgrad_reduce_one_k<bf16_t>), dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(part), S, n4, Cout, Cin, 1,
                         static_cast<bf16_t*>(out), accum ? 1 : 0);
    return;
  }
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(wgrad_reduce1_k, dim3((unsigned)((n4 + 255) / 256), Gn), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(part), S, n4, reinterpret_cast<float4*>(stage));
  const unsigned blocks = (unsigned)((n + 255) / 256);
  if (out_fp32)
    hipLaunchKernelGGL((wgrad_reduce2_k<float>), dim3(blocks), dim3(256), 0, st, stage, Gn, Cout,
                       Cin, static_cast<float*>(out), 1, accum ? 1 : 0);
  else
    hipLaunchKernelGGL((wgrad_reduce2_k<bf16_t>), dim3(blocks), dim3(256), 0, st, stage, Gn, Cout,
                       Cin, static_cast<bf16_t*>(out), 1, accum ? 1 : 0);
}

void conv3x3_rot_weight(const void* w, void* out, int Cout, int Cin, hipStream_t st) {
  hipLaunchKernelGGL(rot_weight_k, dim3((Cout + 63) / 64, (Cin + 63) / 64, 9), dim3(256), 0, st,
                     static_cast<const uint16_t*>(w), static_cast<uint16_t*>(out), Cout, Cin, 9);
}

void prep_weights(const void* const* w, void* const* out, const int* cout, const int* cin,
                  const int* taps, int n, hipStream_t st) {
  for (int b = 0; b < n; b += kPrepMax) {
    PrepArgs a;
    std::memset(&a, 0, sizeof(a));
    a.n = n - b < kPrepMax ? n - b : kPrepMax;
    int tiles = 0;
    for (int i = 0; i < a.n; ++i) {
      const int k = b + i;
      a.d[i] = PrepDesc{static_cast<const uint16_t*>(w[k]), static_cast<uint16_t*>(out[k]),
                        cout[k], cin[k], taps[k], tiles};
      tiles += ((cout[k] + 63) / 64) * ((cin[k] + 63) / 64) * taps[k];
    }
    if (tiles > 0) hipLaunchKernelGGL(prep_weights_k, dim3(tiles), dim3(256), 0, st, a);
  }
}

void conv1x1_transpose_weight(const void* w, void* out, int Cout, int Cin, hipStream_t st) {
  hipLaunchKernelGGL(rot_weight_k, dim3((Cout + 63) / 64, (Cin + 63) / 64, 1), dim3(256), 0, st,
                     static_cast<const uint16_t*>(w), static_cast<uint16_t*>(out), Cout, Cin, 1);
}

void conv_halo_enable(int mode) { g_conv_halo = mode; }
void conv_halo_mtile(int bm) { g_conv_halo_bm = bm; }
void conv_bnbwd_early(int mode) { g_bnbwd_early = mode; }
int conv_halo_enabled() { return g_conv_halo; }

// Stride-1 1x1 forwards on gemm4w (one wave per SIMD, 256 x 256 tiles; BN statistics in
// its EPI 3 epilogue): 0 off, 1 the measured winners, 2 every eligible shape (A/B).
// With the statistics epilogue, ResNet-50 bs 256 (tools/diag/conv1x1_g4w_bench.py,
// profiles/r6/conv1x1_g4w.md, us): 512->2048 @ 7 45 vs 53 (own kernel), 1024->256 @ 14
// 37 vs 45 (hipBLASLt, plus a statistics pass the own path would add), 64->256 @ 56 177 vs
// 178; the own kernel keeps 128->512 @ 28 (76 vs 97: two K-tiles per 256 x 256 tile leave
// gemm4w's epilogue exposed at one workgroup per CU), 256->1024 @ 14 (59 vs 68) and
// 2048->512 @ 7 (40 vs 48).  Off by default: in the model the table lost end to end
// (ResNet-50 same box 11,970 / 11,969 with it vs 12,040 / 12,020 without,
// profiles/r6/conv1x1_g4w.md) - gemm4w holds a whole CU (132 KB LDS, 512 registers per
// lane), so the side-stream weight-gradient kernels no longer overlap those convs.
int g_conv1x1_g4w = 0;

bool conv1x1_g4w(int64_t M, int Cin, int Cout, int stride) {
  if (g_conv1x1_g4w == 0 || stride != 1 || Cout % 256 != 0 || Cin % 64 != 0 ||
      M >= ((int64_t)1 << 31) || !gemm4w_supported((int)M, Cout, Cin))
    return false;
  if (g_conv1x1_g4w == 2) return true;
  return (Cin == 512 && Cout == 2048) || (Cin == 1024 && Cout == 256) ||
         (Cin == 64 && Cout == 256);
}
void conv_1x1_gemm4w(int mode) { g_conv1x1_g4w = mode; }
void conv_nfast(int mode) { g_conv_nfast = mode; }
void conv_halo_nfast(int on) { g_conv3h_nfast = on; }
bool conv_1x1_on_gemm4w(int64_t M, int Cin, int Cout) { return conv1x1_g4w(M, Cin, Cout, 1); }

int conv_fwd_mtiles(int N, int H, int W, int Cout, int stride, int ksize, int Cin) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t M = (int64_t)N * Ho * Wo;
  if (ksize == 3 && conv3h_ok(N, H, W, Cout, stride)) {
    const int bm = conv3h_mtile(N, H, W, Cout);
    return (int)((M + bm - 1) / bm);
  }
  if (ksize == 1 && conv1x1_g4w(M, Cin, Cout, stride)) return (int)((M + 255) / 256);
  return (int)((M + kBM - 1) / kBM);  // launch_conv_tap's M tile (EPI 0)
}

void conv_nhwc_fwd(const void* x, const void* w, void* y, int N, int H, int W, int Cin, int Cout,
                   int ksize, int stride, hipStream_t st, float* stats_slab,
                   const float* stats_shift) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const ConvGeom g{Ho, Wo, H, W, stride, Ho, Wo, 1, Cin, Cout, N * Ho * Wo, ksize * ksize * Cin};
  const auto* xp = static_cast<const bf16_t*>(x);
  const auto* wp = static_cast<const bf16_t*>(w);
  auto* yp = static_cast<bf16_t*>(y);
  if (ksize == 1 && conv1x1_g4w((int64_t)N * Ho * Wo, Cin, Cout, stride)) {
    // y[M, Cout] = x[M, Cin] . W[Cout, Cin]^T (NHWC rows, KRSC weight rows)
    GemmArgs a;
    std::memset(&a, 0, sizeof(a));
    a.A = x;
    a.B = w;
    a.C = y;
    a.M = N * Ho * Wo;
    a.N = Cout;
    a.K = Cin;
    a.lda = Cin;
    a.ldb = Cin;
    a.ldc = Cout;
    a.slab = stats_slab;
    a.shift = stats_shift;
    gemm4w(a, stats_slab ? 3 : 0, st);
    return;
  }
  if (ksize == 3 && conv3h_ok(N, H, W, Cout, stride))
    launch_conv3h<0>(xp, wp, yp, g, N, st, stats_slab, stats_shift, ConvBnEpi{});
  else if (ksize == 3) launch_conv_tap<kFwd3>(xp, wp, yp, g, st, stats_slab, stats_shift);
  else launch_conv_tap<kFwd1>(xp, wp, yp, g, st, stats_slab, stats_shift);
}

int conv_bnbwd_mtiles(int N, int H, int W, int Cout, int ksize, int Cin) {
  const int64_t M = (int64_t)N * H * W;
  // launch_conv_tap's M tile with the BN-backward epilogue (64 rows for the large 1x1s)
  if (ksize == 1 && Cout % 128 == 0 && M >= 50176 && Cin < 256) return (int)((M + 63) / 64);
  if (ksize == 3 && conv3h_ok(N, H, W, Cout, 1)) {
    const int bm = conv3h_mtile(N, H, W, Cout);
    return (int)((M + bm - 1) / bm);
  }
  return (int)((M + kBM - 1) / kBM);
}
void conv_nhwc_fwd_bnbwd(const void* dy, const void* w, void* gout, int N, int H, int W, int Cin,
                         int Cout, int ksize, int stride, const ConvBnEpi& ep, float* slab,
                         hipStream_t st) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const ConvGeom g{Ho, Wo, H, W, stride, Ho, Wo, 1, Cin, Cout, N * Ho * Wo, ksize * ksize * Cin};
  const auto* xp = static_cast<const bf16_t*>(dy);
  const auto* wp = static_cast<const bf16_t*>(w);
  auto* yp = static_cast<bf16_t*>(gout);
  if (ksize == 3 && stride == 1 && conv3h_ok(N, H, W, Cout, 1))
    launch_conv3h<1>(xp, wp, yp, g, N, st, slab, nullptr, ep);
  else if (ksize == 3) launch_conv_tap<kFwd3, 1>(xp, wp, yp, g, st, slab, nullptr, ep);
  else launch_conv_tap<kFwd1, 1>(xp, wp, yp, g, st, slab, nullptr, ep);
}

// Data gradient of a stride-2 conv (3x3 pad 1 or 1x1 pad 0; H = 2*Ho, W = 2*Wo), one
// launch over the 4 input-parity classes (kDgrad3 / kDgrad1 above), so no MFMA
// work is spent on the zeros of the dilated dY.  wt: 3x3 -> conv3x3_rot_weight(W);
// 1x1 -> W^T ([Cin][Cout]).
void conv_nhwc_dgrad_s2(const void* dy, const void* wt, void* dx, int N, int H, int W, int Cin,
                        int Cout, int ksize, hipStream_t st) {
  const int Ho = H / 2, Wo = W / 2;
  const ConvGeom g{Ho, Wo, Ho, Wo, 1, H, W, 2, Cout, Cin, N * Ho * Wo, ksize * ksize * Cout};
  const auto* dyp = static_cast<const bf16_t*>(dy);
  const auto* wp = static_cast<const bf16_t*>(wt);
  auto* dxp = static_cast<bf16_t*>(dx);
  if (ksize == 3) launch_conv_tap<kDgrad3>(dyp, wp, dxp, g, st);
  else launch_conv_tap<kDgrad1>(dyp, wp, dxp, g, st);
}

// conv_nhwc_dgrad_s2 with the BN-backward epilogue (ConvBnEpi, no residual add): the data
// gradient of a stride-2 3x3 conv whose input is a BN(+ReLU) output stores g = mask * dX and
// that BN's backward sums, slab [2][Cin][4 * ceil(N*Ho*Wo / 128)] (every input pixel belongs
// to exactly one parity class, so each g is final in its epilogue)
int conv_dgrad_s2_bnbwd_mtiles(int N, int H, int W) {
  const int64_t M = (int64_t)N * (H / 2) * (W / 2);
  return 4 * (int)((M + kBM - 1) / kBM);
}
void conv_nhwc_dgrad_s2_bnbwd(const void* dy, const void* wt, void* gout, int N, int H, int W,
                              int Cin, int Cout, const ConvBnEpi& ep, float* slab,
                              hipStream_t st) {
  const int Ho = H / 2, Wo = W / 2;
  const ConvGeom g{Ho, Wo, Ho, Wo, 1, H, W, 2, Cout, Cin, N * Ho * Wo, 9 * Cout};
  launch_conv_tap<kDgrad3, 1>(static_cast<const bf16_t*>(dy), static_cast<const bf16_t*>(wt),
                              static_cast<bf16_t*>(gout), g, st, slab, nullptr, ep);
}

}  // namespace amd
