// ResNet stem: 7x7 / stride 2 / pad 3 convolution of a 3-channel NHWC bf16 image
// to 64 channels, on the gfx950 matrix cores.
//
// MIOpen runs this layer at ~170 TFLOP/s (K = 147 is awkward for its tiles);
// here the layer is re-shaped around what the data looks like:
//   * the input is zero-padded once to [N][H+6][W+6][4] (8 bytes per pixel, the
//     4th channel zero), so a filter row r of output pixel (ho, wo) reads ONE
//     contiguous 56-byte window: padded row 2ho+r, pixels 2wo..2wo+6;
//   * K = 7 filter rows x 32 (7 pixels x 4 channels = 28, padded to the 32 of one
//     v_mfma_f32_16x16x32_bf16 step): the packed filter [64][7][32] has zeros at
//     the pad channel and at k = 28..31, so the MFMA may read the 8 bytes after a
//     window (the next pixel: finite data times a zero weight);
//   * all 112 output pixels of one output row read their r-windows from the same
//     padded input row: a wave computes a whole output row (64 channels x 112
//     pixels) from 7 input rows staged in LDS by global_load_lds, and the next
//     output row needs only 2 new input rows (stride 2) - an 8-slot ring of input
//     rows per wave, so each input byte is fetched from HBM/L2 about once;
//   * the accumulator is the transposed product (filter rows as the MFMA A
//     operand): a lane holds 4 consecutive output channels of one pixel; blocks
//     of 16 pixels are re-laid through a free ring slot so the output leaves as
//     fully coalesced 1 KiB stores (8-byte scattered stores ran at ~1/3 the rate).
// Weight gradient: dW^T[(r, s, c)][co] = sum_p Xwin_r[p][(s, c)] dY[p][co], the
// same windows read as transposed MFMA fragments (ds_read_b64_tr_b16 gathers 4
// pixels x 16 window elements with a 16-byte pixel stride), split-K over output
// rows into fp32 partials [S][64][256] reduced by the split-K slab reduction.
#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short v4s_t __attribute__((ext_vector_type(4)));

constexpr int kStemWaves = 8;            // 2 waves per SIMD
constexpr int kSlot = 2048;              // bytes per staged padded input row (Wp <= 256)
constexpr int kRing = 8;                 // input-row slots per wave
constexpr int kWRow = 464;               // LDS bytes per filter row (448 + 16: bank spread)
constexpr int kStemLds = kStemWaves * kRing * kSlot + 64 * kWRow;  // 160,768 B

__device__ uint4 g_stem_zero[4];

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// stage padded input row `key` (= img * Hp + row) into ring slot key & 7:
// 128 chunks of 16 B, those past the row read the zero page
__device__ __forceinline__ void stage_row(const bf16_t* __restrict__ xp, int64_t key, int cpr,
                                          unsigned char* ring, int lane) {
  unsigned char* dst = ring + (int)(key & (kRing - 1)) * kSlot;
  const bf16_t* src = xp + key * (int64_t)cpr * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = h * 64 + lane;
    glds16(c < cpr ? (const void*)(src + c * 8) : (const void*)g_stem_zero, dst + h * 1024);
  }
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16_t x = (bf16_t)a, y = (bf16_t)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

// x -> [N][H+6][W+6][4] zero-padded bf16
__global__ void __launch_bounds__(256)
    stem_pad_k(const bf16_t* __restrict__ x, bf16_t* __restrict__ xp, int N, int H, int W) {
  const int Hp = H + 6, Wp = W + 6;
  const int64_t total = (int64_t)N * Hp * Wp;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int wp = (int)(i % Wp);
  const int64_t q = i / Wp;
  const int hp = (int)(q % Hp);
  const int n = (int)(q / Hp);
  const int h = hp - 3, w = wp - 3;
  uint2 v = make_uint2(0u, 0u);
  if (h >= 0 && h < H && w >= 0 && w < W) {
    const uint16_t* s = reinterpret_cast<const uint16_t*>(x) + (((int64_t)n * H + h) * W + w) * 3;
    v.x = (uint32_t)s[0] | ((uint32_t)s[1] << 16);
    v.y = (uint32_t)s[2];
  }
  reinterpret_cast<uint2*>(xp)[i] = v;
}

// One wave = a run of consecutive output rows; IB = 16-pixel blocks per row.
template <int IB>
__global__ void __launch_bounds__(kStemWaves * 64, 1)
    stem_fwd_k(const bf16_t* __restrict__ xp, const bf16_t* __restrict__ wk,
               bf16_t* __restrict__ y, int Hp, int Wp, int Ho, int Wo, int total_rows,
               int rows_per_wave, float* __restrict__ slab, const float* __restrict__ shift) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[kStemLds];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  unsigned char* ring = lds + wid * kRing * kSlot;
  unsigned char* wimg = lds + kStemWaves * kRing * kSlot;
  // packed filter [64][224] -> LDS rows of kWRow bytes
  for (int c = tid; c < 64 * 28; c += kStemWaves * 64) {
    const int co = c / 28, q = c - co * 28;
    *reinterpret_cast<uint4*>(wimg + co * kWRow + q * 16) =
        *reinterpret_cast<const uint4*>(wk + co * 224 + q * 8);
  }
  __syncthreads();
  const int t0 = (blockIdx.x * kStemWaves + wid) * rows_per_wave;
  const int t1 = t0 + rows_per_wave < total_rows ? t0 + rows_per_wave : total_rows;
  // BatchNorm statistics of y for the stem BN (slab != null): a lane's output stores all
  // cover the same 8 channels (lane & 7), so it sums the bf16-ROUNDED values it stores
  // (exactly what y holds), shifted by the BN's running mean, and each wave writes one
  // column s of the channel-major slab [2][64][S] (S = waves in the grid) - the BN's
  // separate statistics pass over y (411 MB at bs 256) disappears.
  const int S = (int)gridDim.x * kStemWaves, sidx = (int)blockIdx.x * kStemWaves + wid;
  const int scg = lane & 7;
  float s1[8], s2[8], shv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s1[i] = s2[i] = 0.f;
    shv[i] = (slab != nullptr && shift != nullptr) ? shift[scg * 8 + i] : 0.f;
  }
  auto write_stats = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int m = 8; m < 64; m <<= 1) {
        s1[i] += __shfl_xor(s1[i], m);
        s2[i] += __shfl_xor(s2[i], m);
      }
    }
    if (lane < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        slab[(int64_t)(lane * 8 + i) * S + sidx] = s1[i];
        slab[(int64_t)(64 + lane * 8 + i) * S + sidx] = s2[i];
      }
    }
  };
  if (t0 >= t1) {  // wave-uniform, after the only workgroup barrier
    if (slab != nullptr) write_stats();
    return;
  }
  const int cpr = Wp / 2;  // 16-byte chunks per padded row
  const int fr = lane & 15, fg = lane >> 4;

  int n = t0 / Ho, ho = t0 - (t0 / Ho) * Ho;
  int64_t key0 = (int64_t)n * Hp + 2 * ho;
#pragma unroll
  for (int r = 0; r < 7; ++r) stage_row(xp, key0 + r, cpr, ring, lane);

  // Per row: the 2 new input rows of the next output row stream in during this
  // row's MFMAs (slot (key0-1)&7 is free at once, slot key0&7 after filter row 0's
  // reads), and the single vmcnt(0) before the stores then finds both those DMAs
  // and the previous row's stores long done.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int t = t0; t < t1; ++t) {
    const bool nxt = t + 1 < t1;
    const int n1 = (t + 1) / Ho, ho1 = (t + 1) - n1 * Ho;
    const int64_t key1 = (int64_t)n1 * Hp + 2 * ho1;
    const bool seq = nxt && key1 == key0 + 2;
    if (seq) stage_row(xp, key0 + 7, cpr, ring, lane);
    f32x4_t acc[4][IB];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < IB; ++i) acc[j][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      const unsigned char* S = ring + (int)((key0 + r) & (kRing - 1)) * kSlot;
      bf16x8 wf[4], pf[IB];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wf[j] = *reinterpret_cast<const bf16x8*>(wimg + (16 * j + fr) * kWRow + r * 64 + fg * 16);
#pragma unroll
      for (int i = 0; i < IB; ++i)
        pf[i] = *reinterpret_cast<const bf16x8*>(S + 16 * (16 * i + fr + fg));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < IB; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], pf[i], acc[j][i], 0, 0, 0);
      if (r == 0 && seq) {
        // filter row 0's window reads are complete: its slot takes input row key0+8
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage_row(xp, key0 + 8, cpr, ring, lane);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // C[co][pixel]: lane holds pixel 16i + fr, channels 16j + 4fg .. +3.  Each
    // 16-pixel block goes through the free ring slot of input row key0+1 (an XOR-
    // swizzled [16 px][128 B] image) and leaves as two fully coalesced 1 KiB
    // stores (16 consecutive output pixels = 2 KiB contiguous).
    unsigned char* X = ring + (int)((key0 + 1) & (kRing - 1)) * kSlot;
    bf16_t* yrow = y + (int64_t)t * Wo * 64;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int chunk = (2 * j + (fg >> 1)) ^ (fr & 7);
        uint2 v;
        v.x = pack_bf16x2(acc[j][i][0], acc[j][i][1]);
        v.y = pack_bf16x2(acc[j][i][2], acc[j][i][3]);
        *reinterpret_cast<uint2*>(X + fr * 128 + chunk * 16 + (fg & 1) * 8) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int px = h * 8 + (lane >> 3), c = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(X + px * 128 + ((c ^ (px & 7)) << 4));
        const int p = 16 * i + px;
        if (p < Wo) {
          *reinterpret_cast<uint4*>(yrow + p * 64 + c * 8) = v;
          if (slab != nullptr) {
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
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (nxt && !seq) {
      // next image: the 7 input rows of its first output row, synchronously
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int r = 0; r < 7; ++r) stage_row(xp, key1 + r, cpr, ring, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    key0 = key1;
  }
  if (slab != nullptr) write_stats();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// weight gradient.  Workgroup = 4 waves over the same run of output rows; wave w
// owns filter rows r = 2w, 2w+1 (r = 7 is a zero pad slot) x 32 window elements =
// 64 GEMM columns, all 64 output channels: acc = 64 x 64 per wave.  Per output row
// the K dimension is its Wo pixels (padded to a multiple of 32 with zero dY rows).
// dY rows of the output row are staged (128 B per pixel, tr-swizzled) by DMA.
constexpr int kWgWaves = 4;
constexpr int kWgMaxPix = 128;                       // Wo <= 128
constexpr int kDyBytes = kWgMaxPix * 128;            // 16 KB per dY row image
constexpr int kWgLds = 2 * kDyBytes + 2 * kRing * kSlot + 64;  // dY x2 + input rows x2 (+ tail
                                                                 // read by the padded k-steps)

__device__ __forceinline__ int dy_swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1)) << 4);
}

template <int KS>  // 32-pixel k-steps per output row
__global__ void __launch_bounds__(kWgWaves * 64, 2)
    stem_wgrad_k(const bf16_t* __restrict__ xp, const bf16_t* __restrict__ dy,
                 float* __restrict__ part, int Hp, int Wp, int Ho, int Wo, int total_rows,
                 int rows_per_wg) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[kWgLds];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  unsigned char* dyimg = lds;                         // 2 x kDyBytes
  unsigned char* ring = lds + 2 * kDyBytes;           // 2 x 8 slots: wave 0 stages, all read
  const int t0 = blockIdx.x * rows_per_wg;
  int t1 = t0 + rows_per_wg;
  if (t1 > total_rows) t1 = total_rows;
  const int cpr = Wp / 2;
  const int fr = lane & 15, fg = lane >> 4;

  f32x4_t acc[4][4];  // [co block][n block]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // staging of one output row t into buffer `buf`: dY rows (waves 0-3 share:
  // 128 rows x 128 B = 16 x 1 KB, 4 per wave) + the input rows it needs (wave 0..1:
  // 8 input rows 2ho..2ho+7 -> slots 0..7 of ring half `buf`; row 7 is unused data)
  auto stage = [&](int t, int buf) {
    const int n = t / Ho, ho = t - (t / Ho) * Ho;
    unsigned char* D = dyimg + buf * kDyBytes;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (wid * 4 + q) * 8 + (lane >> 3);     // pixel 0..127
      const int pc = lane & 7;
      const int chunk = (dy_swz(row, pc) - row * 128) >> 4;
      const void* src = row < Wo ? (const void*)(dy + ((int64_t)t * Wo + row) * 64 + chunk * 8)
                                 : (const void*)g_stem_zero;
      glds16(src, D + (wid * 4 + q) * 1024);
    }
    unsigned char* R = ring + buf * kRing * kSlot;
    const int64_t key0 = (int64_t)n * Hp + 2 * ho;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int r = wid * 2 + k;                     // 8 rows over 4 waves
      const int64_t key = key0 + (r < 7 ? r : 6);    // slot 7: any finite row
      const bf16_t* src = xp + key * (int64_t)cpr * 8;
      unsigned char* dst = R + r * kSlot;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = h * 64 + lane;
        glds16(c < cpr ? (const void*)(src + c * 8) : (const void*)g_stem_zero, dst + h * 1024);
      }
    }
  };
  constexpr int G = 4 + 4;  // glds per wave per stage

  if (t0 < t1) stage(t0, 0);
  for (int t = t0; t < t1; ++t) {
    const int buf = (t - t0) & 1;
    if (t + 1 < t1) {
      // the buffer of row t+1 was read at iteration t-1; every wave passed the
      // barrier at the end of that iteration
      stage(t + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const unsigned char* D = dyimg + buf * kDyBytes;
    const unsigned char* R = ring + buf * kRing * kSlot;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      // A = dY^T: rows co (16 per block), k = 8 consecutive pixels via tr reads
      const int kb = ks * 32 + fg * 8;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int col = 16 * a + 4 * (fr & 3);             // this lane's 4-column piece
        const int q = fr >> 2;
        const int chunk = col >> 3, half = (col >> 2) & 1;
        v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_t*)(D + dy_swz(kb + q, chunk) + 8 * half));
        v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_t*)(D + dy_swz(kb + 4 + q, chunk) + 8 * half));
        v4s_t* fp = reinterpret_cast<v4s_t*>(&af[a]);
        fp[0] = lo;
        fp[1] = hi;
      }
      // B = window elements: column block b -> filter row r = 2*wid + (b >> 1),
      // elements 16*(b & 1) .. +15 of its 32; pixel p's window starts at 16p bytes
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int r = 2 * wid + (b >> 1);
        const unsigned char* S = R + r * kSlot;
        const int q = fr >> 2;
        const int e = 16 * (b & 1) + 4 * (fr & 3);          // element offset in the window
        v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_t*)(S + 16 * (kb + q) + 2 * e));
        v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_t*)(S + 16 * (kb + 4 + q) + 2 * e));
        v4s_t* fp = reinterpret_cast<v4s_t*>(&bfr[b]);
        fp[0] = lo;
        fp[1] = hi;
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
  // partial [blockIdx.x][co][n = 64 * wid + 16 b + fr]
  float* out = part + (int64_t)blockIdx.x * 64 * 256;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        out[(16 * a + 4 * fg + e) * 256 + 64 * wid + 16 * b + fr] = acc[a][b][e];
}

}  // namespace

bool stem_conv_supported(int N, int H, int W) {
  return H % 2 == 0 && W % 2 == 0 && W + 6 <= 256 && W / 2 <= kWgMaxPix && N > 0 && H > 0;
}

void stem_pad(const void* x, void* xp, int N, int H, int W, hipStream_t st) {
  const int64_t total = (int64_t)N * (H + 6) * (W + 6);
  hipLaunchKernelGGL(stem_pad_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     static_cast<const bf16_t*>(x), static_cast<bf16_t*>(xp), N, H, W);
}

int stem_fwd_grid(int N, int H) {
  const int total_rows = N * (H / 2);
  const int grid = (total_rows + kStemWaves - 1) / kStemWaves;
  return grid > 256 ? 256 : grid;
}

int stem_fwd_slab_width(int N, int H) { return stem_fwd_grid(N, H) * kStemWaves; }

void stem_fwd(const void* xp, const void* wk, void* y, int N, int H, int W, hipStream_t st,
              float* slab, const float* shift) {
  const int Hp = H + 6, Wp = W + 6, Ho = H / 2, Wo = W / 2;
  const int total_rows = N * Ho;
  const int grid = stem_fwd_grid(N, H);
  const int rpw = (total_rows + grid * kStemWaves - 1) / (grid * kStemWaves);
  const auto* xpp = static_cast<const bf16_t*>(xp);
  const auto* wkp = static_cast<const bf16_t*>(wk);
  auto* yp = static_cast<bf16_t*>(y);
  const int ib = (Wo + 15) / 16;
#define STEM_FWD(IB)                                                                          \
  hipLaunchKernelGGL((stem_fwd_k<IB>), dim3(grid), dim3(kStemWaves * 64), 0, st, xpp, wkp, yp, \
                     Hp, Wp, Ho, Wo, total_rows, rpw, slab, shift)
  if (ib <= 1) STEM_FWD(1);
  else if (ib <= 2) STEM_FWD(2);
  else if (ib <= 4) STEM_FWD(4);
  else if (ib <= 7) STEM_FWD(7);
  else STEM_FWD(8);
#undef STEM_FWD
}

int stem_wgrad_splits(int N, int H) {
  const int total_rows = N * (H / 2);
  int S = 512;
  if (S > total_rows) S = total_rows;
  const int rpw = (total_rows + S - 1) / S;
  return (total_rows + rpw - 1) / rpw;
}

void stem_wgrad(const void* xp, const void* dy, float* part, int S, int N, int H, int W,
                hipStream_t st) {
  const int Hp = H + 6, Wp = W + 6, Ho = H / 2, Wo = W / 2;
  const int total_rows = N * Ho;
  const int rpw = (total_rows + S - 1) / S;
  const auto* xpp = static_cast<const bf16_t*>(xp);
  const auto* dyp = static_cast<const bf16_t*>(dy);
  const int ks = (Wo + 31) / 32;
#define STEM_WG(KS)                                                                            \
  hipLaunchKernelGGL((stem_wgrad_k<KS>), dim3(S), dim3(kWgWaves * 64), 0, st, xpp, dyp, part, \
                     Hp, Wp, Ho, Wo, total_rows, rpw)
  if (ks <= 1) STEM_WG(1);
  else if (ks <= 2) STEM_WG(2);
  else if (ks <= 3) STEM_WG(3);
  else STEM_WG(4);
#undef STEM_WG
}

}  // namespace amd
