// Channels-last (NHWC) BatchNorm kernels for gfx950: x viewed as [M, C],
// M = N*H*W.  apex csrc/welford.cu *_c_last semantics.
//
// Layout of work: a lane owns W = 8 consecutive channels (one 16-byte bf16
// load, VEC path) or 1 channel (scalar path for C % 8 != 0 / unaligned data);
// `ctile` lanes cover a row segment of up to 512 channels and the remaining
// lanes of the 256-thread workgroup take further rows (rows_iter >= 4), so the
// per-channel constants and accumulators of a lane never change while it
// streams rows.  Every loop keeps 2-4 independent rows (16-B loads) in flight
// per lane.  Reductions write per-split partial slabs summed by the shared
// finalize kernel (bn_common.h): deterministic, no atomics.
//
// ReLU bitmask: when the forward applies ReLU after a residual add (y =
// relu(bn(x) + z)) it can also write one bit per element (which outputs were
// > 0; one byte per lane's 8 channels per row, 1/16 of a bf16 tensor).  The
// backward passes then read the mask instead of re-reading z to recompute the
// ReLU condition: two full reads of the residual tensor per layer become two
// reads of 1/16 of it, and z need not be kept alive for backward.
#include <cstdio>
#include <cstdlib>

#include "bn_common.h"

namespace amd {

namespace {

struct NGeom {
  int ctile, rows_iter, cblocks;
};

NGeom ngeom(int64_t C, bool vec) {
  NGeom g;
  int64_t cv = vec ? C / 8 : C;
  g.ctile = (int)(cv < 64 ? cv : 64);
  if (g.ctile < 1) g.ctile = 1;
  g.rows_iter = kBNThreads / g.ctile;
  g.cblocks = (int)((cv + g.ctile - 1) / g.ctile);
  return g;
}

}  // namespace

namespace {
thread_local bool g_bn_grad_accumulate = false;
}
bool bn_grad_accumulate() { return g_bn_grad_accumulate; }
void bn_set_grad_accumulate(bool on) { g_bn_grad_accumulate = on; }

BNTuning& bn_tuning() {
  static BNTuning t;
  return t;
}

// rows in flight per lane: 4 in stats_k, 2 in reduce_k and in the elementwise passes
// (apply_k, backward_k).  Same-box A/Bs (profiles/r4/ze/, microbench_bn_eu.txt): "4,4" /
// "8,4" reduction unrolls -2.2 / -2.3 %, 4 elementwise rows in flight -3.4 %.

namespace {

// reduction grid: rows per thread `red_rpt`, at most `red_cap` blocks in total,
// but at least `red_min` blocks (when every thread still gets >= 2 rows) so
// small layers fill the 256 CUs
int reduce_splits(int64_t M, const NGeom& g) {
  const BNTuning& t = bn_tuning();
  int64_t want = (M + (int64_t)g.rows_iter * t.red_rpt - 1) / ((int64_t)g.rows_iter * t.red_rpt);
  const int64_t floor_splits = t.red_min / g.cblocks;
  const int64_t max_by_rows = M / ((int64_t)g.rows_iter * 2);
  if (want < floor_splits) want = floor_splits < max_by_rows ? floor_splits : max_by_rows;
  int64_t cap = t.red_cap / g.cblocks;
  if (cap < 1) cap = 1;
  if (want > cap) want = cap;
  return (int)(want < 1 ? 1 : want);
}

// rows per thread of the elementwise passes.  A per-shape rule from the isolated
// sweep (tools/microbench.py bn-eu, profiles/microbench_bn_eu.txt): tensors larger
// than the 256 MB Infinity Cache at 8 rows per thread, smaller ones at the most rows
// per thread (up to 32) that still leaves >= 384 workgroups.  It cut apply + backward
// 4 % R50-weighted in isolation but measured 0.25 % SLOWER in the training step
// (same-box A/B, 9662 vs 9687 img/s: the isolated loop re-reads a cache-warm tensor),
// so the fixed elem_rpt (8 since the constants moved to LDS, bn_common.h) stays the
// default; bn_set_tuning(elem_rpt=0) selects the rule.
int elem_rpt_for(int64_t M, const NGeom& g, int64_t bytes) {
  const BNTuning& t = bn_tuning();
  if (!t.elem_auto) return t.elem_rpt;
  if (bytes > (int64_t)256 << 20) return 8;
  for (int r = 32; r > 8; r >>= 1) {
    const int64_t blocks = (M + (int64_t)g.rows_iter * r - 1) / ((int64_t)g.rows_iter * r) * g.cblocks;
    if (blocks >= 384) return r;
  }
  return 8;
}

int elem_blocks(int64_t M, const NGeom& g, int64_t bytes) {
  const BNTuning& t = bn_tuning();
  const int rpt = elem_rpt_for(M, g, bytes);
  int64_t want = (M + (int64_t)g.rows_iter * rpt - 1) / ((int64_t)g.rows_iter * rpt);
  const int64_t floor_blocks = t.elem_min / g.cblocks;
  const int64_t max_by_rows = M / ((int64_t)g.rows_iter * 2);
  if (want < floor_blocks) want = floor_blocks < max_by_rows ? floor_blocks : max_by_rows;
  int64_t cap = t.elem_cap / g.cblocks;
  if (cap < 1) cap = 1;
  if (want > cap) want = cap;
  return (int)(want < 1 ? 1 : want);
}

template <typename T, int W>
__device__ __forceinline__ void ldw(const T* p, float (&v)[W]) {
  if constexpr (W == 8) load8(p, v);
  else v[0] = to_f32(p[0]);
}
template <typename T, int W>
__device__ __forceinline__ void stw(T* p, const float (&v)[W]) {
  if constexpr (W == 8) store8(p, v);
  else p[0] = from_f32<T>(v[0]);
}

// combine the rows_iter row-groups of a block (same lane channel set) via LDS and
// write the block's partial slab row: slab[blockIdx.x][0|1][C]
template <int W>
__device__ __forceinline__ void block_slab_write(float (&s1)[W], float (&s2)[W], int ci, int ri,
                                                 int ctile, int rows_iter, int c0, int C,
                                                 float* __restrict__ slab) {
  __shared__ float lds[2][kBNThreads * W];
  if (threadIdx.x < rows_iter * ctile) {
#pragma unroll
    for (int i = 0; i < W; ++i) {
      lds[0][(ri * ctile + ci) * W + i] = s1[i];
      lds[1][(ri * ctile + ci) * W + i] = s2[i];
    }
  }
  __syncthreads();
  if (ri == 0 && c0 < C) {
    for (int r = 1; r < rows_iter; ++r) {
#pragma unroll
      for (int i = 0; i < W; ++i) {
        s1[i] += lds[0][(r * ctile + ci) * W + i];
        s2[i] += lds[1][(r * ctile + ci) * W + i];
      }
    }
    float* o = slab + (size_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      o[c0 + i] = s1[i];
      o[C + c0 + i] = s2[i];
    }
  }
}

// block_slab_write with a CHANNEL-MAJOR slab [2][C][gridDim.x] (the layout the conv epilogues
// write; bn_slab_reduce_grad reads each channel's partials as one contiguous row - the
// row-major [blocks][2][C] form read column-wise cost ~40 us per finalize at the
// elementwise grid's block counts)
template <int W>
__device__ __forceinline__ void block_slab_write_cm(float (&s1)[W], float (&s2)[W], int ci,
                                                    int ri, int ctile, int rows_iter, int c0,
                                                    int C, float* __restrict__ slab) {
  __shared__ float lds[2][kBNThreads * W];
  if (threadIdx.x < rows_iter * ctile) {
#pragma unroll
    for (int i = 0; i < W; ++i) {
      lds[0][(ri * ctile + ci) * W + i] = s1[i];
      lds[1][(ri * ctile + ci) * W + i] = s2[i];
    }
  }
  __syncthreads();
  if (ri == 0 && c0 < C) {
    for (int r = 1; r < rows_iter; ++r) {
#pragma unroll
      for (int i = 0; i < W; ++i) {
        s1[i] += lds[0][(r * ctile + ci) * W + i];
        s2[i] += lds[1][(r * ctile + ci) * W + i];
      }
    }
    const int64_t S = gridDim.x;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      slab[(int64_t)(c0 + i) * S + blockIdx.x] = s1[i];
      slab[(int64_t)(C + c0 + i) * S + blockIdx.x] = s2[i];
    }
  }
}

// ---------------------------------------------------------------- statistics
template <typename T, bool VEC, int U>
__global__ void __launch_bounds__(kBNThreads)
    stats_k(const T* __restrict__ x, int64_t M, int C, int ctile, int rows_iter,
            float* __restrict__ slab) {
  constexpr int W = VEC ? 8 : 1;
  const int ci = threadIdx.x % ctile, ri = threadIdx.x / ctile;
  const int c0 = (blockIdx.y * ctile + ci) * W;
  const bool active = ri < rows_iter && c0 < C;
  const int64_t per = (M + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < M ? r0 + per : M;
  float k[W], s1[W], s2[W];
#pragma unroll
  for (int i = 0; i < W; ++i) k[i] = s1[i] = s2[i] = 0.f;
  if (active) {
    ldw<T, W>(x + c0, k);  // shift = row 0: identical in every split
    for (int64_t r = r0 + ri; r < r1; r += (int64_t)rows_iter * U) {
      float v[U][W];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = r + (int64_t)u * rows_iter;
#pragma unroll
        for (int i = 0; i < W; ++i) v[u][i] = k[i];  // unused slot -> d = 0
        if (rr < r1) ldw<T, W>(x + rr * C + c0, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < W; ++i) {
          const float d = v[u][i] - k[i];
          s1[i] += d;
          s2[i] = fmaf(d, d, s2[i]);
        }
    }
  }
  block_slab_write<W>(s1, s2, ci, ri, ctile, rows_iter, c0, C, slab);
}

// ---------------------------------------------------------------- apply
// channels of one elementwise-pass workgroup: ctile <= 64 lanes x 8 (ngeom)
constexpr int kBNBlockChans = 64 * 8;

// per-channel constants of the workgroup's channel range [cb, cb + n) computed once,
// one channel per thread (f(c, slot) writes LDS slot c - cb), then a barrier - every
// thread of the block must call this before any early exit
template <typename F>
__device__ __forceinline__ void stage_params(int C, int cb, int n, F&& f) {
  const int lim = cb + n < C ? n : C - cb;
  for (int k = threadIdx.x; k < lim; k += blockDim.x) f(cb + k, k);
  __syncthreads();
}

// ZZ (compile time): a residual z is added.  Loads are issued for all U rows first
// (clamped rows, no branches) and pinned ahead of the arithmetic: with `if (z)` and
// `if (rr < M)` around them the compiler waited vmcnt(0) after every row's loads (one row
// in flight per lane, ISA of the round-5 build).
//
// ZA (with ZZ): z is the RAW input of a second BatchNorm (ResNet's downsample BN) whose
// affine (meanz, invstdz, wz, bz) is applied here on load, rounded to T exactly as that BN's
// own apply pass would have stored it - y is bitwise the unfused result and that BN's
// output is never materialised (its apply pass, a read and a write of the tensor, goes).
template <typename T, typename TW, bool VEC, int U, bool ZZ, bool ZA = false>
__global__ void __launch_bounds__(kBNThreads)
    apply_k(const T* __restrict__ x, const float* __restrict__ mean,
            const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
            const T* __restrict__ z, T* __restrict__ y, uint8_t* __restrict__ rmask, int64_t M,
            int C, int ctile, int rows_iter, int relu, const float* __restrict__ meanz = nullptr,
            const float* __restrict__ invstdz = nullptr, const TW* __restrict__ wz = nullptr,
            const TW* __restrict__ bz = nullptr) {
  constexpr int W = VEC ? 8 : 1;
  const int Cb = C >> 3;
  const int ci = threadIdx.x % ctile, ri = threadIdx.x / ctile;
  const int c0 = (blockIdx.y * ctile + ci) * W;
  // the block's channel parameters, one channel per thread, staged in LDS
  __shared__ __attribute__((aligned(16))) float s_par[ZA ? 4 : 2][kBNBlockChans];
  const int cb = blockIdx.y * ctile * W;
  stage_params(C, cb, ctile * W, [&](int c, int k) {
    chan_affine(mean, invstd, wload(w, c, 1.f), wload(b, c, 0.f), c, s_par[0][k], s_par[1][k]);
    if constexpr (ZA)
      chan_affine(meanz, invstdz, wload(wz, c, 1.f), wload(bz, c, 0.f), c, s_par[ZA ? 2 : 0][k],
                  s_par[ZA ? 3 : 1][k]);
  });
  if (ri >= rows_iter || c0 >= C) return;
  float sc[W], sh[W], scz[W], shz[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    sc[i] = s_par[0][c0 - cb + i];
    sh[i] = s_par[1][c0 - cb + i];
    scz[i] = ZA ? s_par[ZA ? 2 : 0][c0 - cb + i] : 0.f;
    shz[i] = ZA ? s_par[ZA ? 3 : 1][c0 - cb + i] : 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * rows_iter;
  for (int64_t r = (int64_t)blockIdx.x * rows_iter + ri; r < M; r += stride * U) {
    float v[U][W], zz[U][W];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = r + (int64_t)u * stride;
      const int64_t rc = rr < M ? rr : M - 1;
      ldw<T, W>(x + rc * C + c0, v[u]);
      if constexpr (ZZ) ldw<T, W>(z + rc * C + c0, zz[u]);
    }
    asm volatile("" ::: "memory");  // every load of the group issues before any store
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = r + (int64_t)u * stride;
      if (rr >= M) continue;
      uint32_t mb = 0;
#pragma unroll
      for (int i = 0; i < W; ++i) {
        float o = fmaf(v[u][i], sc[i], sh[i]);
        if constexpr (ZA) {
          o += to_f32(from_f32<T>(fmaf(zz[u][i], scz[i], shz[i])));
        } else if constexpr (ZZ) {
          o += zz[u][i];
        }
        mb |= (o > 0.f ? 1u : 0u) << i;
        v[u][i] = relu ? fmaxf(o, 0.f) : o;
      }
      stw<T, W>(y + rr * C + c0, v[u]);
      if constexpr (W == 8) {
        if (rmask) rmask[rr * Cb + (c0 >> 3)] = (uint8_t)mb;
      }
    }
  }
}

// ---------------------------------------------------------------- backward reduce
// RM (compile time): 0 no ReLU, 1 ReLU from the 1-bit mask, 2 ReLU recomputed with the
// residual z, 3 ReLU recomputed without z.  With the mode a runtime flag the loop was
// branches around every load, each followed by a vmcnt(0) wait (1-2 loads in flight:
// 2.15 TB/s, profiles/r4/zd); rows past the split end load a clamped (valid) row and
// contribute exactly what the old zero-filled slot did.
template <typename T, typename TW, bool VEC, int U, int RM>
__global__ void __launch_bounds__(kBNThreads)
    reduce_k(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
             const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
             const T* __restrict__ z, const uint8_t* __restrict__ rmask, int64_t M,
             int C, int ctile, int rows_iter, float* __restrict__ slab) {
  constexpr int W = VEC ? 8 : 1;
  const int Cb = C >> 3;
  const int ci = threadIdx.x % ctile, ri = threadIdx.x / ctile;
  const int c0 = (blockIdx.y * ctile + ci) * W;
  const bool active = ri < rows_iter && c0 < C;
  const int64_t per = (M + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < M ? r0 + per : M;
  float mu[W], sc[W], sh[W], s1[W], s2[W];
#pragma unroll
  for (int i = 0; i < W; ++i) mu[i] = sc[i] = sh[i] = s1[i] = s2[i] = 0.f;
  __shared__ __attribute__((aligned(16))) float s_par[3][kBNBlockChans];
  const int cb = blockIdx.y * ctile * W;
  stage_params(C, cb, ctile * W, [&](int c, int k) {
    s_par[0][k] = mean[c];
    chan_affine(mean, invstd, wload(w, c, 1.f), wload(b, c, 0.f), c, s_par[1][k], s_par[2][k]);
  });
  if (active) {
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const int k = c0 - cb + i;
      mu[i] = s_par[0][k];
      sc[i] = s_par[1][k];
      sh[i] = s_par[2][k];
    }
    for (int64_t r = r0 + ri; r < r1; r += (int64_t)rows_iter * U) {
      float xv[U][W], dv[U][W], zv[U][W];
      uint32_t mk[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = r + (int64_t)u * rows_iter;
        ok[u] = rr < r1;
        const int64_t rc = ok[u] ? rr : r1 - 1;
        ldw<T, W>(x + rc * C + c0, xv[u]);
        ldw<T, W>(dy + rc * C + c0, dv[u]);
        mk[u] = 0;
        if constexpr (RM == 1) mk[u] = rmask[rc * Cb + (c0 >> 3)];
        if constexpr (RM == 2) ldw<T, W>(z + rc * C + c0, zv[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < W; ++i) {
          float d = dv[u][i];
          if constexpr (RM == 1) {
            d = ((mk[u] >> ((c0 + i) & 7)) & 1u) ? d : 0.f;
          } else if constexpr (RM >= 2) {
            float o = fmaf(xv[u][i], sc[i], sh[i]);
            if constexpr (RM == 2) o += zv[u][i];
            d = o > 0.f ? d : 0.f;
          }
          d = ok[u] ? d : 0.f;
          const float xe = ok[u] ? xv[u][i] : 0.f;
          s1[i] += d;
          s2[i] = fmaf(d, xe - mu[i], s2[i]);
        }
    }
  }
  block_slab_write<W>(s1, s2, ci, ri, ctile, rows_iter, c0, C, slab);
}

// ---------------------------------------------------------------- backward elementwise
// dx = dy'*k1 + x*k2 + k3  with  k1 = invstd*w, k2 = -invstd^3*w*mean(dy'(x-mu)),
//                                 k3 = -invstd*w*mean(dy') - k2*mu ;  dz = dy'
// RM: the ReLU mode of reduce_k, compile time (rows past M load a clamped row; their
// results are never stored)
//
// X2: the same pass also forms the backward sums of a SECOND BatchNorm whose output was this
// one's residual input z (ResNet's downsample BN: its gradient is this BN's d = dy'):
// sum(d), sum(d * (x2 - mean2)) per block into a channel-major slab2 [2][C][blocks] (for
// bn_slab_reduce_grad) - that BN's own reduction pass, which re-reads d, disappears.
template <typename T, typename TW, bool VEC, int U, int RM, bool X2 = false>
__global__ void __launch_bounds__(kBNThreads)
    backward_k(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
               const float* __restrict__ invstd, const TW* __restrict__ w,
               const TW* __restrict__ b, const float* __restrict__ sum_dy,
               const float* __restrict__ sum_dy_xmu, float inv_n,
               const T* __restrict__ z, const uint8_t* __restrict__ rmask, T* __restrict__ dx,
               T* __restrict__ dz, int64_t M, int C, int ctile, int rows_iter,
               const T* __restrict__ x2 = nullptr, const float* __restrict__ mean2 = nullptr,
               float* __restrict__ slab2 = nullptr) {
  constexpr int W = VEC ? 8 : 1;
  const int Cb = C >> 3;
  const int ci = threadIdx.x % ctile, ri = threadIdx.x / ctile;
  const int c0 = (blockIdx.y * ctile + ci) * W;
  // the block's channel constants, one channel per thread, staged in LDS (per thread
  // they were ~7 scalar global loads per channel x 8 channels beside 16 rows of data)
  __shared__ __attribute__((aligned(16))) float s_par[X2 ? 6 : 5][kBNBlockChans];
  const int cb = blockIdx.y * ctile * W;
  stage_params(C, cb, ctile * W, [&](int c, int k) {
    const float wc = wload(w, c, 1.f);
    chan_affine(mean, invstd, wc, wload(b, c, 0.f), c, s_par[0][k], s_par[1][k]);
    const float is = invstd[c];
    const float mdy = sum_dy[c] * inv_n, mdyx = sum_dy_xmu[c] * inv_n;
    const float q1 = is * wc, q2 = -is * is * is * wc * mdyx;
    s_par[2][k] = q1;
    s_par[3][k] = q2;
    s_par[4][k] = -is * wc * mdy - q2 * mean[c];
    if constexpr (X2) s_par[X2 ? 5 : 0][k] = mean2[c];
  });
  float t1[W], t2[W], m2[W];
#pragma unroll
  for (int i = 0; i < W; ++i) t1[i] = t2[i] = m2[i] = 0.f;
  const bool active = ri < rows_iter && c0 < C;
  if (!X2 && !active) return;
  float sc[W], sh[W], k1[W], k2[W], k3[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const int k = active ? c0 - cb + i : 0;
    sc[i] = s_par[0][k];
    sh[i] = s_par[1][k];
    k1[i] = s_par[2][k];
    k2[i] = s_par[3][k];
    k3[i] = s_par[4][k];
    if constexpr (X2) m2[i] = s_par[X2 ? 5 : 0][k];
  }
  const int64_t stride = (int64_t)gridDim.x * rows_iter;
  for (int64_t r = (int64_t)blockIdx.x * rows_iter + ri; active && r < M; r += stride * U) {
    float xv[U][W], dv[U][W], zv[U][W], x2v[X2 ? U : 1][W];
    uint32_t mk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = r + (int64_t)u * stride;
      const int64_t rc = rr < M ? rr : M - 1;
      mk[u] = 0;
      ldw<T, W>(x + rc * C + c0, xv[u]);
      ldw<T, W>(dy + rc * C + c0, dv[u]);
      if constexpr (RM == 1) mk[u] = rmask[rc * Cb + (c0 >> 3)];
      if constexpr (RM == 2) ldw<T, W>(z + rc * C + c0, zv[u]);
      if constexpr (X2) ldw<T, W>(x2 + rc * C + c0, x2v[u]);
    }
    asm volatile("" ::: "memory");  // every load of the group issues before any store
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = r + (int64_t)u * stride;
      if (rr >= M) continue;
#pragma unroll
      for (int i = 0; i < W; ++i) {
        float d = dv[u][i];
        if constexpr (RM == 1) {
          d = ((mk[u] >> ((c0 + i) & 7)) & 1u) ? d : 0.f;
        } else if constexpr (RM >= 2) {
          float o = fmaf(xv[u][i], sc[i], sh[i]);
          if constexpr (RM == 2) o += zv[u][i];
          d = o > 0.f ? d : 0.f;
        }
        dv[u][i] = d;
        xv[u][i] = fmaf(d, k1[i], fmaf(xv[u][i], k2[i], k3[i]));
        if constexpr (X2) {
          t1[i] += d;
          t2[i] = fmaf(d, x2v[u][i] - m2[i], t2[i]);
        }
      }
      stw<T, W>(dx + rr * C + c0, xv[u]);
      if (dz) stw<T, W>(dz + rr * C + c0, dv[u]);
    }
  }
  if constexpr (X2) block_slab_write_cm<W>(t1, t2, ci, ri, ctile, rows_iter, c0, C, slab2);
}


// ---------------------------------------------------------------- statistics from a
// producer's epilogue (conv_igemm.hip conv_tap_k with a stats slab): the conv wrote the
// shifted sums of each M-tile channel-major, slab[0|1][C][S].  ONE finalize launch sums
// each channel's S tile sums - a contiguous row - with TPC = 256 / CH threads per channel
// (CH channels per workgroup, chosen so each thread adds ~16 values with its loads in
// flight), fixed-order tree in LDS, and produces what stats_finalize does (mean, biased
// var | invstd, running stats, num_batches_tracked += 1) or, for a BN-backward slab,
// what reduce_finalize does.  Round 6: this replaced a fold kernel (32 tile rows at a
// time) + a finalize kernel over the tile-major [S][2][C] layout: ~10 us and two
// launches per BatchNorm on ResNet-50's 56 x 56 layers (profiles/r5/serial/).
constexpr int kSlabPerThread = 16;

static int slab_ch(int S) {
  int ch = 1;
  while (ch < 32 && (int64_t)S * ch * 2 <= (int64_t)kBNThreads * kSlabPerThread) ch *= 2;
  return ch;
}

// (sum of row 0 of channel c, sum of row 1) for the CH channels of this workgroup, into
// out[2 * CH] (LDS); TPC threads per channel, each summing a strided subset in 4 chains
template <int CH>
__device__ __forceinline__ void slab_t_sum(const float* __restrict__ slab, int S, int C, int c0,
                                           float* out) {
  constexpr int TPC = kBNThreads / CH;
  __shared__ float red[2][kBNThreads];
  const int k = threadIdx.x / TPC, t = threadIdx.x - k * TPC;
  const int c = c0 + k;
  // 8 chains per row: 16 independent loads in flight per thread (the 64-row-tile slabs
  // of the 56 x 56 BN-backward convs hold S = 12,544 sums per channel)
  float a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = b[u] = 0.f;
  if (c < C) {
    const float* r0 = slab + (int64_t)c * S;
    const float* r1 = slab + (int64_t)(C + c) * S;
    int s = t;
    for (; s + 7 * TPC < S; s += 8 * TPC) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        va[u] = r0[s + u * TPC];
        vb[u] = r1[s + u * TPC];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] += va[u];
        b[u] += vb[u];
      }
    }
    for (; s < S; s += TPC) {
      a[0] += r0[s];
      b[0] += r1[s];
    }
  }
  red[0][threadIdx.x] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  red[1][threadIdx.x] = ((b[0] + b[1]) + (b[2] + b[3])) + ((b[4] + b[5]) + (b[6] + b[7]));
  __syncthreads();
#pragma unroll
  for (int w = TPC / 2; w > 0; w >>= 1) {
    if (t < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (t == 0) {
    out[k] = red[0][threadIdx.x];
    out[CH + k] = red[1][threadIdx.x];
  }
  __syncthreads();
}

template <int CH>
__global__ void __launch_bounds__(kBNThreads)
    slab_stats_k(const float* __restrict__ slab, int S, int C, int64_t count,
                 const float* __restrict__ shift, BNStatsOut out) {
  __shared__ float sums[2 * CH];
  const int c0 = blockIdx.x * CH;
  slab_t_sum<CH>(slab, S, C, c0, sums);
  const int k = threadIdx.x;
  if (k < CH && c0 + k < C) {
    const int c = c0 + k;
    const float sh = shift ? shift[c] : 0.f;  // read before running_mean is updated
    const double m = (double)sums[k] / (double)count;
    double v = (double)sums[CH + k] / (double)count - m * m;
    if (v < 0.0) v = 0.0;
    const float mean = (float)((double)sh + m);
    out.mean[c] = mean;
    if (out.var) out.var[c] = (float)v;
    if (out.invstd) out.invstd[c] = rsqrtf((float)v + out.eps);
    if (out.running_mean) {
      const double unb = count > 1 ? v * (double)count / (double)(count - 1) : v;
      out.running_mean[c] = (1.f - out.momentum) * out.running_mean[c] + out.momentum * mean;
      out.running_var[c] = (1.f - out.momentum) * out.running_var[c] + out.momentum * (float)unb;
    }
    if (out.nbt && c == 0) *out.nbt += 1;
    if (out.count_out && c == 0) *out.count_out = out.count_val;
  }
}

template <typename TW, int CH>
__global__ void __launch_bounds__(kBNThreads)
    slab_reduce_k(const float* __restrict__ slab, int S, int C, const float* __restrict__ invstd,
                  float* __restrict__ sum_dy, float* __restrict__ sum_dy_xmu, TW* __restrict__ gw,
                  TW* __restrict__ gb, const float* __restrict__ sum_scale, int accum) {
  __shared__ float sums[2 * CH];
  const int c0 = blockIdx.x * CH;
  slab_t_sum<CH>(slab, S, C, c0, sums);
  const int k = threadIdx.x;
  if (k < CH && c0 + k < C) {
    const int c = c0 + k;
    const float s1 = sums[k], s2 = sums[CH + k];
    // SyncBN: the sums leave pre-divided by the global count (device scalar)
    const float sc = sum_scale ? *sum_scale : 1.f;
    sum_dy[c] = s1 * sc;
    sum_dy_xmu[c] = s2 * sc;
    // accum: add into existing gradients (DDP bucket views) instead of overwriting
    if (gw) gw[c] = from_f32<TW>(s2 * invstd[c] + (accum ? to_f32(gw[c]) : 0.f));
    if (gb) gb[c] = from_f32<TW>(s1 + (accum ? to_f32(gb[c]) : 0.f));
  }
}

template <typename F>
static void slab_ch_dispatch(int S, F&& f) {
  switch (slab_ch(S)) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 16: f(std::integral_constant<int, 16>{}); break;
    default: f(std::integral_constant<int, 32>{}); break;
  }
}

template <typename F>
void vec_dispatch(bool vec, F&& f) {
  if (vec) f(std::true_type{});
  else f(std::false_type{});
}

}  // namespace

void bn_set_tuning(int red_rpt, int red_cap, int red_min, int elem_rpt, int elem_cap,
                   int elem_min) {
  BNTuning& t = bn_tuning();
  if (red_rpt > 0) t.red_rpt = red_rpt;
  if (red_cap > 0) t.red_cap = red_cap;
  if (red_min >= 0) t.red_min = red_min;
  if (elem_rpt > 0) {
    t.elem_rpt = elem_rpt;
    t.elem_auto = false;
  } else if (elem_rpt == 0) {
    t.elem_auto = true;  // back to the per-shape rule
  }
  if (elem_cap > 0) t.elem_cap = elem_cap;
  if (elem_min >= 0) t.elem_min = elem_min;
}

void bn_get_tuning(int* o) {
  const BNTuning& t = bn_tuning();
  o[0] = t.red_rpt; o[1] = t.red_cap; o[2] = t.red_min;
  o[3] = t.elem_rpt; o[4] = t.elem_cap; o[5] = t.elem_min;
}

int64_t nhwc_splits(int64_t M, int64_t C, bool vec) { return reduce_splits(M, ngeom(C, vec)); }

void bn_stats_from_slab(const float* slab, int S, int64_t C, int64_t count, const float* shift,
                        const BNStatsOut& out, hipStream_t st) {
  slab_ch_dispatch(S, [&](auto ch) {
    constexpr int CH = decltype(ch)::value;
    hipLaunchKernelGGL((slab_stats_k<CH>), dim3((unsigned)((C + CH - 1) / CH)), dim3(kBNThreads),
                       0, st, slab, S, (int)C, count, shift, out);
  });
}

void bn_slab_train_stats(const float* slab, int S, int64_t C, int64_t count, const float* shift,
                         float* mean, float* invstd, float* running_mean, float* running_var,
                         long long* nbt, float eps, float momentum, hipStream_t st) {
  BNStatsOut o{};
  o.mean = mean;
  o.var = nullptr;
  o.invstd = invstd;
  o.running_mean = running_mean;
  o.running_var = running_var;
  o.nbt = nbt;
  o.eps = eps;
  o.momentum = momentum;
  bn_stats_from_slab(slab, S, C, count, shift, o, st);
}

void bn_slab_packed_stats(const float* slab, int S, int64_t C, int64_t count, const float* shift,
                          float* packed, hipStream_t st) {
  BNStatsOut o{};
  o.mean = packed;
  o.var = packed + C;
  o.invstd = nullptr;
  o.count_out = packed + 2 * C;
  o.count_val = (float)count;
  bn_stats_from_slab(slab, S, C, count, shift, o, st);
}

// BN backward sums from a data-gradient conv's epilogue (conv_nhwc_fwd_bnbwd): the slab
// [2][C][S] holds per-M-tile (sum g, sum g*(x-mean)) channel-major
void bn_slab_reduce_grad(const float* slab, int S, int64_t C, const float* invstd,
                         float* sum_dy, float* sum_dy_xmu, void* gw, void* gb, DType tw,
                         hipStream_t st, const float* sum_scale) {
  bn_dispatch(tw, [&](auto w0) {
    using TW = decltype(w0);
    slab_ch_dispatch(S, [&](auto ch) {
      constexpr int CH = decltype(ch)::value;
      hipLaunchKernelGGL((slab_reduce_k<TW, CH>), dim3((unsigned)((C + CH - 1) / CH)),
                         dim3(kBNThreads), 0, st, slab, S, (int)C, invstd, sum_dy, sum_dy_xmu,
                         static_cast<TW*>(gw), static_cast<TW*>(gb), sum_scale,
                         bn_grad_accumulate() ? 1 : 0);
    });
  });
}

void nhwc_stats(const void* x, DType tx, int64_t M, int64_t C, const BNStatsOut& out, float* ws,
                hipStream_t st) {
  const bool vec = (C % 8 == 0) && all_aligned({x});
  const NGeom g = ngeom(C, vec);
  const int splits = reduce_splits(M, g);
  bn_dispatch(tx, [&](auto t0) {
    using T = decltype(t0);
    const T* xp = static_cast<const T*>(x);
    vec_dispatch(vec, [&](auto V) {
      constexpr bool VV = decltype(V)::value;
      hipLaunchKernelGGL((stats_k<T, VV, 4>), dim3(splits, g.cblocks), dim3(kBNThreads), 0, st,
                         xp, M, (int)C, g.ctile, g.rows_iter, ws);
    });
    launch_stats_finalize<T>(xp, ws, splits, C, M, (int64_t)1, out, st);
  });
}

void nhwc_apply(const void* x, DType tx, const float* mean, const float* invstd, const void* w,
                const void* b, DType tw, const void* z, uint8_t* rmask, void* y, int64_t M,
                int64_t C, int relu, hipStream_t st) {
  const bool vec = (C % 8 == 0) && all_aligned({x, z, y});
  const NGeom g = ngeom(C, vec);
  const int blocks = elem_blocks(M, g, M * C * (tx == DType::F32 ? 4 : 2));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      vec_dispatch(vec, [&](auto V) {
        auto go = [&](auto u) {
          auto launch = [&](auto zz) {
            hipLaunchKernelGGL(
                (apply_k<T, TW, decltype(V)::value, decltype(u)::value, decltype(zz)::value>),
                dim3(blocks, g.cblocks), dim3(kBNThreads), 0, st, static_cast<const T*>(x), mean,
                invstd, static_cast<const TW*>(w), static_cast<const TW*>(b),
                static_cast<const T*>(z), static_cast<T*>(y), vec ? rmask : nullptr, M, (int)C,
                g.ctile, g.rows_iter, relu);
          };
          if (z) launch(std::true_type{});
          else launch(std::false_type{});
        };
        go(std::integral_constant<int, 2>{});
      });
    });
  });
}

void nhwc_reduce(const void* dy, const void* x, DType tx, const float* mean, const float* invstd,
                 const void* w, const void* b, DType tw, int relu, const void* z,
                 const uint8_t* rmask, int64_t M, int64_t C, float* sum_dy, float* sum_dy_xmu,
                 void* gw, void* gb, float* ws, hipStream_t st, const float* sum_scale) {
  const bool vec = (C % 8 == 0) && all_aligned({dy, x, z});
  const NGeom g = ngeom(C, vec);
  const int splits = reduce_splits(M, g);
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      vec_dispatch(vec, [&](auto V) {
        constexpr bool VV = decltype(V)::value;
        const int rm = !relu ? 0 : rmask ? 1 : z ? 2 : 3;
        auto go = [&](auto u) {
          auto launch = [&](auto m) {
            hipLaunchKernelGGL((reduce_k<T, TW, VV, decltype(u)::value, decltype(m)::value>),
                               dim3(splits, g.cblocks), dim3(kBNThreads), 0, st,
                               static_cast<const T*>(dy), static_cast<const T*>(x), mean, invstd,
                               static_cast<const TW*>(w), static_cast<const TW*>(b),
                               static_cast<const T*>(z), rmask, M, (int)C, g.ctile, g.rows_iter,
                               ws);
          };
          if (rm == 0) launch(std::integral_constant<int, 0>{});
          else if (rm == 1) launch(std::integral_constant<int, 1>{});
          else if (rm == 2) launch(std::integral_constant<int, 2>{});
          else launch(std::integral_constant<int, 3>{});
        };
        go(std::integral_constant<int, 2>{});
      });
      launch_reduce_finalize<TW>(ws, splits, C, invstd, sum_dy, sum_dy_xmu, static_cast<TW*>(gw),
                         static_cast<TW*>(gb), st, sum_scale);
    });
  });
}

void nhwc_backward(const void* dy, const void* x, DType tx, const float* mean,
                   const float* invstd, const void* w, const void* b, DType tw,
                   const float* sum_dy, const float* sum_dy_xmu, float inv_count, int relu,
                   const void* z, const uint8_t* rmask, void* dx, void* dz, int64_t M, int64_t C,
                   hipStream_t st) {
  const bool vec = (C % 8 == 0) && all_aligned({dy, x, z, dx, dz});
  const NGeom g = ngeom(C, vec);
  const int blocks = elem_blocks(M, g, M * C * (tx == DType::F32 ? 4 : 2));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      vec_dispatch(vec, [&](auto V) {
        const int rm = !relu ? 0 : rmask ? 1 : z ? 2 : 3;
        auto go = [&](auto u) {
          auto launch = [&](auto m) {
            hipLaunchKernelGGL(
                (backward_k<T, TW, decltype(V)::value, decltype(u)::value, decltype(m)::value>),
                dim3(blocks, g.cblocks), dim3(kBNThreads), 0, st, static_cast<const T*>(dy),
                static_cast<const T*>(x), mean, invstd, static_cast<const TW*>(w),
                static_cast<const TW*>(b), sum_dy, sum_dy_xmu, inv_count,
                static_cast<const T*>(z), rmask, static_cast<T*>(dx), static_cast<T*>(dz), M,
                (int)C, g.ctile, g.rows_iter);
          };
          if (rm == 0) launch(std::integral_constant<int, 0>{});
          else if (rm == 1) launch(std::integral_constant<int, 1>{});
          else if (rm == 2) launch(std::integral_constant<int, 2>{});
          else launch(std::integral_constant<int, 3>{});
        };
        go(std::integral_constant<int, 2>{});
      });
    });
  });
}

// relu(BN(x) + BNz(xz)) with the ReLU bitmask: apply_k's ZA mode (both BNs' affines on load)
void nhwc_apply2(const void* x, DType tx, const float* mean, const float* invstd, const void* w,
                 const void* b, DType tw, const void* xz, const float* meanz,
                 const float* invstdz, const void* wz, const void* bz, uint8_t* rmask, void* y,
                 int64_t M, int64_t C, hipStream_t st) {
  const NGeom g = ngeom(C, true);
  const int blocks = elem_blocks(M, g, M * C * (tx == DType::F32 ? 4 : 2));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      hipLaunchKernelGGL((apply_k<T, TW, true, 2, true, true>), dim3(blocks, g.cblocks),
                         dim3(kBNThreads), 0, st, static_cast<const T*>(x), mean, invstd,
                         static_cast<const TW*>(w), static_cast<const TW*>(b),
                         static_cast<const T*>(xz), static_cast<T*>(y), rmask, M, (int)C,
                         g.ctile, g.rows_iter, 1, meanz, invstdz, static_cast<const TW*>(wz),
                         static_cast<const TW*>(bz));
    });
  });
}

// nhwc_backward (no ReLU, no z, no mask: the consumer-epilogue path, where dy is already the
// masked gradient) plus the backward sums and finalize of a second BN over the same rows
// whose gradient is the same dy: x2 its input, mean2 / invstd2 / w2 its statistics and
// weight -> sum_dy2, sum_dy_xmu2 (and gw2, gb2 in tw when non-null)
void nhwc_backward_x2(const void* dy, const void* x, DType tx, const float* mean,
                      const float* invstd, const void* w, const void* b, DType tw,
                      const float* sum_dy, const float* sum_dy_xmu, float inv_count, void* dx,
                      int64_t M, int64_t C, const void* x2, const float* mean2,
                      const float* invstd2, float* sum_dy2, float* sum_dy_xmu2, void* gw2,
                      void* gb2, float* ws, hipStream_t st) {
  const NGeom g = ngeom(C, true);
  const int blocks = elem_blocks(M, g, M * C * (tx == DType::F32 ? 4 : 2));
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      hipLaunchKernelGGL((backward_k<T, TW, true, 2, 0, true>), dim3(blocks, g.cblocks),
                         dim3(kBNThreads), 0, st, static_cast<const T*>(dy),
                         static_cast<const T*>(x), mean, invstd, static_cast<const TW*>(w),
                         static_cast<const TW*>(b), sum_dy, sum_dy_xmu, inv_count,
                         static_cast<const T*>(nullptr), static_cast<const uint8_t*>(nullptr),
                         static_cast<T*>(dx), static_cast<T*>(nullptr), M, (int)C, g.ctile,
                         g.rows_iter, static_cast<const T*>(x2), mean2, ws);
    });
  });
  bn_slab_reduce_grad(ws, blocks, C, invstd2, sum_dy2, sum_dy_xmu2, gw2, gb2, tw, st);
}

int64_t nhwc_backward_x2_workspace(int64_t M, int64_t C, DType tx) {
  const NGeom g = ngeom(C, true);
  return (int64_t)elem_blocks(M, g, M * C * (tx == DType::F32 ? 4 : 2)) * 2 * C;
}

}  // namespace amd
