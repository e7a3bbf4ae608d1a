// One-launch BatchNorm for activations that fit in the register file of the
// chip (channels-last bf16, local statistics): the forward's stats -> finalize ->
// apply and the backward's reduce -> finalize -> elementwise each become ONE
// persistent launch with a grid-wide barrier in the middle.
//
// Why (MI355X): the 14x14 / 7x7 / 28x28-narrow BatchNorms of ResNet-50 move
// 13-51 MB per tensor, so a separate stats pass, finalize launch and apply pass
// are dominated by per-launch ramp + drain and by re-reading the tensor
// (profiles/microbench_mb_bn.txt: 1.0-3.2 TB/s on those layers).  Here every
// lane loads its R rows x 8 channels (one 16-byte load each) into registers
// ONCE, reduces them, and after the barrier applies the affine (+ residual)
// (+ ReLU) from the same registers: the tensor is read once and written once.
// The backward keeps the masked dy' (and x, when it fits) in registers across
// the barrier the same way.
//
// Cross-workgroup reduction: each workgroup sums its rows in LDS (fixed order)
// and adds its per-channel partial to a device-resident [2][C] fp32 accumulator
// with no-return float atomics (two contiguous 256-byte atomic wave-instructions
// per 64 channels); results may differ from the split-slab kernels in the last
// bits (summation order), not beyond.  The barrier (MI355X_MICROARCH.md
// visibility recipe): every wave drains, workgroup barrier, one lane releases
// (agent) and arrives on a counter; the last arriver zeroes the OTHER parity's
// accumulator for the next launch, resets the counter and bumps a generation
// word; the others poll the generation relaxed with s_sleep, then acquire.  The
// state (count, generation, two accumulator parities) lives in a per-device
// block initialised once; launches alternate parity by generation, so no memset
// per call and the launch is hipGraph-capturable.  The spin is bounded: a
// barrier that does not complete within ~1 s sets an error word
// (bn_persist_error) instead of hanging the GPU.
//
// Residency: the grid is at most CUs x (occupancy - 1) workgroups (one below the
// occupancy API's answer, which can over-admit by one: MI355X_MICROARCH.md
// "Residency and cooperative launch"), so every workgroup is resident before
// any waits; shapes that do not fit run the split kernels (bn_nhwc.hip).
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "bn_common.h"

namespace amd {

namespace {

constexpr int kPMaxC = 2048;
constexpr int kFZ = 1, kFMask = 2, kFRelu = 4;             // forward variants
constexpr int kBRelu = 1, kBMask = 2, kBZ = 4, kBDz = 8;   // backward variants
constexpr unsigned kSpinLimit = 1u << 22;

struct PState {
  unsigned count, gen, err, pad;
  float acc[2][2][kPMaxC];  // [parity][sum | sum of squares / sum dy'(x-mu)][C]
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ldf_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Combine the rows_iter row groups of the workgroup (same channel set per lane)
// through LDS, then add the workgroup's partial to acc[par][0|1][c] with one
// thread per channel (contiguous atomics).
__device__ __forceinline__ void block_partial_atomic(const float (&s1)[8], const float (&s2)[8],
                                                     int ci, int ri, int ctile, int rows_iter,
                                                     int cbase, int C, float* acc0, float* acc1) {
  __shared__ float red[2][kBNThreads * 8];
  if (ri < rows_iter) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[0][(ri * ctile + ci) * 8 + i] = s1[i];
      red[1][(ri * ctile + ci) * 8 + i] = s2[i];
    }
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < ctile * 8; cc += kBNThreads) {
    const int c = cbase + cc;
    if (c >= C) continue;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rows_iter; ++r) {
      a += red[0][r * ctile * 8 + cc];
      b += red[1][r * ctile * 8 + cc];
    }
    atomicAdd(acc0 + c, a);
    atomicAdd(acc1 + c, b);
  }
}

// Grid-wide barrier over all gridDim.x * gridDim.y workgroups (see header).
// g0 = generation read by thread 0 before this workgroup's first atomic.
// Fences: the hand-off data are memory-side float atomics read back with sc1 loads
// ({agent atomics both sides}: MI355X_MICROARCH.md valid forms), so the release /
// acquire fences guard only the L1/L2 state no one reads; fences = 0 drops them (APEX_AMD_BN_PERSIST=2, A/B).
__device__ __forceinline__ void grid_barrier(PState* ps, unsigned g0, int par, int fences) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (fences) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned G = gridDim.x * gridDim.y;
    const unsigned t = __hip_atomic_fetch_add(&ps->count, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == G - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (s_last) {
    // every other workgroup has arrived: clear the other parity for the next launch
    float* other = &ps->acc[par ^ 1][0][0];
    for (int i = threadIdx.x; i < 2 * kPMaxC; i += kBNThreads)
      __hip_atomic_store(other + i, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(&ps->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&ps->gen, g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fences) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  } else if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (ld_agent(&ps->gen) == g0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > kSpinLimit) {
        __hip_atomic_store(&ps->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (fences) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- buffer IO
// All tensor accesses go through buffer descriptors with a 32-bit byte offset per
// row (one VGPR, recomputed per row from a scalar stride) instead of a 64-bit
// address per row kept live across the barrier; an out-of-range offset (rows past
// M, idle lanes) loads 0 and drops the store.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
__device__ __forceinline__ void unpack8(const u32x4& u, float (&v)[8]) {
  const bf16x8 a = __builtin_bit_cast(bf16x8, u);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
}
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  bf16x8 a;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (bf16_t)v[i];
  return __builtin_bit_cast(u32x4, a);
}
__device__ __forceinline__ void opaque(u32x4& u) {
  asm volatile("" : "+v"(u));
}

// ---------------------------------------------------------------- forward
// y = relu?(x*sc + sh (+ z)), sc = invstd*w, sh = b - mean*sc; statistics of x
// over the M rows (shifted by row 0 of x, as stats_k); running stats, mean,
// invstd and num_batches_tracked written by the workgroups of row block 0.
// F: kFZ = residual z, kFMask = write the ReLU bitmask, kFRelu = apply ReLU
template <typename TW, int R, int F>
__global__ void __launch_bounds__(kBNThreads)
    bnp_fwd_k(const bf16_t* __restrict__ x, const TW* __restrict__ w, const TW* __restrict__ b,
              const bf16_t* __restrict__ z, bf16_t* __restrict__ y, uint8_t* __restrict__ rmask,
              BNStatsOut out, int64_t M, int C, int ctile, int rows_iter, PState* ps, int fences) {
  __shared__ unsigned s_gen;
  const int ci = threadIdx.x % ctile, ri = threadIdx.x / ctile;
  const int cbase = blockIdx.y * ctile * 8;
  const int c0 = cbase + ci * 8;
  const bool active = ri < rows_iter && c0 < C;
  const int64_t rbase = (int64_t)blockIdx.x * R * rows_iter + ri;
  if (threadIdx.x == 0) s_gen = ld_agent(&ps->gen);
  const int64_t bytes = M * C * 2;
  const auto xr = rsrc(x, bytes), yr = rsrc(y, bytes);
  // byte offset of row rbase + r*rows_iter = off0 + r*rstep
  const unsigned off0 = active ? (unsigned)((rbase * C + c0) * 2) : kOOB;
  const unsigned rstep = (unsigned)(rows_iter * C * 2);
  const int64_t nvalid = active && rbase < M ? (M - rbase + rows_iter - 1) / rows_iter : 0;

  u32x4 ks = bload(xr, active ? (unsigned)(c0 * 2) : kOOB);  // shift = row 0
  u32x4 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = bload(xr, off0 + r * rstep);
  float k[8], s1[8], s2[8];
  unpack8(ks, k);
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s2[i] = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float f[8];
    unpack8(v[r], f);
    const float vm = r < nvalid ? 1.f : 0.f;  // rows past M (loaded as 0) -> d = 0
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = (f[i] - k[i]) * vm;
      s1[i] += d;
      s2[i] = fmaf(d, d, s2[i]);
    }
    __builtin_amdgcn_sched_barrier(0);  // one row's floats live at a time
  }
  __syncthreads();  // s_gen visible
  const unsigned g0 = s_gen;
  const int par = (int)(g0 & 1u);
  block_partial_atomic(s1, s2, ci, ri, ctile, rows_iter, cbase, C, ps->acc[par][0],
                       ps->acc[par][1]);
  grid_barrier(ps, g0, par, fences);
  if (!active) return;
#pragma unroll
  for (int r = 0; r < R; ++r) opaque(v[r]);

  float sc[8], sh[8];
  const double inv_n = 1.0 / (double)M;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = c0 + i;
    const double m = (double)ldf_agent(&ps->acc[par][0][c]) * inv_n;
    double var = (double)ldf_agent(&ps->acc[par][1][c]) * inv_n - m * m;
    if (var < 0.0) var = 0.0;
    const float mean = (float)(k[i] + m);
    const float is = rsqrtf((float)var + out.eps);
    sc[i] = is * wload(w, c, 1.f);
    sh[i] = wload(b, c, 0.f) - mean * sc[i];
    if (blockIdx.x == 0 && ri == 0) {
      out.mean[c] = mean;
      out.invstd[c] = is;
      if (out.running_mean) {
        const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
        out.running_mean[c] = (1.f - out.momentum) * out.running_mean[c] + out.momentum * mean;
        out.running_var[c] = (1.f - out.momentum) * out.running_var[c] + out.momentum * (float)unb;
      }
      if (out.nbt && c == 0) *out.nbt += 1;
    }
  }
  const auto zr = rsrc(z, z ? bytes : 0);
  const auto mr = rsrc(rmask, rmask ? bytes / 16 : 0);
  const int Cb = C >> 3;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const unsigned off = off0 + r * rstep;
    float f[8], zz[8];
    unpack8(v[r], f);
    if constexpr ((F & kFZ) != 0) unpack8(bload(zr, off), zz);
    uint32_t mb = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float o = fmaf(f[i], sc[i], sh[i]);
      if constexpr ((F & kFZ) != 0) o += zz[i];
      mb |= (o > 0.f ? 1u : 0u) << i;
      f[i] = (F & kFRelu) ? fmaxf(o, 0.f) : o;
    }
    bstore(yr, off, pack8(f));
    if ((F & kFMask) && r < nvalid)
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)mb, mr,
                                           (unsigned)((rbase + (int64_t)r * rows_iter) * Cb + (c0 >> 3)),
                                           0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------- backward
// dy' = dy masked by the forward's ReLU condition (mask bits, or recomputed from
// x (+ z)); s1 = sum dy', s2 = sum dy'(x - mean); then
// dx = dy'*k1 + x*k2 + k3 (backward_k's constants), dz = dy'; gw = s2*invstd,
// gb = s1 (workgroups of row block 0).  HOLDX keeps x in registers across the
// barrier, else phase 2 re-reads it.
// F: kBRelu = ReLU fused, kBMask = its condition from the bitmask (else recomputed
// from x, + z with kBZ), kBDz = write dz
template <typename TW, int R, bool HOLDX, int F>
__global__ void __launch_bounds__(kBNThreads)
    bnp_bwd_k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
              const float* __restrict__ mean, const float* __restrict__ invstd,
              const TW* __restrict__ w, const TW* __restrict__ b, const bf16_t* __restrict__ z,
              const uint8_t* __restrict__ rmask, bf16_t* __restrict__ dx,
              bf16_t* __restrict__ dz, TW* __restrict__ gw, TW* __restrict__ gb, int64_t M,
              int C, int ctile, int rows_iter, PState* ps, int fences) {
  __shared__ unsigned s_gen;
  const int ci = threadIdx.x % ctile, ri = threadIdx.x / ctile;
  const int cbase = blockIdx.y * ctile * 8;
  const int c0 = cbase + ci * 8;
  const bool active = ri < rows_iter && c0 < C;
  const int64_t rbase = (int64_t)blockIdx.x * R * rows_iter + ri;
  const int Cb = C >> 3;
  if (threadIdx.x == 0) s_gen = ld_agent(&ps->gen);
  const int64_t bytes = M * C * 2;
  const auto dyr = rsrc(dy, bytes), xr = rsrc(x, bytes);
  const auto mr = rsrc(rmask, rmask ? bytes / 16 : 0), zr = rsrc(z, z ? bytes : 0);
  const unsigned off0 = active ? (unsigned)((rbase * C + c0) * 2) : kOOB;
  const unsigned rstep = (unsigned)(rows_iter * C * 2);
  const unsigned moff0 = active ? (unsigned)(rbase * Cb + (c0 >> 3)) : kOOB;
  const unsigned mstep = (unsigned)(rows_iter * Cb);

  float mu[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mu[i] = sc[i] = sh[i] = s1[i] = s2[i] = 0.f;
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mu[i] = mean[c0 + i];
      chan_affine(mean, invstd, wload(w, c0 + i, 1.f), wload(b, c0 + i, 0.f), c0 + i, sc[i],
                  sh[i]);
    }
  }
  u32x4 dv[R];
  u32x4 xv[HOLDX ? R : 1];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const unsigned off = off0 + r * rstep;
    u32x4 du = bload(dyr, off);  // rows past M: dy = 0 -> no contribution
    const u32x4 xu = bload(xr, off);
    float d[8], xf[8];
    unpack8(du, d);
    unpack8(xu, xf);
    if constexpr ((F & kBRelu) != 0) {
      if constexpr ((F & kBMask) != 0) {
        const uint32_t mk = __builtin_amdgcn_raw_buffer_load_b8(mr, moff0 + r * mstep, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = ((mk >> i) & 1u) ? d[i] : 0.f;
      } else {
        float zz[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) zz[i] = 0.f;
        if constexpr ((F & kBZ) != 0) unpack8(bload(zr, off), zz);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float o = fmaf(xf[i], sc[i], sh[i]) + zz[i];
          d[i] = o > 0.f ? d[i] : 0.f;
        }
      }
      du = pack8(d);  // exact: each element is dy or 0
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s1[i] += d[i];
      s2[i] = fmaf(d[i], xf[i] - mu[i], s2[i]);
    }
    dv[r] = du;
    if constexpr (HOLDX) xv[r] = xu;
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  const unsigned g0 = s_gen;
  const int par = (int)(g0 & 1u);
  block_partial_atomic(s1, s2, ci, ri, ctile, rows_iter, cbase, C, ps->acc[par][0],
                       ps->acc[par][1]);
  grid_barrier(ps, g0, par, fences);
  if (!active) return;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    opaque(dv[r]);
    if constexpr (HOLDX) opaque(xv[r]);
  }

  float k1[8], k2[8], k3[8];
  const float inv_n = 1.f / (float)M;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = c0 + i;
    const float t1 = ldf_agent(&ps->acc[par][0][c]), t2 = ldf_agent(&ps->acc[par][1][c]);
    const float is = invstd[c], wc = wload(w, c, 1.f);
    k1[i] = is * wc;
    k2[i] = -is * is * is * wc * (t2 * inv_n);
    k3[i] = -is * wc * (t1 * inv_n) - k2[i] * mu[i];
    if (blockIdx.x == 0 && ri == 0 && gw) {
      gw[c] = from_f32<TW>(t2 * is);
      gb[c] = from_f32<TW>(t1);
    }
  }
  const auto dxr = rsrc(dx, bytes), dzr = rsrc(dz, dz ? bytes : 0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const unsigned off = off0 + r * rstep;
    float d[8], xf[8];
    unpack8(dv[r], d);
    if constexpr (HOLDX) unpack8(xv[r], xf);
    else unpack8(bload(xr, off), xf);
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = fmaf(d[i], k1[i], fmaf(xf[i], k2[i], k3[i]));
    bstore(dxr, off, pack8(xf));
    if constexpr ((F & kBDz) != 0) bstore(dzr, off, dv[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------- host side
struct DevState {
  PState* ps = nullptr;
  int cus = 0;
};

std::mutex g_mu;
std::unordered_map<int, DevState> g_state;

DevState& dev_state() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mu);
  DevState& s = g_state[dev];
  if (!s.ps) {
    if (hipMalloc(&s.ps, sizeof(PState)) != hipSuccess) {
      s.ps = nullptr;
      return s;
    }
    (void)hipMemset(s.ps, 0, sizeof(PState));
    (void)hipDeviceSynchronize();
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, dev);
    s.cus = p.multiProcessorCount;
  }
  return s;
}

// resident workgroups for a kernel: CUs x (occupancy answer - 1, at most 7)
template <typename K>
int64_t resident_cap(K kernel, int cus) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> occ;
  int n = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = occ.find((const void*)kernel);
    if (it != occ.end()) {
      n = it->second;
    } else {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, kBNThreads, 0) != hipSuccess)
        n = 0;
      occ[(const void*)kernel] = n;
    }
  }
  // admitted per CU = min(API, 8, 800 / (SGPR alloc + 16)): these kernels use <= 112
  // SGPRs, so 6 is always admitted; the spin bound covers a miscount
  if (n > 6) n = 6;
  return n < 1 ? 0 : (int64_t)n * cus;
}

// OFF by default (measured slower, profiles/microbench_bn_persist.txt): the forward
// took 64-85 us vs 31 us for the split kernels at (256, 256, 14, 14) - the grid
// barrier (784 workgroups arriving on one counter and polling one word) and the
// finalize in every workgroup cost more than the saved re-read; only the masked
// backward without fences won (47 vs 56 us), on shapes ResNet-50 does not use.
// APEX_AMD_BN_PERSIST=1 (2 = barrier without fences) enables it for A/B runs;
// bn_persist_enable overrides it at run time (tests).
int& persist_flag() {
  static int m = [] {
    const char* e = std::getenv("APEX_AMD_BN_PERSIST");
    return e ? std::atoi(e) : 0;
  }();
  return m;
}
int persist_mode() { return persist_flag(); }
long long g_launches = 0;  // persistent launches issued (tests check the path ran)

struct PGeom {
  int ctile, rows_iter, cblocks;
};
PGeom pgeom(int64_t C) {
  PGeom g;
  const int cv = (int)(C / 8);
  g.ctile = cv < 64 ? cv : 64;
  g.rows_iter = kBNThreads / g.ctile;
  g.cblocks = (cv + g.ctile - 1) / g.ctile;
  return g;
}

bool shape_ok(int64_t M, int64_t C) {
  return persist_mode() != 0 && C % 8 == 0 && C >= 8 && C <= kPMaxC && M >= 2 &&
         M * C <= ((int64_t)1 << 29);
}

}  // namespace

template <int N, typename F>
void static_for(F&& f) {
  if constexpr (N > 0) {
    static_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}

bool bn_persist_forward(const void* x, const void* w, const void* b, DType tw, const void* z,
                        void* y, uint8_t* rmask, float* mean, float* invstd, float* running_mean,
                        float* running_var, long long* nbt, float eps, float momentum, int64_t M,
                        int64_t C, int relu, hipStream_t st) {
  // BatchNorm parameters stay fp32 under amp O2 (the only variant instantiated)
  if (tw != DType::F32 || !shape_ok(M, C) || !all_aligned({x, z, y})) return false;
  DevState& s = dev_state();
  if (!s.ps) return false;
  const BNStatsOut out{mean, nullptr, invstd, running_mean, running_var, nbt, eps, momentum};
  const PGeom g = pgeom(C);
  const int flags = (z ? kFZ : 0) | (rmask ? kFMask : 0) | (relu ? kFRelu : 0);
  bool launched = false;
  auto go = [&](auto rc, auto fc) -> bool {
    constexpr int R = decltype(rc)::value, F = decltype(fc)::value;
    auto kern = bnp_fwd_k<float, R, F>;
    const int64_t gx = (M + (int64_t)R * g.rows_iter - 1) / ((int64_t)R * g.rows_iter);
    if (gx * g.cblocks > resident_cap(kern, s.cus)) return false;
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, g.cblocks), dim3(kBNThreads), 0, st,
                       static_cast<const bf16_t*>(x), static_cast<const float*>(w),
                       static_cast<const float*>(b), static_cast<const bf16_t*>(z),
                       static_cast<bf16_t*>(y), rmask, out, M, (int)C, g.ctile, g.rows_iter, s.ps,
                       persist_mode() == 2 ? 0 : 1);
    ++g_launches;
    return true;
  };
  static_for<8>([&](auto fc) {
    if (launched || decltype(fc)::value != flags) return;
    launched = go(std::integral_constant<int, 8>{}, fc) || go(std::integral_constant<int, 16>{}, fc);
  });
  return launched;
}

bool bn_persist_backward(const void* dy, const void* x, const float* mean, const float* invstd,
                         const void* w, const void* b, DType tw, int relu, const void* z,
                         const uint8_t* rmask, void* dx, void* dz, void* gw, void* gb, int64_t M,
                         int64_t C, hipStream_t st) {
  if (tw != DType::F32 || !shape_ok(M, C) || !all_aligned({dy, x, z, dx, dz})) return false;
  DevState& s = dev_state();
  if (!s.ps) return false;
  const PGeom g = pgeom(C);
  int flags = dz ? kBDz : 0;
  if (relu) flags |= kBRelu | (rmask ? kBMask : (z ? kBZ : 0));
  bool launched = false;
  auto go = [&](auto rc, auto hx, auto fc) -> bool {
    constexpr int R = decltype(rc)::value, F = decltype(fc)::value;
    constexpr bool HX = decltype(hx)::value;
    auto kern = bnp_bwd_k<float, R, HX, F>;
    const int64_t gx = (M + (int64_t)R * g.rows_iter - 1) / ((int64_t)R * g.rows_iter);
    if (gx * g.cblocks > resident_cap(kern, s.cus)) return false;
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, g.cblocks), dim3(kBNThreads), 0, st,
                       static_cast<const bf16_t*>(dy), static_cast<const bf16_t*>(x), mean, invstd,
                       static_cast<const float*>(w), static_cast<const float*>(b),
                       static_cast<const bf16_t*>(z), rmask, static_cast<bf16_t*>(dx),
                       static_cast<bf16_t*>(dz), static_cast<float*>(gw), static_cast<float*>(gb),
                       M, (int)C, g.ctile, g.rows_iter, s.ps,
                       persist_mode() == 2 ? 0 : 1);
    ++g_launches;
    return true;
  };
  static_for<16>([&](auto fc) {
    constexpr int F = decltype(fc)::value;
    // valid combinations only: mask / z imply ReLU, never both
    if constexpr (((F & (kBMask | kBZ)) != 0 && (F & kBRelu) == 0) ||
                  ((F & kBMask) != 0 && (F & kBZ) != 0)) {
      return;
    } else {
      if (launched || F != flags) return;
      launched = go(std::integral_constant<int, 8>{}, std::true_type{}, fc) ||
                 go(std::integral_constant<int, 16>{}, std::false_type{}, fc);
    }
  });
  return launched;
}

// error word of the barrier (1 = a barrier timed out since the last reset) and a
// reset of the whole state (tests)
int bn_persist_error() {
  DevState& s = dev_state();
  if (!s.ps) return -1;
  unsigned e = 0;
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(&e, &s.ps->err, sizeof(e), hipMemcpyDeviceToHost);
  return (int)e;
}

void bn_persist_enable(int mode) { persist_flag() = mode; }
int bn_persist_mode() { return persist_flag(); }
long long bn_persist_launches() { return g_launches; }

void bn_persist_reset() {
  DevState& s = dev_state();
  if (!s.ps) return;
  (void)hipDeviceSynchronize();
  (void)hipMemset(s.ps, 0, sizeof(PState));
  (void)hipDeviceSynchronize();
}

}  // namespace amd
