// Multi-tensor elementwise kernels: scale (+overflow check), axpby, check-finite,
// zero-fill, and the l2/max norm partial + finalize reductions.
//
// Behavioural spec: apex@f3a960f8 csrc/multi_tensor_scale_kernel.cu,
// multi_tensor_axpby_kernel.cu, multi_tensor_l2norm_kernel.cu (amp_C N-05..N-07
// in SURVEY.md).  Implementation is MI355X-native: device-resident launch table
// (mt_table.h), one workgroup per 8192-element tile, 16-byte lane accesses,
// deterministic two-pass reductions (no float atomics).
#include "amd_dev.h"
#include "amd_kernels.h"
#include "mt_table.h"
#include "mt_device.h"

namespace amd {

// --------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void __launch_bounds__(kMTThreads) scale_kernel(MTLaunch L, ScaleArg s, int* noop) {
  TileCtx c = tile_ctx(L);
  const float sc = get_scale(s);
  const bool al = c.t->aligned;
  float v[kMTUnroll][8];
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    ld<TI>(c.t->ptr[0], c.start + off, cnt, al && cnt >= 8, v[u]);
  }
  bool finite = true;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      finite &= finite_f32(v[u][i]);
      v[u][i] *= sc;
    }
    st<TO>(c.t->ptr[1], c.start + off, cnt, al && cnt >= 8, v[u]);
  }
  if (noop && !finite) *noop = 1;
}

template <typename TI>
__global__ void __launch_bounds__(kMTThreads) check_finite_kernel(MTLaunch L, int* noop) {
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  bool finite = true;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    float v[8];
    ld<TI>(c.t->ptr[0], c.start + off, cnt, al && cnt >= 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) finite &= finite_f32(v[i]);
  }
  if (noop && !finite) *noop = 1;
}

template <typename TX, typename TY, typename TO>
__global__ void __launch_bounds__(kMTThreads)
    axpby_kernel(MTLaunch L, ScaleArg sa, ScaleArg sb, int arg_to_check, int* noop) {
  TileCtx c = tile_ctx(L);
  const float a = get_scale(sa), b = get_scale(sb);
  const bool al = c.t->aligned;
  bool finite = true;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    bool vec = al && cnt >= 8;
    float x[8], y[8], o[8];
    ld<TX>(c.t->ptr[0], c.start + off, cnt, vec, x);
    ld<TY>(c.t->ptr[1], c.start + off, cnt, vec, y);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (arg_to_check == -1) finite &= finite_f32(x[i]) & finite_f32(y[i]);
      else if (arg_to_check == 0) finite &= finite_f32(x[i]);
      else finite &= finite_f32(y[i]);
      o[i] = a * x[i] + b * y[i];
    }
    st<TO>(c.t->ptr[2], c.start + off, cnt, vec, o);
  }
  if (noop && !finite) *noop = 1;
}

template <typename T>
__global__ void __launch_bounds__(kMTThreads) zero_kernel(MTLaunch L) {
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    st<T>(c.t->ptr[0], c.start + off, cnt, al && cnt >= 8, z);
  }
}

// dst = src only when *flag != 0 (the overflow flag of a skipped step): restores the
// pre-step snapshot of a guarded (non-fused) optimizer without a host round trip
template <typename T>
__global__ void __launch_bounds__(kMTThreads) copy_if_kernel(MTLaunch L, const int* flag) {
  if (*flag == 0) return;
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    if (cnt <= 0) continue;
    float v[8];
    ld<T>(c.t->ptr[0], c.start + off, cnt, al && cnt >= 8, v);
    st<T>(c.t->ptr[1], c.start + off, cnt, al && cnt >= 8, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(kMTThreads)
    norm_partials_kernel(MTLaunch L, int max_norm, float* partials, int* noop) {
  __shared__ float scratch[kMTThreads / kWave];
  TileCtx c = tile_ctx(L);
  const bool al = c.t->aligned;
  float acc = 0.f;
  bool finite = true;
#pragma unroll
  for (int u = 0; u < kMTUnroll; ++u) {
    int off = lane_off(u);
    int cnt = c.n - off;
    float v[8];
    ld<T>(c.t->ptr[0], c.start + off, cnt, al && cnt >= 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      finite &= finite_f32(v[i]);
      if (max_norm) acc = fmaxf(acc, fabsf(v[i]));
      else acc = fmaf(v[i], v[i], acc);
    }
  }
  float r = max_norm ? block_max(acc, scratch) : block_sum(acc, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
  if (noop && !finite) *noop = 1;
}

// One workgroup per (tensor, set) for per-tensor results; an extra workgroup per
// set for the global value.  Sums run over chunks in a fixed order.
__global__ void __launch_bounds__(256)
    norm_finalize_kernel(MTLaunch L, const float* partials, int max_norm, float* out_global,
                         float* out_per_tensor) {
  __shared__ float scratch[4];
  const int set = blockIdx.y;
  const float* part = partials + (int64_t)set * L.nchunks;
  int t = blockIdx.x;
  int begin, end;
  if (t < L.ntensors) {
    const TensorDesc& d = L.tensors[t];
    begin = d.first_chunk;
    end = begin + (int)((d.numel + kTile - 1) / kTile);
  } else {
    begin = 0;
    end = L.nchunks;
  }
  float acc = 0.f;
  for (int i = begin + threadIdx.x; i < end; i += blockDim.x)
    acc = max_norm ? fmaxf(acc, part[i]) : acc + part[i];
  float r = max_norm ? block_max(acc, scratch) : block_sum(acc, scratch);
  if (threadIdx.x == 0) {
    float v = max_norm ? r : sqrtf(r);
    if (t < L.ntensors) {
      if (out_per_tensor) out_per_tensor[(int64_t)set * L.ntensors + t] = v;
    } else if (out_global) {
      out_global[set] = v;
    }
  }
}

// --------------------------------------------------------------------------

void mt_scale(const MTLaunch& L, DType in, DType out, ScaleArg s, int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(in, [&](auto ti) {
    dispatch1(out, [&](auto to) {
      using TI = decltype(ti);
      using TO = decltype(to);
      hipLaunchKernelGGL((scale_kernel<TI, TO>), mt_grid(L), dim3(kMTThreads), 0, st, L, s, noop);
    });
  });
}

void mt_check_finite(const MTLaunch& L, DType in, int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(in, [&](auto ti) {
    using TI = decltype(ti);
    hipLaunchKernelGGL((check_finite_kernel<TI>), mt_grid(L), dim3(kMTThreads), 0, st, L, noop);
  });
}

void mt_axpby(const MTLaunch& L, DType x, DType y, DType out, ScaleArg a, ScaleArg b,
              int arg_to_check, int* noop, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(x, [&](auto tx) {
    dispatch1(y, [&](auto ty) {
      dispatch1(out, [&](auto to) {
        using TX = decltype(tx);
        using TY = decltype(ty);
        using TO = decltype(to);
        hipLaunchKernelGGL((axpby_kernel<TX, TY, TO>), mt_grid(L), dim3(kMTThreads), 0, st, L, a,
                           b, arg_to_check, noop);
      });
    });
  });
}

void mt_fill_zero(const MTLaunch& L, DType t, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(t, [&](auto tt) {
    using T = decltype(tt);
    hipLaunchKernelGGL((zero_kernel<T>), mt_grid(L), dim3(kMTThreads), 0, st, L);
  });
}

void mt_copy_if(const MTLaunch& L, DType t, const int* flag, hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(t, [&](auto tt) {
    using T = decltype(tt);
    hipLaunchKernelGGL((copy_if_kernel<T>), mt_grid(L), dim3(kMTThreads), 0, st, L, flag);
  });
}

void mt_norm_partials(const MTLaunch& L, DType in, int max_norm, float* partials, int* noop,
                      hipStream_t st) {
  if (L.nchunks == 0) return;
  dispatch1(in, [&](auto ti) {
    using T = decltype(ti);
    hipLaunchKernelGGL((norm_partials_kernel<T>), mt_grid(L), dim3(kMTThreads), 0, st, L,
                       max_norm, partials, noop);
  });
}

void mt_norm_finalize(const MTLaunch& L, const float* partials, int npart_sets, int max_norm,
                      float* out_global, float* out_per_tensor, hipStream_t st) {
  if (L.nchunks == 0) return;
  int nx = (out_per_tensor ? L.ntensors : 0) + 1;
  // When per-tensor output is not requested, only the global workgroup runs:
  // index it as tensor == ntensors by offsetting through a shifted launch.
  if (!out_per_tensor) {
    MTLaunch G = L;
    G.ntensors = 0;  // every block takes the global path
    hipLaunchKernelGGL(norm_finalize_kernel, dim3(1, npart_sets), dim3(256), 0, st, G, partials,
                       max_norm, out_global, nullptr);
    return;
  }
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(nx, npart_sets), dim3(256), 0, st, L, partials,
                     max_norm, out_global, out_per_tensor);
}

// --------------------------------------------------------------------------
// flat (single contiguous buffer) scale / cast with finiteness check
template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
    flat_scale_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n, ScaleArg s,
                      int* noop) {
  const float sc = get_scale(s);
  bool finite = true;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < n; i += stride) {
    float v[8];
    int cnt = (n - i) < 8 ? (int)(n - i) : 8;
    if (cnt == 8) load8(in + i, v);
    else load8_tail(in + i, cnt, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      finite &= (k >= cnt) || finite_f32(v[k]);
      v[k] *= sc;
    }
    if (out) {
      if (cnt == 8) store8(out + i, v);
      else store8_tail(out + i, cnt, v);
    }
  }
  if (noop && !finite) *noop = 1;
}

void flat_scale(const void* in, DType tin, void* out, DType tout, int64_t n, ScaleArg s,
                int* noop, hipStream_t st) {
  if (n == 0) return;
  int64_t groups = (n + 7) / 8;
  int64_t blocks = (groups + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  dispatch1(tin, [&](auto ti) {
    dispatch1(tout, [&](auto to) {
      using TI = decltype(ti);
      using TO = decltype(to);
      hipLaunchKernelGGL((flat_scale_kernel<TI, TO>), dim3((unsigned)blocks), dim3(256), 0, st,
                         static_cast<const TI*>(in), static_cast<TO*>(out), n, s, noop);
    });
  });
}

// --------------------------------------------------------------------------
__global__ void update_loss_scale_kernel(float* scale, int* unskipped, int* skipped_total,
                                         const int* overflow, float factor, int window,
                                         float min_scale, float max_scale, int dynamic,
                                         float* applied) {
  if (threadIdx.x != 0) return;
  // the scale this step's gradients carry, for optimizers that unscale in-kernel
  // AFTER this update (the growth step must not unscale by the doubled value)
  if (applied) *applied = *scale;
  if (*overflow) {
    if (dynamic) {
      float s = *scale / factor;
      if (min_scale > 0.f && s < min_scale) s = min_scale;
      *scale = s;
    }
    *unskipped = 0;
    if (skipped_total) *skipped_total += 1;
  } else {
    int u = *unskipped + 1;
    if (dynamic && u == window) {
      float s = *scale * factor;
      if (s > max_scale) s = max_scale;
      *scale = s;
      u = 0;
    }
    *unskipped = u;
  }
}

void update_loss_scale(float* scale, int* unskipped, int* skipped_total, const int* overflow,
                       float factor, int window, float min_scale, float max_scale, int dynamic,
                       hipStream_t st, float* applied) {
  hipLaunchKernelGGL(update_loss_scale_kernel, dim3(1), dim3(64), 0, st, scale, unskipped,
                     skipped_total, overflow, factor, window, min_scale, max_scale, dynamic,
                     applied);
}

__global__ void mark_step_done_kernel(int* flag, const int* noop) {
  if (threadIdx.x == 0 && !(noop && *noop)) *flag = 1;
}
void mark_step_done(int* flag, const int* noop, hipStream_t st) {
  hipLaunchKernelGGL(mark_step_done_kernel, dim3(1), dim3(64), 0, st, flag, noop);
}

__global__ void advance_step_kernel(int* step, const int* noop) {
  if (threadIdx.x == 0 && !(noop && *noop)) *step += 1;
}
void advance_step(int* step, const int* noop, hipStream_t st) {
  hipLaunchKernelGGL(advance_step_kernel, dim3(1), dim3(64), 0, st, step, noop);
}

}  // namespace amd

namespace amd {

// Device memcpy whose SOURCE travels in the kernel arguments: usable while a
// hipGraph is being captured (no host buffer is referenced by the graph, and
// no pinned allocation is needed) - used to upload multi-tensor launch tables
// that are first built during a capture.
struct ArgChunk {
  uint32_t nbytes;
  uint32_t pad;
  uint8_t data[3584];
};

__global__ void __launch_bounds__(256) copy_from_args_kernel(uint8_t* dst, ArgChunk c) {
  for (uint32_t i = threadIdx.x; i < c.nbytes; i += blockDim.x) dst[i] = c.data[i];
}

void upload_by_args(void* dst, const void* src, size_t bytes, hipStream_t st) {
  const uint8_t* s = static_cast<const uint8_t*>(src);
  uint8_t* d = static_cast<uint8_t*>(dst);
  for (size_t off = 0; off < bytes; off += sizeof(ArgChunk::data)) {
    ArgChunk c;
    size_t n = bytes - off < sizeof(c.data) ? bytes - off : sizeof(c.data);
    c.nbytes = (uint32_t)n;
    c.pad = 0;
    for (size_t i = 0; i < n; ++i) c.data[i] = s[off + i];
    hipLaunchKernelGGL(copy_from_args_kernel, dim3(1), dim3(256), 0, st, d + off, c);
  }
}

}  // namespace amd
