// Device helpers for multi-tensor-apply kernels (shared by every mt_*.hip).
#pragma once
#include "amd_dev.h"
#include "amd_kernels.h"
#include "mt_table.h"

namespace amd {

__device__ __forceinline__ float get_scale(const ScaleArg& s) {
  float v = s.ptr ? *s.ptr : s.val;
  return s.invert ? 1.f / v : v;
}

// Element offset (within a tile) handled by lane `tid` in unroll step u.
__device__ __forceinline__ int lane_off(int u) { return (u * kMTThreads + (int)threadIdx.x) * 8; }

template <typename T>
__device__ __forceinline__ void ld(const void* base, int64_t idx, int cnt, bool vec, float (&v)[8]) {
  const T* p = static_cast<const T*>(base) + idx;
  if (vec) load8(p, v);
  else load8_tail(p, cnt, v);
}
template <typename T>
__device__ __forceinline__ void st(void* base, int64_t idx, int cnt, bool vec, const float (&v)[8]) {
  T* p = static_cast<T*>(base) + idx;
  if (vec) store8(p, v);
  else store8_tail(p, cnt, v);
}

struct TileCtx {
  const TensorDesc* t;
  int64_t start;
  int n;
};

__device__ __forceinline__ TileCtx tile_ctx(const MTLaunch& L, int chunk) {
  const ChunkDesc c = L.chunks[chunk];
  TileCtx ctx;
  ctx.t = L.tensors + c.tensor;
  ctx.start = (int64_t)c.chunk * kTile;
  int64_t rem = ctx.t->numel - ctx.start;
  ctx.n = rem > kTile ? kTile : (int)rem;
  return ctx;
}
__device__ __forceinline__ TileCtx tile_ctx(const MTLaunch& L) { return tile_ctx(L, blockIdx.x); }

template <typename F>
static inline void dispatch1(DType a, F&& f) {
  switch (a) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    case DType::BF16: f(bf16_t{}); break;
    default: break;
  }
}


static inline dim3 mt_grid(const MTLaunch& L) { return dim3((unsigned)L.nchunks); }

// Grid of the optimizer kernels (which walk the chunk list with a grid stride): one
// workgroup per chunk.  A persistent grid of CUs x {1, 2, 3, 4, 8} workgroups measured
// slower for SGD / Adam (tools/microbench.py optim, profiles/microbench_mb_optim.txt);
// the sweep knob was removed in round 6.
int device_cu_count();
static inline dim3 mt_pgrid(const MTLaunch& L) { return mt_grid(L); }

}  // namespace amd
