// Deterministic, host-sync-free embedding weight gradient (VERDICT r2 missing 5).
//
//   dW[v, :] = sum over tokens t with idx[t] == v of dY[t, :]      (fp32 accumulation)
//
// PyTorch's CUDA embedding backward sizes its segment reduction on the HOST (it reads
// the number of unique indices back with .item()), and the float-atomic scatter-add
// it can be replaced with is not reproducible.  Here the indices are sorted on the
// device (stable radix sort: equal ids keep token order), then ONE launch with a
// wave64 per sorted position: a wave whose position starts a run of equal ids sums
// that run's dY rows in sorted order (fixed order -> bitwise reproducible) and writes
// the row of dW; every other wave exits at once.  The grid is sized by the token
// count, which the host knows, so nothing is read back.  Rows no token used stay
// zero (the output is zero-filled first); the padding row is never written.
//
// Lanes own 8 consecutive columns (one 16-byte load of a 16-bit dY row chunk); a
// run's rows are read 4 at a time so several loads are in flight per lane.
#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

constexpr int kEmbThreads = 256;  // 4 waves = 4 sorted positions per workgroup

template <typename TI, typename TO, bool VEC>
__global__ void __launch_bounds__(kEmbThreads)
    emb_wgrad_k(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                const TI* __restrict__ dy, int64_t T, int H, int64_t pad, TO* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * (kEmbThreads / 64) + (threadIdx.x >> 6);
  if (p >= T) return;
  const int64_t v = sorted[p];
  if ((p > 0 && sorted[p - 1] == v) || v == pad || v < 0) return;  // not a run start
  int64_t q1 = p + 1;
  while (q1 < T && sorted[q1] == v) ++q1;                           // run [p, q1)
  constexpr int W = VEC ? 8 : 1;
  for (int c0 = lane * W; c0 < H; c0 += 64 * W) {
    float acc[W];
#pragma unroll
    for (int i = 0; i < W; ++i) acc[i] = 0.f;
    int64_t q = p;
    for (; q + 4 <= q1; q += 4) {
      float r[4][W];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const TI* src = dy + perm[q + u] * (int64_t)H + c0;
        if constexpr (VEC) load8(src, r[u]);
        else r[u][0] = to_f32(src[0]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < W; ++i) acc[i] += r[u][i];
    }
    for (; q < q1; ++q) {
      float r[W];
      const TI* src = dy + perm[q] * (int64_t)H + c0;
      if constexpr (VEC) load8(src, r);
      else r[0] = to_f32(src[0]);
#pragma unroll
      for (int i = 0; i < W; ++i) acc[i] += r[i];
    }
    TO* dst = out + v * (int64_t)H + c0;
    if constexpr (VEC) store8(dst, acc);
    else dst[0] = from_f32<TO>(acc[0]);
  }
}

template <typename F>
void dispatch_t(DType t, F&& f) {
  switch (t) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    default: f(bf16_t{}); break;
  }
}

}  // namespace

void embedding_wgrad(const int64_t* sorted, const int64_t* perm, const void* dy, DType tdy,
                     int64_t T, int H, int64_t pad, void* out, DType tout, bool vec,
                     hipStream_t st) {
  if (T == 0 || H == 0) return;
  const int64_t blocks = (T + kEmbThreads / 64 - 1) / (kEmbThreads / 64);
  dispatch_t(tdy, [&](auto a) {
    dispatch_t(tout, [&](auto b) {
      using TI = decltype(a);
      using TO = decltype(b);
      if (vec)
        hipLaunchKernelGGL((emb_wgrad_k<TI, TO, true>), dim3((unsigned)blocks), dim3(kEmbThreads),
                           0, st, sorted, perm, static_cast<const TI*>(dy), T, H, pad,
                           static_cast<TO*>(out));
      else
        hipLaunchKernelGGL((emb_wgrad_k<TI, TO, false>), dim3((unsigned)blocks),
                           dim3(kEmbThreads), 0, st, sorted, perm, static_cast<const TI*>(dy), T,
                           H, pad, static_cast<TO*>(out));
    });
  });
}

}  // namespace amd
