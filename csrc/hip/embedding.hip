// Deterministic, host-sync-free embedding weight gradient (VERDICT r2 missing 5).
//
//   dW[v, :] = sum over tokens t with idx[t] == v of dY[t, :]      (fp32 accumulation)
//
// PyTorch's CUDA embedding backward sizes its segment reduction on the HOST (it reads
// the number of unique indices back with .item()), and the float-atomic scatter-add
// it can be replaced with is not reproducible.  Here the indices are sorted on the
// device (stable radix sort: equal ids keep token order), then one launch with a
// wave64 per sorted position: a wave whose position starts a run of equal ids (or a
// 256-position chunk of a longer run) sums those dY rows in sorted order and writes
// the row of dW (or a partial row, joined in chunk order by a second launch) - a fixed
// order, so bitwise reproducible; every other wave exits at once.  The grid is sized by the token
// count, which the host knows, so nothing is read back.  Rows no token used stay
// zero (the output is zero-filled first); the padding row is never written.
//
// Lanes own 8 consecutive columns (one 16-byte load of a 16-bit dY row chunk); a
// run's rows are read 4 at a time so several loads are in flight per lane.
#include <cstdlib>

#include "amd_dev.h"
#include "amd_kernels.h"

namespace amd {

namespace {

constexpr int kEmbThreads = 256;  // 4 waves = 4 sorted positions per workgroup
// A run longer than kEmbChunk sorted positions is summed in chunk-aligned segments by
// separate waves (fp32 partial rows), then joined in order by a second launch: a run of
// thousands of equal ids (BERT's 2-row token-type table takes all 16,384 tokens in two
// runs) was one wave's serial loop - 2.9 ms of a 52 ms BERT-large step.
constexpr int kEmbChunk = 256;

// Segment starts: a run start, or a chunk boundary inside a run.  A segment ends at
// the run end or the next chunk boundary.  A whole run writes its row of dW; a piece
// of a longer run writes its fp32 partial to slotA[c] (segment starting at the chunk
// boundary c * kEmbChunk) or slotB[c] (a run start inside chunk c, run continuing past
// the chunk) - at most one of each per chunk.
template <typename TI, typename TO, bool VEC>
__global__ void __launch_bounds__(kEmbThreads)
    emb_wgrad_k(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                const TI* __restrict__ dy, int64_t T, int H, int64_t pad, TO* __restrict__ out,
                float* __restrict__ slots, int64_t nchunks) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * (kEmbThreads / 64) + (threadIdx.x >> 6);
  if (p >= T) return;
  const int64_t v = sorted[p];
  if (v == pad || v < 0) return;
  const bool run_start = p == 0 || sorted[p - 1] != v;
  if (!run_start && p % kEmbChunk != 0) return;  // not a segment start
  const int64_t cend = (p / kEmbChunk + 1) * kEmbChunk;
  const int64_t lim = cend < T ? cend : T;
  // segment [p, q1): the run's end within the chunk, 64 positions per ballot (a serial
  // scan was a chain of up to 255 dependent L2 loads)
  int64_t q1 = p + 1;
  for (;;) {
    const int64_t q = q1 + lane;
    const unsigned long long m = __ballot(q < lim && sorted[q] == v);
    const int n = ~m == 0ull ? 64 : __builtin_ctzll(~m);
    q1 += n;
    if (n < 64) break;
  }
  const bool whole = run_start && (q1 == T || sorted[q1] != v);
  float* slot = nullptr;
  if (!whole)
    slot = slots + ((p % kEmbChunk == 0 ? 0 : nchunks) + p / kEmbChunk) * (int64_t)H;
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
    if (whole) {
      TO* dst = out + v * (int64_t)H + c0;
      if constexpr (VEC) store8(dst, acc);
      else dst[0] = from_f32<TO>(acc[0]);
    } else {
#pragma unroll
      for (int i = 0; i < W; ++i) slot[c0 + i] = acc[i];
    }
  }
}

// One wave per (chunk c, block of 64*W columns): if a run starts in chunk c and
// continues past it, sum its segment partials in chunk order (slotA / slotB of chunk
// c, then slotA of every following chunk the run reaches) for those columns and write
// them to the run's row of dW.  The run's chunk count comes from one ballot over 64
// chunk starts at a time, so the partial loads are independent and issued 8 deep (a
// loop testing sorted[] before every partial was a chain of dependent loads: 60 us).
template <typename TO, bool VEC>
__global__ void __launch_bounds__(kEmbThreads)
    emb_wgrad_join_k(const int64_t* __restrict__ sorted, int64_t T, int H, int64_t pad,
                     TO* __restrict__ out, const float* __restrict__ slots, int64_t nchunks,
                     int ncb) {
  constexpr int W = VEC ? 4 : 1;
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)blockIdx.x * (kEmbThreads / 64) + (threadIdx.x >> 6);
  const int64_t c = wv / ncb;
  const int cb = (int)(wv - c * ncb);
  if (c >= nchunks) return;
  const int64_t c_lo = c * kEmbChunk;
  const int64_t last = (c_lo + kEmbChunk < T ? c_lo + kEmbChunk : T) - 1;
  if (last + 1 >= T) return;
  const int64_t v = sorted[last];
  if (v == pad || v < 0 || sorted[last + 1] != v) return;  // no run crosses the chunk end
  const bool from_boundary = sorted[c_lo] == v;
  if (from_boundary && c > 0 && sorted[c_lo - 1] == v) return;  // started in an earlier chunk
  int64_t kend = c + 1;  // the run covers the starts of chunks [c + 1, kend)
  for (;;) {
    const int64_t k = kend + lane;
    const bool cont = k * kEmbChunk < T && sorted[k * kEmbChunk] == v;
    const unsigned long long m = __ballot(cont);
    const int n = ~m == 0ull ? 64 : __builtin_ctzll(~m);
    kend += n;
    if (n < 64) break;
  }
  const int c0 = (cb * 64 + lane) * W;
  if (c0 >= H) return;
  const float* first = slots + ((from_boundary ? 0 : nchunks) + c) * (int64_t)H + c0;
  float acc[W];
#pragma unroll
  for (int i = 0; i < W; ++i) acc[i] = first[i];
  int64_t k = c + 1;
  for (; k + 8 <= kend; k += 8) {
    float r[8][W];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float* src = slots + (k + u) * (int64_t)H + c0;
      if constexpr (VEC) {
        const float4 t = *reinterpret_cast<const float4*>(src);
        r[u][0] = t.x; r[u][1] = t.y; r[u][2] = t.z; r[u][3] = t.w;
      } else {
        r[u][0] = src[0];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < W; ++i) acc[i] += r[u][i];
  }
  for (; k < kend; ++k)
#pragma unroll
    for (int i = 0; i < W; ++i) acc[i] += slots[k * (int64_t)H + c0 + i];
  TO* dst = out + v * (int64_t)H + c0;
#pragma unroll
  for (int i = 0; i < W; ++i) dst[i] = from_f32<TO>(acc[i]);
}

template <typename F>
void dispatch_t(DType t, F&& f) {
  switch (t) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(half_t{}); break;
    case DType::BF16: f(bf16_t{}); break;
    default: abort();  // callers (csrc/torch/emb_ops.cpp) admit fp32 / fp16 / bf16 only
  }
}

}  // namespace

int64_t embedding_wgrad_slots(int64_t T, int H) {
  return 2 * ((T + kEmbChunk - 1) / kEmbChunk) * (int64_t)H;
}

void embedding_wgrad(const int64_t* sorted, const int64_t* perm, const void* dy, DType tdy,
                     int64_t T, int H, int64_t pad, void* out, DType tout, bool vec,
                     float* slots, hipStream_t st) {
  if (T == 0 || H == 0) return;
  const int64_t blocks = (T + kEmbThreads / 64 - 1) / (kEmbThreads / 64);
  const int64_t nchunks = (T + kEmbChunk - 1) / kEmbChunk;
  dispatch_t(tdy, [&](auto a) {
    dispatch_t(tout, [&](auto b) {
      using TI = decltype(a);
      using TO = decltype(b);
      if (vec)
        hipLaunchKernelGGL((emb_wgrad_k<TI, TO, true>), dim3((unsigned)blocks), dim3(kEmbThreads),
                           0, st, sorted, perm, static_cast<const TI*>(dy), T, H, pad,
                           static_cast<TO*>(out), slots, nchunks);
      else
        hipLaunchKernelGGL((emb_wgrad_k<TI, TO, false>), dim3((unsigned)blocks),
                           dim3(kEmbThreads), 0, st, sorted, perm, static_cast<const TI*>(dy), T,
                           H, pad, static_cast<TO*>(out), slots, nchunks);
      if (nchunks > 1) {
        const bool v4 = H % 4 == 0;  // slots rows are then 16-byte aligned (fp32, H % 4)
        const int ncb = v4 ? (H + 255) / 256 : (H + 63) / 64;
        const int64_t waves = nchunks * ncb;
        const int64_t jblocks = (waves + kEmbThreads / 64 - 1) / (kEmbThreads / 64);
        if (v4)
          hipLaunchKernelGGL((emb_wgrad_join_k<TO, true>), dim3((unsigned)jblocks),
                             dim3(kEmbThreads), 0, st, sorted, T, H, pad, static_cast<TO*>(out),
                             slots, nchunks, ncb);
        else
          hipLaunchKernelGGL((emb_wgrad_join_k<TO, false>), dim3((unsigned)jblocks),
                             dim3(kEmbThreads), 0, st, sorted, T, H, pad, static_cast<TO*>(out),
                             slots, nchunks, ncb);
      }
    });
  });
}

}  // namespace amd
