// BatchNorm / SyncBatchNorm for gfx950: public entry points + NCHW kernels.
// The channels-last (NHWC) kernels live in bn_nhwc.hip.
//
// Behavioural spec: apex@f3a960f8 csrc/welford.cu:
// welford_mean_var(_c_last), welford_parallel, batchnorm_forward(_c_last) with
// optional +z and fused ReLU, reduce_bn(_c_last), batchnorm_backward(_c_last),
// relu_bw_c_last.
//
// MI355X design:
//  * every tensor is viewed as [outer, C, inner]: NHWC = [N*H*W, C, 1],
//    NCHW = [N, C, H*W];
//  * per-channel reductions are SPLIT over many workgroups (apex launches one
//    block per channel: 64 blocks for a C=64 layer on a 256-CU chip) and every
//    split writes a partial slab; a finalize kernel sums the slabs in a fixed
//    order -> deterministic, no float atomics, no inter-workgroup hand-off;
//  * statistics use sums shifted by a per-channel sample value (the channel's
//    first element) so the one-pass sum / sum-of-squares does not cancel;
//  * forward apply fuses (x*scale + shift) [+ residual z] [ReLU]; backward fuses
//    the ReLU mask (recomputed from x, no saved activation) and emits dz for the
//    residual branch.
#include "bn_common.h"

namespace amd {

namespace {

// NCHW reduction splits per channel: >= 2048 elements per split, ~2048 blocks.
int nchw_splits(int64_t N, int64_t C, int64_t HW) {
  int64_t per_ch = N * HW;
  int64_t want = (2048 + C - 1) / C;
  int64_t maxs = (per_ch + 2047) / 2048;
  if (want > maxs) want = maxs;
  return (int)(want < 1 ? 1 : want);
}

bool nchw_vec(int64_t HW, std::initializer_list<const void*> ps) {
  return HW % 8 == 0 && all_aligned(ps);
}

int elem_grid(int64_t work_items) {
  int64_t b = (work_items + kBNThreads - 1) / kBNThreads;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

// ---------------------------------------------------------------- statistics
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
    stats_nchw(const T* __restrict__ x, int64_t N, int C, int64_t HW, int vec,
               float* __restrict__ slab) {
  __shared__ float scratch[kBNThreads / kWave];
  const int c = blockIdx.y;
  const int64_t L = N * HW;  // elements of this channel
  const float k = to_f32(x[(int64_t)c * HW]);
  float s1 = 0.f, s2 = 0.f;
  if (vec) {
    const int64_t LV = L / 8;
    const int64_t per = (LV + gridDim.x - 1) / gridDim.x;
    const int64_t v0 = (int64_t)blockIdx.x * per;
    const int64_t v1 = v0 + per < LV ? v0 + per : LV;
    for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      int64_t e = v * 8;
      int64_t n = e / HW, hw = e - n * HW;
      float a[8];
      load8(x + (n * C + c) * HW + hw, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = a[i] - k;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
    }
  } else {
    const int64_t per = (L + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per;
    const int64_t e1 = e0 + per < L ? e0 + per : L;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      int64_t n = e / HW, hw = e - n * HW;
      float d = to_f32(x[(n * C + c) * HW + hw]) - k;
      s1 += d;
      s2 = fmaf(d, d, s2);
    }
  }
  s1 = block_sum(s1, scratch);
  s2 = block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    slab[(size_t)blockIdx.x * 2 * C + c] = s1;
    slab[(size_t)blockIdx.x * 2 * C + C + c] = s2;
  }
}

// ---------------------------------------------------------------- combine
template <typename TR>
__global__ void __launch_bounds__(256)
    combine_kernel(const float* __restrict__ means, const float* __restrict__ vars,
                   const float* __restrict__ counts, int world, int C, float eps, float momentum,
                   float* __restrict__ mean_out, float* __restrict__ invstd_out,
                   float* __restrict__ running_mean, TR* __restrict__ running_var,
                   float* __restrict__ var_out, long long* __restrict__ nbt,
                   float* __restrict__ inv_total) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (c == 0) {
    if (nbt) *nbt += 1;
    if (inv_total) {
      float t = 0.f;
      for (int w = 0; w < world; ++w) t += counts[w];
      *inv_total = 1.f / t;
    }
  }
  float mean = 0.f, m2 = 0.f, n = 0.f;
  for (int w = 0; w < world; ++w) {
    float nb = counts[w];
    welford_combine(mean, m2, n, means[(size_t)w * C + c], vars[(size_t)w * C + c] * nb, nb);
  }
  float var_b = n > 0.f ? m2 / n : 0.f;
  mean_out[c] = mean;
  invstd_out[c] = rsqrtf(var_b + eps);
  if (var_out) var_out[c] = var_b;
  if (running_mean) {
    float unb = n > 1.f ? m2 / (n - 1.f) : var_b;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    float rv = to_f32(running_var[c]);
    running_var[c] = from_f32<TR>((1.f - momentum) * rv + momentum * unb);
  }
}

// ---------------------------------------------------------------- apply
template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    apply_nchw(const T* __restrict__ x, const float* __restrict__ mean,
               const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
               const T* __restrict__ z, T* __restrict__ y, int64_t N, int C, int64_t HW, int vec,
               int relu) {
  const int64_t total = N * C * HW;
  const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
  if (vec) {
    const int64_t nv = total / 8;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gstride) {
      int64_t e = v * 8;
      int c = (int)((e / HW) % C);
      float sc, sh;
      chan_affine(mean, invstd, wload(w, c, 1.f), wload(b, c, 0.f), c, sc, sh);
      float a[8], zz[8];
      load8(x + e, a);
      if (z) load8(z + e, zz);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = fmaf(a[i], sc, sh);
        if (z) o += zz[i];
        a[i] = relu ? fmaxf(o, 0.f) : o;
      }
      store8(y + e, a);
    }
  } else {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gstride) {
      int c = (int)((e / HW) % C);
      float sc, sh;
      chan_affine(mean, invstd, wload(w, c, 1.f), wload(b, c, 0.f), c, sc, sh);
      float o = fmaf(to_f32(x[e]), sc, sh);
      if (z) o += to_f32(z[e]);
      y[e] = from_f32<T>(relu ? fmaxf(o, 0.f) : o);
    }
  }
}

// ---------------------------------------------------------------- backward reduce
template <typename T, typename TW>
__global__ void __launch_bounds__(kBNThreads)
    reduce_nchw(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
                const float* __restrict__ invstd, const TW* __restrict__ w,
                const TW* __restrict__ b, const T* __restrict__ z, int relu, int64_t N, int C,
                int64_t HW, int vec, float* __restrict__ slab) {
  __shared__ float scratch[kBNThreads / kWave];
  const int c = blockIdx.y;
  const int64_t L = N * HW;
  const float mu = mean[c];
  float sc, sh;
  chan_affine(mean, invstd, wload(w, c, 1.f), wload(b, c, 0.f), c, sc, sh);
  float s1 = 0.f, s2 = 0.f;
  if (vec) {
    const int64_t LV = L / 8;
    const int64_t per = (LV + gridDim.x - 1) / gridDim.x;
    const int64_t v0 = (int64_t)blockIdx.x * per;
    const int64_t v1 = v0 + per < LV ? v0 + per : LV;
    for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      int64_t e = v * 8;
      int64_t n = e / HW, hw = e - n * HW;
      int64_t off = (n * C + c) * HW + hw;
      float xv[8], dv[8], zv[8];
      load8(x + off, xv);
      load8(dy + off, dv);
      if (relu && z) load8(z + off, zv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = dv[i];
        if (relu) {
          float o = fmaf(xv[i], sc, sh);
          if (z) o += zv[i];
          d = o > 0.f ? d : 0.f;
        }
        s1 += d;
        s2 = fmaf(d, xv[i] - mu, s2);
      }
    }
  } else {
    const int64_t per = (L + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per;
    const int64_t e1 = e0 + per < L ? e0 + per : L;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      int64_t n = e / HW, hw = e - n * HW;
      int64_t off = (n * C + c) * HW + hw;
      float xv = to_f32(x[off]);
      float d = to_f32(dy[off]);
      if (relu) {
        float o = fmaf(xv, sc, sh);
        if (z) o += to_f32(z[off]);
        d = o > 0.f ? d : 0.f;
      }
      s1 += d;
      s2 = fmaf(d, xv - mu, s2);
    }
  }
  s1 = block_sum(s1, scratch);
  s2 = block_sum(s2, scratch);
  if (threadIdx.x == 0) {
    slab[(size_t)blockIdx.x * 2 * C + c] = s1;
    slab[(size_t)blockIdx.x * 2 * C + C + c] = s2;
  }
}

// ---------------------------------------------------------------- backward elementwise
template <typename T, typename TW, bool VEC>
__global__ void __launch_bounds__(kBNThreads)
    bwd_nchw(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
             const float* __restrict__ invstd, const TW* __restrict__ w, const TW* __restrict__ b,
             const float* __restrict__ sum_dy, const float* __restrict__ sum_dy_xmu, float inv_n,
             int relu, const T* __restrict__ z, T* __restrict__ dx, T* __restrict__ dz, int64_t N,
             int C, int64_t HW) {
  constexpr int W = VEC ? 8 : 1;
  const int64_t total = N * C * HW;
  const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nitems = total / W;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < nitems; it += gstride) {
    const int64_t e = it * W;
    const int c = (int)((e / HW) % C);
    const float wc = wload(w, c, 1.f);
    float sc, sh;
    chan_affine(mean, invstd, wc, wload(b, c, 0.f), c, sc, sh);
    const float is = invstd[c], mu = mean[c];
    const float mdy = sum_dy[c] * inv_n, mdyx = sum_dy_xmu[c] * inv_n;
    const float k1 = is * wc, k2 = -is * is * mdyx * is * wc, k3 = -mdy * is * wc;
    float xv[W], dv[W], zv[W];
    if constexpr (VEC) {
      load8(x + e, xv);
      load8(dy + e, dv);
      if (relu && z) load8(z + e, zv);
    } else {
      xv[0] = to_f32(x[e]);
      dv[0] = to_f32(dy[e]);
      if (relu && z) zv[0] = to_f32(z[e]);
    }
#pragma unroll
    for (int i = 0; i < W; ++i) {
      float d = dv[i];
      if (relu) {
        float o = fmaf(xv[i], sc, sh);
        if (z) o += zv[i];
        d = o > 0.f ? d : 0.f;
      }
      dv[i] = d;
      xv[i] = fmaf(d, k1, fmaf(xv[i] - mu, k2, k3));
    }
    if constexpr (VEC) {
      store8(dx + e, xv);
      if (dz) store8(dz + e, dv);
    } else {
      dx[e] = from_f32<T>(xv[0]);
      if (dz) dz[e] = from_f32<T>(dv[0]);
    }
  }
}

}  // namespace

// ============================================================================ public API
int64_t bn_stats_workspace(int64_t outer, int64_t C, int64_t inner, int channel_last) {
  int64_t s = channel_last ? std::max(nhwc_splits(outer, C, true), nhwc_splits(outer, C, false))
                           : nchw_splits(outer, C, inner);
  return s * 2 * C;
}

static void local_stats_impl(const void* x, DType tx, int64_t outer, int64_t C, int64_t inner,
                             int channel_last, const BNStatsOut& out, float* ws, hipStream_t st) {
  const int64_t count = outer * inner;
  if (count == 0 || C == 0) return;
  if (channel_last) return nhwc_stats(x, tx, outer, C, out, ws, st);
  const int splits = nchw_splits(outer, C, inner);
  const int vec = nchw_vec(inner, {x}) ? 1 : 0;
  bn_dispatch(tx, [&](auto t0) {
    using T = decltype(t0);
    const T* xp = static_cast<const T*>(x);
    hipLaunchKernelGGL((stats_nchw<T>), dim3(splits, (unsigned)C), dim3(kBNThreads), 0, st, xp,
                       outer, (int)C, inner, vec, ws);
    launch_stats_finalize<T>(xp, ws, splits, C, count, inner, out, st);
  });
}

void bn_local_stats(const void* x, DType tx, int64_t outer, int64_t C, int64_t inner,
                    int channel_last, float* mean, float* var_biased, float* ws, hipStream_t st,
                    float* count_out) {
  BNStatsOut out{mean, var_biased, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f};
  out.count_out = count_out;
  out.count_val = (float)(outer * inner);
  local_stats_impl(x, tx, outer, C, inner, channel_last, out, ws, st);
}

void bn_local_train_stats(const void* x, DType tx, int64_t outer, int64_t C, int64_t inner,
                          int channel_last, float* mean, float* invstd, float* running_mean,
                          float* running_var, long long* nbt, float eps, float momentum, float* ws,
                          hipStream_t st) {
  BNStatsOut out{mean, nullptr, invstd, running_mean, running_var, nbt, eps, momentum};
  local_stats_impl(x, tx, outer, C, inner, channel_last, out, ws, st);
}

void bn_combine_stats(const float* means, const float* vars, const float* counts, int world,
                      int64_t C, float eps, float momentum, float* mean_out, float* invstd_out,
                      float* running_mean, DType trm, void* running_var_any, float* var_out,
                      hipStream_t st, long long* nbt, float* inv_total) {
  (void)trm;
  hipLaunchKernelGGL((combine_kernel<float>), dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st,
                     means, vars, counts, world, (int)C, eps, momentum, mean_out, invstd_out,
                     running_mean, static_cast<float*>(running_var_any), var_out, nbt, inv_total);
}

void bn_apply(const void* x, DType tx, const float* mean, const float* invstd,
              const void* weight, const void* bias, DType tw, const void* z, uint8_t* relu_mask,
              void* y, int64_t outer, int64_t C, int64_t inner, int channel_last, int relu,
              hipStream_t st) {
  if (outer * inner * C == 0) return;
  if (channel_last)
    return nhwc_apply(x, tx, mean, invstd, weight, bias, tw, z, relu_mask, y, outer, C, relu, st);
  const bool vec = nchw_vec(inner, {x, z, y});
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      int64_t items = vec ? outer * C * inner / 8 : outer * C * inner;
      hipLaunchKernelGGL((apply_nchw<T, TW>), dim3(elem_grid(items)), dim3(kBNThreads), 0, st,
                         static_cast<const T*>(x), mean, invstd, static_cast<const TW*>(weight),
                         static_cast<const TW*>(bias), static_cast<const T*>(z),
                         static_cast<T*>(y), outer, (int)C, inner, vec ? 1 : 0, relu);
    });
  });
}

void bn_reduce_grad(const void* dy, const void* x, DType tx, const float* mean,
                    const float* invstd, const void* weight, const void* bias, DType tw,
                    int relu, const void* z, const uint8_t* relu_mask, int64_t outer, int64_t C,
                    int64_t inner, int channel_last, float* sum_dy, float* sum_dy_xmu,
                    void* grad_weight, void* grad_bias, float* ws, hipStream_t st,
                    const float* sum_scale) {
  if (outer * inner * C == 0) return;
  if (channel_last)
    return nhwc_reduce(dy, x, tx, mean, invstd, weight, bias, tw, relu, z, relu_mask, outer, C,
                       sum_dy, sum_dy_xmu, grad_weight, grad_bias, ws, st, sum_scale);
  const int splits = nchw_splits(outer, C, inner);
  const int vec = nchw_vec(inner, {dy, x, z}) ? 1 : 0;
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      hipLaunchKernelGGL((reduce_nchw<T, TW>), dim3(splits, (unsigned)C), dim3(kBNThreads), 0, st,
                         static_cast<const T*>(dy), static_cast<const T*>(x), mean, invstd,
                         static_cast<const TW*>(weight), static_cast<const TW*>(bias),
                         static_cast<const T*>(z), relu, outer, (int)C, inner, vec, ws);
      launch_reduce_finalize<TW>(ws, splits, C, invstd, sum_dy, sum_dy_xmu, static_cast<TW*>(grad_weight),
                         static_cast<TW*>(grad_bias), st, sum_scale);
    });
  });
}

void bn_backward_elemt(const void* dy, const void* x, DType tx, const float* mean,
                       const float* invstd, const void* weight, const void* bias, DType tw,
                       const float* sum_dy, const float* sum_dy_xmu, float inv_count,
                       int relu, const void* z, const uint8_t* relu_mask, void* dx, void* dz,
                       int64_t outer, int64_t C, int64_t inner, int channel_last,
                       hipStream_t st) {
  if (outer * inner * C == 0) return;
  if (channel_last)
    return nhwc_backward(dy, x, tx, mean, invstd, weight, bias, tw, sum_dy, sum_dy_xmu,
                         inv_count, relu, z, relu_mask, dx, dz, outer, C, st);
  const bool vec = nchw_vec(inner, {dy, x, z, dx, dz});
  bn_dispatch(tx, [&](auto t0) {
    bn_dispatch(tw, [&](auto w0) {
      using T = decltype(t0);
      using TW = decltype(w0);
      const int64_t items = vec ? outer * C * inner / 8 : outer * C * inner;
      auto launch = [&](auto V) {
        hipLaunchKernelGGL((bwd_nchw<T, TW, decltype(V)::value>), dim3(elem_grid(items)),
                           dim3(kBNThreads), 0, st, static_cast<const T*>(dy),
                           static_cast<const T*>(x), mean, invstd, static_cast<const TW*>(weight),
                           static_cast<const TW*>(bias), sum_dy, sum_dy_xmu, inv_count, relu,
                           static_cast<const T*>(z), static_cast<T*>(dx), static_cast<T*>(dz),
                           outer, (int)C, inner);
      };
      if (vec) launch(std::true_type{});
      else launch(std::false_type{});
    });
  });
}

}  // namespace amd
