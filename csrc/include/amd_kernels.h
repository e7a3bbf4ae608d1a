// Host-callable launchers for every HIP kernel of the framework.
//
// These functions take raw device pointers, element dtypes and a hipStream_t;
// they never allocate or synchronise, so every one of them is safe inside a
// hipGraph capture.  The torch-facing layer (csrc/torch/*.cpp) owns tensors,
// validation and the multi-tensor table cache.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mt_table.h"

namespace amd {

enum class DType : int;

// A scale factor given either by value or by a device scalar; `invert` uses
// 1/x.  This is how the loss scale reaches kernels without a host sync.
struct ScaleArg {
  const float* ptr;
  float val;
  int invert;
};

// ----- multi-tensor elementwise (amp_C.multi_tensor_scale / axpby) ---------
void mt_scale(const MTLaunch& L, DType in, DType out, ScaleArg s, int* noop, hipStream_t st);
void mt_check_finite(const MTLaunch& L, DType in, int* noop, hipStream_t st);
void mt_axpby(const MTLaunch& L, DType x, DType y, DType out, ScaleArg a, ScaleArg b,
              int arg_to_check, int* noop, hipStream_t st);
void mt_fill_zero(const MTLaunch& L, DType t, hipStream_t st);
// [src, dst]: dst = src where *flag != 0 (guarded optimizer step restore)
void mt_copy_if(const MTLaunch& L, DType t, const int* flag, hipStream_t st);

// ----- norms (amp_C.multi_tensor_l2norm / _norm_out / max norm) ------------
// Per-chunk partials (sum of squares, or max|x| when max_norm) -> partials[nchunks].
void mt_norm_partials(const MTLaunch& L, DType in, int max_norm, float* partials, int* noop,
                      hipStream_t st);
// Reduce partials to a global norm (out_global, may be null) and per-tensor norms
// (out_per_tensor[ntensors], may be null).  `npart_sets` partial arrays are laid out
// back to back (stride nchunks); set k's results go to out_*[k*...].
void mt_norm_finalize(const MTLaunch& L, const float* partials, int npart_sets, int max_norm,
                      float* out_global, float* out_per_tensor, hipStream_t st);

// ----- optimizers ----------------------------------------------------------
struct SgdArgs {
  float wd, momentum, dampening, lr;
  int nesterov, first_run, wd_after_momentum;
  ScaleArg scale;           // grad multiplier (1/loss_scale when unscale is folded in)
  const float* lr_ptr;      // optional device lr (overrides lr)
  int* first_run_flag;      // optional device flag: first_run = (*flag == 0)
};
// depth 3: [g, p, m]; depth 4: [g, p, m, p_copy]
void mt_sgd(const MTLaunch& L, int depth, DType g, DType p, DType m, DType copy,
            const SgdArgs& a, const int* noop, hipStream_t st);
// two SGD launch sets in one launch: A = [g, p32, m32, copy16] (depth 4), B = [g32, p32, m32]
// (depth 3); false (nothing launched) for other dtype combinations
bool mt_sgd_pair(const MTLaunch& A, DType ga, DType pa, DType ca, const SgdArgs& aa,
                 const MTLaunch& B, DType gb, DType pb, const SgdArgs& ab, const int* noop,
                 hipStream_t st);
// after an SGD step: first_run_flag = 1 unless the step was skipped (noop set)
void mark_step_done(int* flag, const int* noop, hipStream_t st);

struct AdamArgs {
  float lr, beta1, beta2, eps, wd;
  int step;                 // host step (used when step_ptr == null)
  const int* step_ptr;      // optional device step counter (count of completed steps)
  int mode;                 // 0: L2 (g += wd*p), 1: decoupled (AdamW)
  int bias_correction;
  ScaleArg scale;           // grad multiplier
  const float* lr_ptr;
};
// depth 4: [g, p, m, v]; depth 5: [g, p, m, v, p_copy]   (m, v share p's dtype)
void mt_adam(const MTLaunch& L, int depth, DType g, DType p, DType copy, const AdamArgs& a,
             const int* noop, hipStream_t st);
// step counters: step += 1 unless noop set
void advance_step(int* step, const int* noop, hipStream_t st);

struct LambArgs {
  float lr, beta1, beta2, eps, wd;
  int step;
  const int* step_ptr;
  int mode;                 // 0: L2, 1: decoupled
  int bias_correction;
  int grad_averaging;
  const float* global_grad_norm;  // device scalar (already sqrt'ed)
  float max_grad_norm;
  int use_nvlamb;
  ScaleArg scale;
  const float* lr_ptr;
};
// stage 1: [g, p, m, v] -> updated m, v + partials (||p||^2, ||u||^2 per chunk)
void mt_lamb_stage1(const MTLaunch& L, DType g, DType p, const LambArgs& a, float* partials,
                    const int* noop, hipStream_t st);
// stage 2: [p, m, v] or [p, m, v, p_copy] (u recomputed); per-tensor norms from
// mt_norm_finalize
void mt_lamb_stage2(const MTLaunch& L, int depth, DType p, DType copy, const LambArgs& a,
                    const float* param_norms, const float* update_norms, const int* noop,
                    hipStream_t st);
// Legacy two-stage LAMB interface (apex multi_tensor_lamb_stage1_cuda / stage2_cuda):
// stage 1 lists [g, p, m, v, u]: Adam moments of g / clip (clip = max(1, ||g|| / max_norm),
// ||g|| a device scalar), u = m^ / (sqrt(v^) + eps) + decay[t] * p;  stage 2 lists [p, u]:
// p -= ratio_t * u with ratio_t = lr * ||p_t|| / ||u_t|| (nvlamb or wd != 0; lr when a norm
// is 0) - per-tensor decay / norms are device arrays [ntensors]
struct LambLegacyArgs {
  float beta1, beta2, eps, bc1, bc2;  // bias corrections 1 - beta^step
  const float* global_grad_norm;
  float max_grad_norm;
  const float* decay;
  float lr, wd;
  int use_nvlamb;
  const float* param_norms;
  const float* update_norms;
};
void mt_lamb_legacy_stage1(const MTLaunch& L, DType g, DType p, const LambLegacyArgs& a,
                           const int* noop, hipStream_t st);
void mt_lamb_legacy_stage2(const MTLaunch& L, DType p, DType u, const LambLegacyArgs& a,
                           const int* noop, hipStream_t st);

struct NovoArgs {
  float lr, beta1, beta2, eps, wd;
  int step;
  const int* step_ptr;
  int mode;                 // 0: L2-style (wd added to normalized grad), 1: decoupled
  int bias_correction;
  int grad_averaging;
  int norm_type;            // 0: inf norm, 2: L2 norm
  float init_zero;          // unused placeholder for API symmetry
  ScaleArg scale;
  const float* lr_ptr;
};
// NovoGrad: [g, p, m] with per-tensor second moments v[ntensors] (fp32, device)
// `grad_norms` holds this step's per-tensor grad norms; v is blended in-kernel
// by the first chunk of each tensor only after every chunk has read it -> the
// blend is done by a separate tiny kernel (novograd_blend) before the update.
void novograd_blend(float* v, const float* grad_norms, int ntensors, float beta2, int norm_type,
                    int first_step, const int* noop, hipStream_t st);
void mt_novograd(const MTLaunch& L, DType g, DType p, const NovoArgs& a, const float* v,
                 const int* noop, hipStream_t st);

struct AdagradArgs {
  float lr, eps, wd;
  int mode;                 // 0: L2, 1: decoupled
  ScaleArg scale;
  const float* lr_ptr;
};
// [g, p, h]
void mt_adagrad(const MTLaunch& L, DType g, DType p, const AdagradArgs& a, const int* noop,
                hipStream_t st);

// ----- loss scaler state machine (device resident) --------------------------
// if *overflow: scale = max(scale/factor, min_scale), unskipped = 0, ++skipped
// else: ++unskipped; if unskipped == window: scale = min(scale*factor, max), unskipped = 0
// applied (optional): receives the PRE-update scale (the one this step's grads carry)
void update_loss_scale(float* scale, int* unskipped, int* skipped_total, const int* overflow,
                       float factor, int window, float min_scale, float max_scale, int dynamic,
                       hipStream_t st, float* applied = nullptr);

// ----- flat buffers ---------------------------------------------------------
// out[i] = in[i] * s (cast between dtypes), optional finiteness flag.
// Copy host bytes to device memory through kernel arguments (graph-capture safe).
void upload_by_args(void* dst, const void* src, size_t bytes, hipStream_t st);

void flat_scale(const void* in, DType tin, void* out, DType tout, int64_t n, ScaleArg s,
                int* noop, hipStream_t st);

// ----- LayerNorm (apex fused_layer_norm_cuda) --------------------------------
struct LnFuse {
  const void* h = nullptr;     // fwd: sublayer output
  void* s = nullptr;           // fwd: residual sum out (LN input)
  const void* dres = nullptr;  // bwd: extra gradient of s (pre-LN residual stream), nullable
  void* dh = nullptr;          // bwd: gradient of h
  uint32_t seed = 0, thresh = 0;  // keep iff hash >= thresh (thresh = p * 2^32)
  float scale = 1.f;              // 1 / (1 - p)
  int th = -1;                    // DType of h / dh: -1 = the LN input's; an fp32 residual
                                  // stream may take an F16 / BF16 sublayer output (amp O1)
  int ty = -1;                    // >= 0 (mixed only): y / dy are in h's 16-bit type, the
                                  // dtype the consuming autocast GEMM reads (no cast kernel)
  void* dhsum = nullptr;          // bwd (with dgamma / dbeta): column sums of dh in gamma's
                                  // dtype - the bias gradient of the dense layer producing h
};
// fast-path requirements of the fused residual+dropout LayerNorm (16-B aligned, n2 % 8 == 0, <= 2048)
bool layer_norm_fused_ok(const void* x, const void* h, const void* s, const void* gamma,
                         const void* beta, const void* y, int64_t n2);
// x[n1, n2] (T), gamma/beta [n2] (TW, nullable), y [n1,n2] (T), mean/invvar [n1] fp32
void layer_norm_fwd(const void* x, DType tx, const void* gamma, const void* beta, DType tw,
                    void* y, float* mean, float* invvar, int64_t n1, int64_t n2, float eps,
                    int rms, hipStream_t st, const LnFuse* fuse = nullptr);
// dx [n1,n2]; dgamma/dbeta [n2] (TW) computed if non-null. `part` workspace
// must hold layer_norm_bwd_workspace(n1, n2) floats.
int64_t layer_norm_bwd_workspace(int64_t n1, int64_t n2);
// whether the fused-join backward can also form the dh column sums (LnFuse::dhsum) for n2
// nhwc_backward without ReLU / z / mask, plus the reduction (and finalize) of a second BN
// over the same rows and gradient (X2 mode of backward_k); ws: nhwc_backward_x2_workspace
void nhwc_backward_x2(const void* dy, const void* x, DType tx, const float* mean,
                      const float* invstd, const void* w, const void* b, DType tw,
                      const float* sum_dy, const float* sum_dy_xmu, float inv_count, void* dx,
                      int64_t M, int64_t C, const void* x2, const float* mean2,
                      const float* invstd2, float* sum_dy2, float* sum_dy_xmu2, void* gw2,
                      void* gb2, float* ws, hipStream_t st);
int64_t nhwc_backward_x2_workspace(int64_t M, int64_t C, DType tx);
// relu(BN(x) + BNz(xz)) + ReLU bitmask [M][C/8] in one pass (NHWC, C % 8 == 0, 16-byte
// aligned): the residual BN's output is formed on load, rounded as its apply would store it
void nhwc_apply2(const void* x, DType tx, const float* mean, const float* invstd, const void* w,
                 const void* b, DType tw, const void* xz, const float* meanz,
                 const float* invstdz, const void* wz, const void* bz, uint8_t* rmask, void* y,
                 int64_t M, int64_t C, hipStream_t st);
bool layer_norm_bwd_hsum_ok(int64_t n2);
// backward partial combine through one [R][n2] LDS row set instead of per-wave rows (A/B,
// default off: measured slower end to end)
void layer_norm_bwd_one_row(int on);
bool layer_norm_bwd_one_row_on();
void layer_norm_bwd(const void* dy, const void* x, DType tx, const void* gamma, DType tw,
                    const float* mean, const float* invvar, void* dx, void* dgamma, void* dbeta,
                    float* part, int64_t n1, int64_t n2, int rms, hipStream_t st,
                    const LnFuse* fuse = nullptr);

// ----- BatchNorm / SyncBN (apex syncbn) --------------------------------------
// Layout: NCHW  -> x viewed as [N, C, HW]; NHWC (channel-last) -> [M, C] with M = N*H*W.
// Per-channel statistics use split reductions: partial Welford (mean, M2, count)
// slabs then a combine, so small-C layers still cover all 256 CUs.
int64_t bn_stats_workspace(int64_t outer, int64_t C, int64_t inner, int channel_last);
// NHWC BN grid-sizing knobs (-1 keeps a value); get returns the 6 current values
void bn_set_tuning(int red_rpt, int red_cap, int red_min, int elem_rpt, int elem_cap, int elem_min);
void bn_get_tuning(int* out6);
// count_out (optional): receives the element count per channel (SyncBN packed stats)
void bn_local_stats(const void* x, DType tx, int64_t outer, int64_t C, int64_t inner,
                    int channel_last, float* mean, float* var_biased, float* ws, hipStream_t st,
                    float* count_out = nullptr);
// local (single-GPU) training stats: mean, invstd, running-stat update and
// num_batches_tracked += 1 in the finalize kernel
void bn_local_train_stats(const void* x, DType tx, int64_t outer, int64_t C, int64_t inner,
                          int channel_last, float* mean, float* invstd, float* running_mean,
                          float* running_var, long long* nbt, float eps, float momentum, float* ws,
                          hipStream_t st);
// combine world_size x (mean, var_biased, count) -> mean, invstd, unbiased var; and
// update running stats (may be null) with momentum.
void bn_combine_stats(const float* means, const float* vars, const float* counts, int world,
                      int64_t C, float eps, float momentum, float* mean_out, float* invstd_out,
                      float* running_mean, DType trm, void* running_var_any, float* var_out,
                      hipStream_t st, long long* nbt = nullptr, float* inv_total = nullptr);
// y = (x - mean) * invstd * w + b  [+ z] [relu]; relu_mask (channel-last, C % 8 == 0,
// 16-B aligned x/z/y; else ignored) receives one bit per element: output > 0
void bn_apply(const void* x, DType tx, const float* mean, const float* invstd,
              const void* weight, const void* bias, DType tw, const void* z, uint8_t* relu_mask,
              void* y, int64_t outer, int64_t C, int64_t inner, int channel_last, int relu,
              hipStream_t st);
// per-channel sum_dy, sum_dy_xmu (fp32) and grad_weight/grad_bias (TW) ; when relu
// is fused, dy is masked by (y > 0), read from relu_mask (channel-last only) or
// recomputed from x (and z).
void bn_reduce_grad(const void* dy, const void* x, DType tx, const float* mean,
                    const float* invstd, const void* weight, const void* bias, DType tw,
                    int relu, const void* z, const uint8_t* relu_mask, int64_t outer, int64_t C,
                    int64_t inner,
                    int channel_last, float* sum_dy, float* sum_dy_xmu, void* grad_weight,
                    void* grad_bias, float* ws, hipStream_t st,
                    const float* sum_scale = nullptr);
// dx = (dy' - mean_dy - (x-mean)*invstd^2*mean_dy_xmu) * invstd * w ; dz = dy' if z
void bn_backward_elemt(const void* dy, const void* x, DType tx, const float* mean,
                       const float* invstd, const void* weight, const void* bias, DType tw,
                       const float* sum_dy, const float* sum_dy_xmu, float inv_count,
                       int relu, const void* z, const uint8_t* relu_mask, void* dx, void* dz,
                       int64_t outer, int64_t C, int64_t inner, int channel_last, hipStream_t st);


// ---- NHWC max pooling (pool.hip) -------------------------------------------
// mean != nullptr: pool relu(x * invstd*w + (b - mean*invstd*w)) (BatchNorm + ReLU
// applied on load; w / b optional, all fp32 [C])
void maxpool2d_nhwc_fwd(const void* x, DType t, void* y, uint8_t* idx, int N, int H, int W, int C,
                        int OH, int OW, int k, int s, int p, hipStream_t st,
                        const float* mean = nullptr, const float* invstd = nullptr,
                        const float* bw = nullptr, const float* bb = nullptr);
void maxpool2d_nhwc_bwd(const void* dy, const uint8_t* idx, DType t, void* dx, int N, int H,
                        int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st);
// the 3x3 / stride-2 / pad-1 backward of the fused stem (C == 64, 16-bit) that also writes the
// BatchNorm + ReLU backward sums of dx: slab [2][64][maxpool_bwd_bn_grid(N, H, W)] of
// sum(d), sum(d * (x - mean)) with d = dx * (x * invstd*w + b - mean*invstd*w > 0)
bool maxpool2d_nhwc_bwd_bn_ok(int H, int W, int C, int OH, int OW, int k, int s, int p);
int maxpool_bwd_bn_grid(int N, int H, int W);
void maxpool2d_nhwc_bwd_bn(const void* dy, const uint8_t* idx, DType t, void* dx, int N, int H,
                           int W, int C, int OH, int OW, const void* x, const float* mean,
                           const float* invstd, const float* bw, const float* bb, float* slab,
                           hipStream_t st);
// global average pool backward: dx[N, HW, C] (channels-last) = dy[N, C] / HW
void gap_nhwc_bwd(const void* dy, DType t, void* dx, int64_t N, int64_t HW, int C,
                  hipStream_t st);

// ---- 256 x 256 one-wave-per-SIMD MFMA GEMM (gemm4w.hip) -------------------------
// C[M, N] = A[M, K] . B[N, K]^T, bf16 / fp16 row-major (K contiguous), fp32 accumulation.
// epi 0: C = bf16(acc); 1: pre = bf16(acc + bias) -> aux (if non-null), C = gelu(pre);
// 2: C = bf16(bf16(acc) * gelu'(aux)) and colsum[M-tile][N] = per-tile column sums of C.
// Requires N % 256 == 0, K % 64 == 0 (gemm4w_supported); M ragged.
struct GemmArgs {
  const void* A;               // bf16
  const void* B;               // bf16
  void* C;                     // bf16
  int M, N, K, lda, ldb, ldc;  // ldc also strides aux
  const void* bias;            // [N] bf16 (or fp32 when bias_f32), epi 1
  int bias_f32;
  void* aux;                   // bf16 [M][ldc] pre-activation: written (epi 1) / read (epi 2)
  float* colsum;               // [ceil(M / 256)][N] (epi 2), may be null
  int tanh;                    // GELU flavour: 1 tanh approximation, 0 erf
  int fp16;                    // operands / outputs fp16 instead of bf16
  int group_m;                 // tile order: groups of group_m m-tiles (set by gemm4w())
  float* slab;                 // epi 3: BatchNorm statistics [2][N][ceil(M / 256)] (channel-major)
  const float* shift;          // epi 3: per-column shift s of the sums (v - s), (v - s)^2; may be null
};
bool gemm4w_supported(int M, int N, int K);
void gemm4w(const GemmArgs& a, int epi, hipStream_t st);
// dense weight gradients P[s] = A_s^T B_s over row splits (wgrad4w.hip): A [T, M], B [T, N]
// row-major bf16 / fp16, fp32 partials P [S][M][N]; M, N % 256 == 0, (T / S) % 64 == 0
struct WgradArgs {
  const void* A;
  const void* B;
  float* P;
  int M, N, lda, ldb;
  int rows;     // rows of A / B per split (T / S)
  int S;
  int fp16;
  int group_m;  // <= 0: default (4)
  float* colsum = nullptr;  // optional [S][M]: column sums of A per split (the bias gradient
                            // of dY, formed from the MFMA fragments)
};
bool wgrad4w_supported(int64_t T, int M, int N, int S);
void wgrad4w(const WgradArgs& a, hipStream_t st);

// ---- implicit-GEMM convolutions, NHWC bf16, MFMA (conv_igemm.hip) ----------
// 3x3 pad 1 or 1x1 pad 0, stride 1 or 2; channel counts multiples of 64
bool conv3x3_nhwc_supported(int Cin, int Cout);
// 3x3 stride-1 convs run the halo-resident kernel (conv3h_k) where their window fits,
// unless disabled here: mode 0 off, 1 automatic, 64 / 128 force that output-tile width
// where possible (A/B switch; the M tile, hence the stats slab width, follows)
void conv_halo_enable(int mode);
// conv_tap_k tile order: N tiles folded into grid x, N fastest: 0 off, 1 by shape
// (default), 2 every launch (A/B switch)
void conv_nfast(int mode);
void conv_halo_nfast(int on);  // the same for the halo 3x3 kernel (A/B)
// halo kernel pixel tile: 0 automatic (by grid rounds), 224 / 256 forced (A/B)
void conv_halo_mtile(int bm);
int conv_halo_enabled();
void conv_bnbwd_early(int mode);
// stride-1 1x1 forwards with Cout % 256 == 0 on gemm4w (statistics epilogue): 0 off, 1 the
// measured winners, 2 every eligible shape; the query tells whether conv_nhwc_fwd takes it
void conv_1x1_gemm4w(int mode);
bool conv_1x1_on_gemm4w(int64_t M, int Cin, int Cout);
// y is N x Ho x Wo x Cout, Ho = (H-1)/stride + 1; w is [Cout][k*k][Cin]
// stats_slab (optional, fp32 [conv_fwd_mtiles(...)][2][Cout]): per M-tile shifted sums
// sum(y - shift[c]), sum((y - shift[c])^2) of the bf16 output for the consuming BN
void conv_nhwc_fwd(const void* x, const void* w, void* y, int N, int H, int W, int Cin, int Cout,
                   int ksize, int stride, hipStream_t st, float* stats_slab = nullptr,
                   const float* stats_shift = nullptr);
int conv_fwd_mtiles(int N, int H, int W, int Cout, int stride, int ksize, int Cin);
// M tiles (slab rows) of conv_nhwc_fwd_bnbwd's stride-1 launch
int conv_bnbwd_mtiles(int N, int H, int W, int Cout, int ksize, int Cin);
// BatchNorm-backward epilogue of a data-gradient conv (conv_nhwc_fwd on dY with the
// rotated / transposed filter): the conv output o (+ add, the residual gradient) is
// the gradient of a BN(+ReLU) output; the kernel stores g = relu_mask(x) * o instead
// and writes that BN's per-M-tile sums [2][C][S]: sum(g), sum(g * (x - mean)).
// relu_mode 0: no ReLU; 1: bitmask rmask [M][C/8] from the forward; 2: recompute
// x * invstd * w + (b - mean * invstd * w) > 0 (w, b fp32 or null = 1 / 0).
struct ConvBnEpi {
  const void* add;       // bf16 [M][C] or null
  const void* xbn;       // bf16 [M][C]: the BN input
  const uint8_t* rmask;  // relu_mode 1
  const float* mean;     // [C]
  const float* invstd;   // [C] (relu_mode 2)
  const float* w;        // [C] or null (relu_mode 2)
  const float* b;        // [C] or null (relu_mode 2)
  int relu_mode;
  int add_s2;            // 1: `add` is COMPACT [N][H/2][W/2][C] and lands on the even
                         // (h, w) pixels only (a stride-2 1x1 downsample's input gradient)
};
void conv_nhwc_fwd_bnbwd(const void* dy, const void* w, void* g, int N, int H, int W, int Cin,
                         int Cout, int ksize, int stride, const ConvBnEpi& ep, float* slab,
                         hipStream_t st);
// BatchNorm statistics from such a slab: local training mode (mean, invstd, running
// stats, num_batches_tracked) or SyncBN's packed [mean | biased var | count]
// (slab is channel-major [2][C][S]: one launch, no workspace)
void bn_slab_train_stats(const float* slab, int S, int64_t C, int64_t count, const float* shift,
                         float* mean, float* invstd, float* running_mean, float* running_var,
                         long long* nbt, float eps, float momentum, hipStream_t st);
void bn_slab_packed_stats(const float* slab, int S, int64_t C, int64_t count, const float* shift,
                          float* packed, hipStream_t st);
// BN backward sums (sum_dy, sum_dy_xmu [* sum_scale], dgamma, dbeta) from a
// conv_nhwc_fwd_bnbwd slab [2][C][S]
// Host-side switch read when the BN backward finalize is launched (this thread): dgamma /
// dbeta ACCUMULATE into the caller's gradient buffers - DDP bucket views - instead of
// being written fresh, saving autograd's two add kernels per BatchNorm (BNAccumScope)
bool bn_grad_accumulate();
void bn_set_grad_accumulate(bool on);
struct BNAccumScope {
  bool prev;
  explicit BNAccumScope(bool on) : prev(bn_grad_accumulate()) { bn_set_grad_accumulate(on); }
  ~BNAccumScope() { bn_set_grad_accumulate(prev); }
};
void bn_slab_reduce_grad(const float* slab, int S, int64_t C, const float* invstd,
                         float* sum_dy, float* sum_dy_xmu, void* gw, void* gb, DType tw,
                         hipStream_t st, const float* sum_scale = nullptr);
// data gradient of a stride-2 conv (H, W even); wt = rotated 3x3 filter / W^T for 1x1
void conv_nhwc_dgrad_s2(const void* dy, const void* wt, void* dx, int N, int H, int W, int Cin,
                        int Cout, int ksize, hipStream_t st);
// the 3x3 form with the BN-backward epilogue (ep.add must be null); slab [2][Cin][S],
// S = conv_dgrad_s2_bnbwd_mtiles(N, H, W)
int conv_dgrad_s2_bnbwd_mtiles(int N, int H, int W);
void conv_nhwc_dgrad_s2_bnbwd(const void* dy, const void* wt, void* gout, int N, int H, int W,
                              int Cin, int Cout, const ConvBnEpi& ep, float* slab,
                              hipStream_t st);
// weight gradient: split-K over output pixels into fp32 partials [S][k*k][Cout][Cin],
// then a reduce into dW (KRSC, bf16 or fp32).  algo 0 = per-tap MFMA kernel,
// 1 = all-9-taps strip kernel (3x3 stride 1, W <= 56), 4 = 64-channel strip-ring kernel
// (3x3 stride 1, Cin = Cout = 64, W <= 56: conv3x3_wgrad_c64_ok)
int conv_wgrad_splits(int N, int H, int W, int Cin, int Cout, int ksize, int stride, int algo);
bool conv3x3_wgrad_supported(int W, int algo);
bool conv3x3_wgrad_c64_ok(int W, int Cin, int Cout, int ksize, int stride);
int64_t conv_wgrad_workspace(int S, int Cin, int Cout, int ksize);  // floats
// generic split-K slab reduction: out[co][ci] = sum_s part[s][co][ci] (n % 4 == 0)
int64_t splitk_reduce_workspace(int S, int64_t n);
void splitk_reduce(const float* part, int S, int Cout, int Cin, float* stage, void* out,
                   bool out_fp32, hipStream_t st, bool accum = false);
// 16-bit W'[ci][2-r][2-s][co] = W[co][r][s][ci] (data-gradient filter)
void conv3x3_rot_weight(const void* w, void* out, int Cout, int Cin, hipStream_t st);
// W^T ([Cin][Cout]) of a 16-bit 1x1 filter [Cout][Cin] (LDS-tiled transpose)
void conv1x1_transpose_weight(const void* w, void* out, int Cout, int Cin, hipStream_t st);
// batched backward weight layouts in one launch: filter k [cout][taps][cin] (16-bit) ->
// out[cin][taps-1-t][cout] (taps 9: the rotated 3x3 filter; taps 1: W^T)
void prep_weights(const void* const* w, void* const* out, const int* cout, const int* cin,
                  const int* taps, int n, hipStream_t st);
void conv_nhwc_wgrad(const void* dy, const void* x, float* part, void* dw, bool dw_fp32, int N,
                     int H, int W, int Cin, int Cout, int ksize, int stride, int S, int algo,
                     hipStream_t st, bool accum = false);

// ---- ResNet stem: 7x7 / stride 2 / pad 3, 3 -> 64 channels, NHWC bf16 (stem_conv.hip) ----
bool stem_conv_supported(int N, int H, int W);
// x [N][H][W][3] -> xp [N][H+6][W+6][4] (zero border, zero 4th channel)
void stem_pad(const void* x, void* xp, int N, int H, int W, hipStream_t st);
// wk: packed filter [64][7][32] (wk[co][r][4s+c] = W[co][c][r][s], zeros elsewhere);
// y [N][H/2][W/2][64]; with `slab` also the BatchNorm statistics of y (sums of y - shift and
// (y - shift)^2 per channel, shift may be null) as a channel-major slab [2][64][S],
// S = stem_fwd_slab_width(N, H)
void stem_fwd(const void* xp, const void* wk, void* y, int N, int H, int W, hipStream_t st,
              float* slab = nullptr, const float* shift = nullptr);
int stem_fwd_slab_width(int N, int H);
// fp32 partials [S][64][256] of the packed filter gradient (n = 32 r + 4 s + c)
int stem_wgrad_splits(int N, int H);
void stem_wgrad(const void* xp, const void* dy, float* part, int S, int N, int H, int W,
                hipStream_t st);

// ---- dense-layer bias gradients (bias_grad.hip) ------------------------------
// bias_grad[n] = sum_m g[m, n] for a row-major [M, N] (bf16 / fp16 / fp32, N % 8 ==
// 0, 16-byte aligned); act_mode 1 / 2: g = dh * gelu'(pre) (erf / tanh GELU), 3 / 4:
// g = dh * relu'(y) / dh * sigmoid'(y) from the saved output y (passed as `pre`) is
// computed in the same pass and written to out_dpre.  part: S * N floats.
int colsum_splits(int64_t M, int N);
// out[n] = sum_s part[s][n] (fp32 partial slab [S][N]) in dtype tb
void colsum_finalize(const float* part, int S, int N, void* out, DType tb, hipStream_t st);
// y = gelu(x) (erf or tanh), n % 8 == 0, 16-byte aligned
void gelu_fwd(const void* x, void* y, DType t, int64_t n, bool tanh_approx, hipStream_t st);
void colsum(const void* x, const void* pre, void* out_dpre, DType t, int64_t M, int N,
            int act_mode, float* part, int S, void* bias_grad, DType tb, hipStream_t st);

// ---- fused attention, head dim 64 (attention.hip) ---------------------------
struct AttnLaunch {
  const void* q;
  const void* k;
  const void* v;
  int64_t qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh;  // element strides of [B,S,H,64] views
  void* o;      // [B][S][H][64] contiguous
  float* lse;   // [B][H][S]
  int B, H, S;
  float scale, dropout;
  uint32_t seed;
  int lse_stride;  // row stride of lse, a multiple of 64 (attn_lse_stride(S))
  bool causal;
  DType dtype;  // BF16 or F16
};
int attn_lse_stride(int S);
void attn_fwd(const AttnLaunch& L, hipStream_t st);

// backward: preprocess D = rowsum(dO*O), dK/dV kernel, dQ kernel (no atomics)
struct AttnBwdLaunch {
  const void* q;
  const void* k;
  const void* v;
  const void* o;
  const void* dout;
  int64_t qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss, osh, dsb, dss, dsh;
  void* dq;     // strided [B,S,H,64] outputs
  void* dk;
  void* dv;
  int64_t dqsb, dqss, dqsh, dksb, dkss, dksh, dvsb, dvss, dvsh;
  const float* lse;  // [B][H][lse_stride]
  float* D;          // workspace [B][H][lse_stride]
  int lse_stride;
  int B, H, S;
  float scale, dropout;
  uint32_t seed;
  bool causal;
  DType dtype;
};
void attn_bwd(const AttnBwdLaunch& L, hipStream_t st);

// ---- fused softmax cross entropy with label smoothing (xentropy.hip) ---------
// x [rows, V] row-major (T = fp32/fp16/bf16); loss [rows] (TO), lse [rows] fp32
void xentropy_fwd(const void* x, DType tx, const int64_t* labels, int64_t rows, int V,
                  float smoothing, int64_t padding_idx, void* loss, DType tloss, float* lse,
                  hipStream_t st);
// dx [rows, V] (x's dtype) = dloss * (softmax - (1-eps) onehot - eps/V)
void xentropy_bwd(const void* dloss, DType tg, const void* x, DType tx, const float* lse,
                  const int64_t* labels, int64_t rows, int V, float smoothing,
                  int64_t padding_idx, void* dx, hipStream_t st);

// ---- deterministic embedding weight gradient (embedding.hip) ------------------
// sorted / perm: the stable sort of the T token ids and its permutation; out [V, H]
// must be zero-filled; runs of equal ids are summed in sorted order (fp32), runs
// longer than 256 positions in chunk partials (slots: embedding_wgrad_slots(T, H)
// floats of workspace) joined in chunk order.
int64_t embedding_wgrad_slots(int64_t T, int H);
void embedding_wgrad(const int64_t* sorted, const int64_t* perm, const void* dy, DType tdy,
                     int64_t T, int H, int64_t pad, void* out, DType tout, bool vec,
                     float* slots, hipStream_t st);

}  // namespace amd
