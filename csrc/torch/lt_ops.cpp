// hipBLASLt GEMMs with fused epilogues for the transformer FFN (fused_dense):
//
//   dense_gelu_fwd:    h = gelu(x @ W1^T + b1) and pre = x @ W1^T + b1 from ONE GEMM
//                      (HIPBLASLT_EPILOGUE_GELU_AUX_BIAS: pre is the epilogue's aux
//                      output) - no separate GELU pass over the [tokens x 4h] tensor;
//   dense_dgelu_bgrad: dpre = (dy @ W2) * gelu'(pre) and db1 = sum_rows(dpre) from ONE
//                      GEMM (HIPBLASLT_EPILOGUE_DGELU_BGRAD, pre read as aux input) -
//                      dh is never written or re-read.
//
// hipBLASLt's GELU is the tanh approximation (apex's fused_dense semantics: its
// cuBLASLt GELU epilogues are the same function), so these back
// FusedDenseGeluDense(approximate="tanh").  Row-major tensors are handed to the
// column-major library as their transposes: a row-major [M, N] output is a
// column-major [N, M] matrix whose rows (length-N bias / bias-gradient vectors)
// are the output features.  Algorithms come from the library heuristic once per
// (epilogue, shape, dtype) and are cached; when the library offers none for a
// shape the op reports it and the caller falls back to GEMM + kernel passes.
#include "lt_ops.h"

#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace amd {

namespace {

#define LT_CHECK(expr)                                                                   \
  do {                                                                                   \
    hipblasStatus_t s_ = (expr);                                                         \
    TORCH_CHECK(s_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt call failed (", (int)s_, "): ", \
                #expr);                                                                  \
  } while (0)

constexpr size_t kWorkspace = 32u << 20;

hipblasLtHandle_t handle_for_device() {
  static std::mutex mu;
  static std::map<int, hipblasLtHandle_t> handles;
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice failed");
  std::lock_guard<std::mutex> g(mu);
  auto it = handles.find(dev);
  if (it != handles.end()) return it->second;
  hipblasLtHandle_t h;
  LT_CHECK(hipblasLtCreate(&h));
  handles[dev] = h;
  return h;
}

hipDataType hip_type(at::ScalarType t) {
  switch (t) {
    case at::kBFloat16: return HIP_R_16BF;
    case at::kHalf: return HIP_R_16F;
    case at::kFloat: return HIP_R_32F;
    default: TORCH_CHECK(false, "hipBLASLt epilogue GEMM: unsupported dtype ", t);
  }
  return HIP_R_32F;
}

struct Desc {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  ~Desc() {
    if (a) hipblasLtMatrixLayoutDestroy(a);
    if (b) hipblasLtMatrixLayoutDestroy(b);
    if (c) hipblasLtMatrixLayoutDestroy(c);
    if (op) hipblasLtMatmulDescDestroy(op);
  }
};

using AlgoKey = std::tuple<int, int64_t, int64_t, int64_t, int, int, int, int>;

struct AlgoCache {
  std::mutex mu;
  std::map<AlgoKey, std::pair<bool, hipblasLtMatmulAlgo_t>> map;
};
AlgoCache& algo_cache() {
  static AlgoCache c;
  return c;
}

// D[m, n] (column-major, ld = m) = op(A) op(B) with the epilogue configured in d.op;
// returns false when the heuristic has no algorithm for this problem
bool run(Desc& d, const AlgoKey& key, const void* A, const void* B, void* D, int64_t m,
         int64_t n, hipDataType dt) {
  hipblasLtHandle_t h = handle_for_device();
  hipblasLtMatmulAlgo_t algo;
  {
    AlgoCache& c = algo_cache();
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.map.find(key);
    if (it == c.map.end()) {
      hipblasLtMatmulPreference_t pref;
      LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
      uint64_t ws = kWorkspace;
      LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(
          pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
      hipblasLtMatmulHeuristicResult_t res[1];
      int got = 0;
      hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, d.op, d.a, d.b, d.c, d.c, pref, 1,
                                                           res, &got);
      hipblasLtMatmulPreferenceDestroy(pref);
      const bool ok = st == HIPBLAS_STATUS_SUCCESS && got > 0 &&
                      res[0].state == HIPBLAS_STATUS_SUCCESS;
      it = c.map.emplace(key, std::make_pair(ok, ok ? res[0].algo : hipblasLtMatmulAlgo_t{}))
               .first;
    }
    if (!it->second.first) return false;
    algo = it->second.second;
  }
  (void)m;
  (void)n;
  (void)dt;
  at::Tensor ws = at::empty({(int64_t)kWorkspace},
                            at::TensorOptions().dtype(at::kByte).device(at::kCUDA));
  const float alpha = 1.f, beta = 0.f;
  LT_CHECK(hipblasLtMatmul(h, d.op, &alpha, A, d.a, B, d.b, &beta, D, d.c, D, d.c, &algo,
                           ws.data_ptr(), kWorkspace, cur_stream()));
  return true;
}

void set_attr(hipblasLtMatmulDesc_t op, hipblasLtMatmulDescAttributes_t a, const void* v,
              size_t n) {
  LT_CHECK(hipblasLtMatmulDescSetAttribute(op, a, v, n));
}

}  // namespace

std::vector<at::Tensor> dense_gelu_fwd_op(at::Tensor x2, at::Tensor w, at::Tensor b) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(x2.is_cuda() && x2.dim() == 2 && w.dim() == 2 && b.dim() == 1,
              "dense_gelu_fwd: x [M, K], w [N, K], b [N] on the GPU");
  TORCH_CHECK(x2.scalar_type() == w.scalar_type() && b.scalar_type() == w.scalar_type(),
              "dense_gelu_fwd: x, w and b must share one dtype");
  x2 = x2.contiguous();
  w = w.contiguous();
  b = b.contiguous();
  const int64_t M = x2.size(0), K = x2.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && b.size(0) == N, "dense_gelu_fwd: shape mismatch");
  const hipDataType dt = hip_type(x2.scalar_type());
  at::Tensor h = at::empty({M, N}, x2.options());
  at::Tensor pre = at::empty({M, N}, x2.options());
  Desc d;
  // column-major: H'[N, M] = W'[K, N]^T X'[K, M]
  LT_CHECK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const uint32_t epi = HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  const void* bp = b.data_ptr();
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
  const int32_t bdt = dt;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bdt, sizeof(bdt));
  void* ap = pre.data_ptr();
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &ap, sizeof(ap));
  const int64_t ald = N;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ald, sizeof(ald));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.a, dt, K, N, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.b, dt, K, M, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.c, dt, N, M, N));
  const AlgoKey key{(int)epi, M, N, K, (int)dt, 1, 0, 0};
  if (!run(d, key, w.data_ptr(), x2.data_ptr(), h.data_ptr(), N, M, dt)) return {};
  return {h, pre};
}

std::vector<at::Tensor> dense_dgelu_bgrad_op(at::Tensor dy2, at::Tensor w2, at::Tensor pre,
                                             at::ScalarType bias_dtype) {
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dy2.is_cuda() && dy2.dim() == 2 && w2.dim() == 2 && pre.dim() == 2,
              "dense_dgelu_bgrad: dy [M, N2], w2 [N2, N], pre [M, N] on the GPU");
  TORCH_CHECK(dy2.scalar_type() == w2.scalar_type() && pre.scalar_type() == w2.scalar_type(),
              "dense_dgelu_bgrad: dy, w2 and pre must share one dtype");
  dy2 = dy2.contiguous();
  w2 = w2.contiguous();
  pre = pre.contiguous();
  const int64_t M = dy2.size(0), N2 = dy2.size(1), N = w2.size(1);
  TORCH_CHECK(w2.size(0) == N2 && pre.size(0) == M && pre.size(1) == N,
              "dense_dgelu_bgrad: shape mismatch");
  const hipDataType dt = hip_type(dy2.scalar_type());
  at::Tensor dpre = at::empty({M, N}, dy2.options());
  at::Tensor db = at::empty({N}, dy2.options().dtype(bias_dtype));
  Desc d;
  // column-major: DPRE'[N, M] = W2'[N, N2] DY'[N2, M], epilogue * gelu'(PRE'), row sums
  LT_CHECK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const uint32_t epi = HIPBLASLT_EPILOGUE_DGELU_BGRAD;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  void* bp = db.data_ptr();
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
  const int32_t bdt = hip_type(bias_dtype);
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bdt, sizeof(bdt));
  const void* ap = pre.data_ptr();
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &ap, sizeof(ap));
  const int64_t ald = N;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ald, sizeof(ald));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.a, dt, N, N2, N));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.b, dt, N2, M, N2));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.c, dt, N, M, N));
  const AlgoKey key{(int)epi, M, N, N2, (int)dt, 0, 0, (int)bdt};
  if (!run(d, key, w2.data_ptr(), dy2.data_ptr(), dpre.data_ptr(), N, M, dt)) return {};
  return {dpre, db};
}

std::vector<at::Tensor> dense_wgrad_bgrad_op(at::Tensor dy2, at::Tensor x2,
                                             at::ScalarType w_dtype, at::ScalarType bias_dtype) {
  // dW[N, K] = dy2[M, N]^T x2[M, K] with db[N] = column sums of dy2 from the SAME
  // GEMM (HIPBLASLT_EPILOGUE_BGRADB): the GEMM streams dy anyway, so the bias
  // gradient costs no extra pass over it.  Column-major: dW'[K, N] = X'[K, M] op(DY')
  // with DY' stored [N, M] and op = T; BGRADB reduces op(B) over the k (= M) axis.
  c10::NoGradGuard no_grad_;
  TORCH_CHECK(dy2.is_cuda() && dy2.dim() == 2 && x2.dim() == 2 && dy2.size(0) == x2.size(0),
              "dense_wgrad_bgrad: dy [M, N], x [M, K] on the GPU");
  TORCH_CHECK(dy2.scalar_type() == x2.scalar_type(), "dense_wgrad_bgrad: dy / x dtype mismatch");
  dy2 = dy2.contiguous();
  x2 = x2.contiguous();
  const int64_t M = dy2.size(0), N = dy2.size(1), K = x2.size(1);
  const hipDataType dt = hip_type(dy2.scalar_type()), ot = hip_type(w_dtype);
  at::Tensor dw = at::empty({N, K}, dy2.options().dtype(w_dtype));
  at::Tensor db = at::empty({N}, dy2.options().dtype(bias_dtype));
  Desc d;
  LT_CHECK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_T;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const uint32_t epi = HIPBLASLT_EPILOGUE_BGRADB;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  void* bp = db.data_ptr();
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
  const int32_t bdt = hip_type(bias_dtype);
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bdt, sizeof(bdt));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.a, dt, K, M, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.b, dt, N, M, N));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.c, ot, K, N, K));
  const AlgoKey key{(int)epi, M, N, K, (int)dt, (int)ot, 1, (int)bdt};
  if (!run(d, key, x2.data_ptr(), dy2.data_ptr(), dw.data_ptr(), K, N, dt)) return {};
  return {dw, db};
}

int64_t lt_probe_op(int64_t m, int64_t n, int64_t k, int64_t epilogue, int64_t ta, int64_t tb,
                    at::ScalarType dtype, int64_t aux_type, int64_t bias_type) {
  // diagnostics: how many algorithms the heuristic offers for an epilogue / layout
  Desc d;
  const hipDataType dt = hip_type(dtype);
  LT_CHECK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t a = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, b = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &a, sizeof(a));
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &b, sizeof(b));
  const uint32_t epi = (uint32_t)epilogue;
  set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  if (bias_type >= 0) {
    const int32_t bt = (int32_t)bias_type;
    set_attr(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  if (aux_type >= 0) {
    const int32_t at_ = (int32_t)aux_type;
    set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at_, sizeof(at_));
    const int64_t ld = m;
    set_attr(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
  }
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.a, dt, ta ? k : m, ta ? m : k, ta ? k : m));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.b, dt, tb ? n : k, tb ? k : n, tb ? n : k));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.c, dt, m, n, m));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspace;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES,
                                                 &ws, sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(handle_for_device(), d.op, d.a, d.b, d.c,
                                                       d.c, pref, 8, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  return st == HIPBLAS_STATUS_SUCCESS ? got : -(int64_t)st;
}

void lt_algo_cache_clear() {
  AlgoCache& c = algo_cache();
  std::lock_guard<std::mutex> g(c.mu);
  c.map.clear();
}

}  // namespace amd
