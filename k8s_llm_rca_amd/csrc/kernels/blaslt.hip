// Native hipBLASLt front end for the library GEMMs of the engine (B4).
//
// Y[M][N] = X[M][K] . W[N][K]^T, bf16 in/out, fp32 compute -- the projections
// that the measured dispatch leaves to the library (prefill-sized M, and the
// decode buckets where hipBLASLt beats the hand-written kernels).
//
// Why not torch.nn.functional.linear: an eager mixed prefill+decode step
// issues ~130 GEMMs, and each F.linear costs ~28 us of host time on this
// stack (dispatcher + per-call descriptor setup + algorithm heuristic), which
// is ~3.6 ms of an eager step's ~8.8 ms issue time (cProfile of the engine
// thread, tools/_host_prof.sh) -- time in which the GPU can run dry.  Here the
// matmul/layout descriptors and the heuristic's algorithm are built once per
// (M, N, K, ldx, ldy) and cached, so a call is a hash lookup plus
// hipblasLtMatmul.  Same solution family as torch's path (top heuristic
// result), so the GPU time is unchanged.
//
// Layout: hipBLASLt is column-major.  Row-major Y[M][N] is column-major
// Y^T[N][M] (ld = ldy) = W . X^T: A = the column-major K x N image of W
// (lda = K) transposed, B = the column-major K x M image of X (ldb = ldx).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <mutex>
#include <unordered_map>

#include "common.h"

namespace {

struct Key {
  int M, N, K, ldx, ldy;
  bool operator==(const Key& o) const {
    return M == o.M && N == o.N && K == o.K && ldx == o.ldx && ldy == o.ldy;
  }
};

struct KeyHash {
  size_t operator()(const Key& k) const {
    size_t h = (size_t)k.M * 0x9E3779B97F4A7C15ull;
    h ^= (size_t)k.N * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2);
    h ^= (size_t)k.K * 0x165667B19E3779F9ull + (h << 6) + (h >> 2);
    h ^= (size_t)k.ldx * 0x27D4EB2F165667C5ull + (h << 6) + (h >> 2);
    h ^= (size_t)k.ldy + (h << 6) + (h >> 2);
    return h;
  }
};

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
};

std::mutex g_mu;
hipblasLtHandle_t g_handle = nullptr;
std::unordered_map<Key, Plan, KeyHash> g_plans;

int build_plan(const Key& k, size_t ws_limit, Plan* out) {
  Plan p;
  hipblasStatus_t st;
  st = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  if (st != HIPBLAS_STATUS_SUCCESS) return 1000 + (int)st;
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  // A: K x N (lda = K), B: K x M (ldb = ldx), C/D: N x M (ldc = ldy)
  if (hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, k.K, k.N, k.K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, k.K, k.M, k.ldx) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, k.N, k.M, k.ldy) != HIPBLAS_STATUS_SUCCESS)
    return 1100;
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsl = ws_limit;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsl, sizeof(wsl));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  st = hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.a, p.b, p.c, p.c, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return 1200 + (int)st;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  *out = p;
  return 0;
}

}  // namespace

// ws: device scratch of ws_bytes (reused by every call on the stream; must
// outlive any HIP graph that captured a call).
K8S_API int k8s_blaslt_gemm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, void* ws,
                            size_t ws_bytes, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldy < N) return (int)hipErrorInvalidValue;
  const Key key{M, N, K, ldx, ldy};
  Plan* plan;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_handle == nullptr && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return 900;
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      Plan p;
      const int rc = build_plan(key, ws_bytes, &p);
      if (rc) return rc;
      it = g_plans.emplace(key, p).first;
    }
    plan = &it->second;
  }
  if (plan->ws > ws_bytes) return 1300;
  const float alpha = 1.f, beta = 0.f;
  hipblasStatus_t st = hipblasLtMatmul(g_handle, plan->desc, &alpha, w, plan->a, x, plan->b, &beta, y, plan->c, y,
                                       plan->c, &plan->algo, ws, plan->ws, s);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : 1400 + (int)st;
}

K8S_API int k8s_blaslt_num_plans() {
  std::lock_guard<std::mutex> g(g_mu);
  return (int)g_plans.size();
}
