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
//
// Measured algorithm choice (k8s_blaslt_tune): at prefill-sized M (256..8192)
// the heuristic's first solution is not always the fastest one it lists, so
// the engine times the top candidates once per (N, K) at a ladder of M at
// init; a later plan for any M takes the candidate tuned at the largest
// ladder M <= M, if hipBLASLt confirms it supports the problem; below the
// ladder (decode sizes: data/gemm_dispatch_*.json) and otherwise, the heuristic's.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <iterator>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace {

struct Key {
  int M, N, K, ldx, ldy, f32out;
  bool operator==(const Key& o) const {
    return M == o.M && N == o.N && K == o.K && ldx == o.ldx && ldy == o.ldy && f32out == o.f32out;
  }
};

struct KeyHash {
  size_t operator()(const Key& k) const {
    size_t h = (size_t)k.M * 0x9E3779B97F4A7C15ull;
    h ^= (size_t)k.N * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2);
    h ^= (size_t)k.K * 0x165667B19E3779F9ull + (h << 6) + (h >> 2);
    h ^= (size_t)k.ldx * 0x27D4EB2F165667C5ull + (h << 6) + (h >> 2);
    h ^= (size_t)k.ldy + (h << 6) + (h >> 2);
    h ^= (size_t)k.f32out * 0x9E3779B1ull;
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
// (N, K) -> ladder M -> tuned algorithm, used for M in [ladder M, hi]
struct Tuned {
  hipblasLtMatmulAlgo_t algo;
  int hi;
};
std::map<std::pair<int, int>, std::map<int, Tuned>> g_tuned;

int make_desc(const Key& k, Plan* p) {
  hipblasStatus_t st = hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  if (st != HIPBLAS_STATUS_SUCCESS) return 1000 + (int)st;
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  // A: K x N (lda = K), B: K x M (ldb = ldx), C/D: N x M (ldc = ldy)
  if (hipblasLtMatrixLayoutCreate(&p->a, HIP_R_16BF, k.K, k.N, k.K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p->b, HIP_R_16BF, k.K, k.M, k.ldx) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p->c, k.f32out ? HIP_R_32F : HIP_R_16BF, k.N, k.M, k.ldy) != HIPBLAS_STATUS_SUCCESS)
    return 1100;
  return 0;
}

int heuristic(const Plan& p, size_t ws_limit, int want, hipblasLtMatmulHeuristicResult_t* res, int* n) {
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsl = ws_limit;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsl, sizeof(wsl));
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.a, p.b, p.c, p.c, pref, want, res, n);
  hipblasLtMatmulPreferenceDestroy(pref);
  return (st != HIPBLAS_STATUS_SUCCESS || *n < 1) ? 1200 + (int)st : 0;
}

int build_plan(const Key& k, size_t ws_limit, Plan* out) {
  Plan p;
  int rc = make_desc(k, &p);
  if (rc) return rc;
  auto t = g_tuned.find({k.N, k.K});
  if (!k.f32out && t != g_tuned.end() && !t->second.empty()) {
    auto it = t->second.upper_bound(k.M);  // first ladder M > M
    hipblasLtMatmulAlgo_t algo;
    size_t wsz = 0;
    const float alpha = 1.f, beta = 0.f;
    if (it != t->second.begin() && k.M <= std::prev(it)->second.hi && (algo = std::prev(it)->second.algo, true) &&
        hipblaslt_ext::matmulIsAlgoSupported(g_handle, p.desc, &alpha, p.a, p.b, &beta, p.c, p.c, algo, wsz) ==
            HIPBLAS_STATUS_SUCCESS &&
        wsz <= ws_limit) {
      p.algo = algo;
      p.ws = wsz;
      *out = p;
      return 0;
    }
  }
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  rc = heuristic(p, ws_limit, 1, res, &n);
  if (rc) return rc;
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  *out = p;
  return 0;
}

}  // namespace

// ws: device scratch of ws_bytes (reused by every call on the stream; must
// outlive any HIP graph that captured a call).  f32out: Y is fp32 (the lm_head's
// logits, B9: sampling reads fp32 logits), else bf16.
K8S_API int k8s_blaslt_gemm2(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, void* ws,
                             size_t ws_bytes, hipStream_t s, int f32out) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldy < N) return (int)hipErrorInvalidValue;
  const Key key{M, N, K, ldx, ldy, f32out ? 1 : 0};
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

K8S_API int k8s_blaslt_gemm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, void* ws,
                            size_t ws_bytes, hipStream_t s) {
  return k8s_blaslt_gemm2(x, ldx, w, y, ldy, M, N, K, ws, ws_bytes, s, 0);
}

K8S_API int k8s_blaslt_num_plans() {
  std::lock_guard<std::mutex> g(g_mu);
  return (int)g_plans.size();
}

// Time the heuristic's top `max_algos` solutions for this problem (`iters`
// launches each on stream s, after 2 warm-up launches) and keep the fastest
// for (N, K) at ladder point M.  Plans already built for (N, K) are dropped so
// later calls re-plan against the tuned table (their descriptors are kept
// alive: a concurrent caller may still hold one).  Not capturable (events +
// synchronisation): call at init, before any HIP-graph capture.
// times[0] = heuristic first choice (us), times[1] = chosen (us).
// Returns the chosen candidate's rank in the heuristic list, or < 0 on error.
K8S_API int k8s_blaslt_tune(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, void* ws,
                            size_t ws_bytes, int max_algos, int iters, hipStream_t s, float* times) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldy < N || max_algos < 1 || iters < 1) return -(int)hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(g_mu);
  if (g_handle == nullptr && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return -900;
  const Key key{M, N, K, ldx, ldy, 0};
  Plan p;
  int rc = make_desc(key, &p);
  if (rc) return -rc;
  std::vector<hipblasLtMatmulHeuristicResult_t> res(max_algos);
  int n = 0;
  rc = heuristic(p, ws_bytes, max_algos, res.data(), &n);
  if (rc) return -rc;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -901;
  const float alpha = 1.f, beta = 0.f;
  int best = -1;
  float best_us = 0.f, first_us = -1.f;
  for (int i = 0; i < n; ++i) {
    if (res[i].workspaceSize > ws_bytes) continue;
    bool ok = true;
    for (int r = 0; r < 2 && ok; ++r)
      ok = hipblasLtMatmul(g_handle, p.desc, &alpha, w, p.a, x, p.b, &beta, y, p.c, y, p.c, &res[i].algo, ws,
                           res[i].workspaceSize, s) == HIPBLAS_STATUS_SUCCESS;
    if (!ok || hipStreamSynchronize(s) != hipSuccess) continue;
    hipEventRecord(e0, s);
    for (int r = 0; r < iters; ++r)
      hipblasLtMatmul(g_handle, p.desc, &alpha, w, p.a, x, p.b, &beta, y, p.c, y, p.c, &res[i].algo, ws,
                      res[i].workspaceSize, s);
    hipEventRecord(e1, s);
    if (hipEventSynchronize(e1) != hipSuccess) continue;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const float us = 1000.f * ms / iters;
    if (i == 0) first_us = us;
    if (best < 0 || us < best_us) {
      best = i;
      best_us = us;
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (best < 0) return -1500;
  g_tuned[{N, K}][M] = Tuned{res[best].algo, 1 << 30};
  for (auto it = g_plans.begin(); it != g_plans.end();) {
    if (it->first.N == N && it->first.K == K)
      it = g_plans.erase(it);  // descriptors intentionally not destroyed (see above)
    else
      ++it;
  }
  if (times) {
    times[0] = first_us;
    times[1] = best_us;
  }
  return best;
}

// Time EVERY solution the library has for this problem (getAllAlgos +
// matmulIsAlgoSupported), not only the heuristic's list: at mid M (256..2048)
// with N = 4096 the heuristic's solutions use 256x256 macro tiles that leave
// most CUs idle, and smaller-tile / split-K solutions it ranks low are what
// fills the chip.  Writes the `max_out` fastest (solution index, us) pairs,
// fastest first, and returns how many it wrote (< 0: error).  times[0] = the
// heuristic's first choice (us).  A tool / init-time call (not capturable).
// `nw` weight copies `w_stride` elements apart are rotated (cold weights, as
// the engine's per-layer calls see them).
K8S_API int k8s_blaslt_sweep(const void* x, int ldx, const void* w, int nw, size_t w_stride, void* y, int ldy, int M,
                             int N, int K, void* ws, size_t ws_bytes, int iters, hipStream_t s, int max_out,
                             int* out_idx, float* out_us, float* times) {
  if (M <= 0 || N <= 0 || K <= 0 || ldx < K || ldy < N || iters < 1 || max_out < 1 || nw < 1)
    return -(int)hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(g_mu);
  if (g_handle == nullptr && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return -900;
  const Key key{M, N, K, ldx, ldy, 0};
  Plan p;
  int rc = make_desc(key, &p);
  if (rc) return -rc;
  auto wk = [&](int r) { return (const void*)((const uint16_t*)w + (size_t)(r % nw) * w_stride); };
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  if (hipblaslt_ext::getAllAlgos(g_handle, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, HIPBLAS_OP_T, HIPBLAS_OP_N,
                                 HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F,
                                 all) != HIPBLAS_STATUS_SUCCESS)
    return -1600;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -901;
  const float alpha = 1.f, beta = 0.f;
  auto time_algo = [&](hipblasLtMatmulAlgo_t& algo, size_t wsz) -> float {
    for (int r = 0; r < 2; ++r)
      if (hipblasLtMatmul(g_handle, p.desc, &alpha, wk(r), p.a, x, p.b, &beta, y, p.c, y, p.c, &algo, ws, wsz, s) !=
          HIPBLAS_STATUS_SUCCESS)
        return -1.f;
    if (hipStreamSynchronize(s) != hipSuccess) return -1.f;
    hipEventRecord(e0, s);
    for (int r = 0; r < iters; ++r)
      hipblasLtMatmul(g_handle, p.desc, &alpha, wk(r), p.a, x, p.b, &beta, y, p.c, y, p.c, &algo, ws, wsz, s);
    hipEventRecord(e1, s);
    if (hipEventSynchronize(e1) != hipSuccess) return -1.f;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return 1000.f * ms / iters;
  };
  if (times) {
    hipblasLtMatmulHeuristicResult_t h[1];
    int n = 0;
    times[0] = heuristic(p, ws_bytes, 1, h, &n) == 0 ? time_algo(h[0].algo, h[0].workspaceSize) : -1.f;
  }
  std::vector<std::pair<float, int>> best;
  for (auto& r : all) {
    size_t wsz = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(g_handle, p.desc, &alpha, p.a, p.b, &beta, p.c, p.c, r.algo, wsz) !=
            HIPBLAS_STATUS_SUCCESS ||
        wsz > ws_bytes)
      continue;
    const float us = time_algo(r.algo, wsz);
    if (us > 0.f) best.emplace_back(us, hipblaslt_ext::getIndexFromAlgo(r.algo));
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  std::sort(best.begin(), best.end());
  const int n = std::min<int>(max_out, (int)best.size());
  for (int i = 0; i < n; ++i) {
    out_us[i] = best[i].first;
    out_idx[i] = best[i].second;
  }
  return n;
}

// Register solution `idx` (from k8s_blaslt_sweep, kept in a data file) for
// (N, K) from ladder point M up: plans built afterwards use it where the
// library confirms it supports the problem (build_plan), else the heuristic.
static int set_algo_range(int M, int hi, int N, int K, int idx) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_handle == nullptr && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return 900;
  std::vector<int> ids{idx};
  std::vector<hipblasLtMatmulHeuristicResult_t> res;
  if (hipblaslt_ext::getAlgosFromIndex(g_handle, ids, res) != HIPBLAS_STATUS_SUCCESS || res.empty()) return 1700;
  g_tuned[{N, K}][M] = Tuned{res[0].algo, hi};
  for (auto it = g_plans.begin(); it != g_plans.end();) {
    if (it->first.N == N && it->first.K == K)
      it = g_plans.erase(it);
    else
      ++it;
  }
  return 0;
}

// The heuristic's first-choice solution index for (M, N, K) (x / y dense,
// ldx = K, ldy = N): candidates for a neighbouring M's bucket
// (tools/blaslt_tune_buckets.py), where the heuristic's own pick misfires.
K8S_API int k8s_blaslt_heuristic_index(int M, int N, int K, size_t ws_bytes) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_handle == nullptr && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return -900;
  Plan p;
  if (make_desc(Key{M, N, K, K, N, 0}, &p)) return -1100;
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const int rc = heuristic(p, ws_bytes, 1, res, &n);
  const int idx = (rc || n < 1) ? -1200 : hipblaslt_ext::getIndexFromAlgo(res[0].algo);
  // a throw-away plan (no kernel was enqueued with it): release its descriptors
  hipblasLtMatrixLayoutDestroy(p.a);
  hipblasLtMatrixLayoutDestroy(p.b);
  hipblasLtMatrixLayoutDestroy(p.c);
  hipblasLtMatmulDescDestroy(p.desc);
  return idx;
}

K8S_API int k8s_blaslt_set_algo(int M, int N, int K, int idx) { return set_algo_range(M, 1 << 30, N, K, idx); }

// Bucketed form (tools/blaslt_tune_buckets.py): solution `idx` for M in [lo, hi]
// only; M outside every registered bucket keeps the heuristic's choice.
K8S_API int k8s_blaslt_set_algo_range(int lo, int hi, int N, int K, int idx) {
  return set_algo_range(lo, hi, N, K, idx);
}

K8S_API void k8s_blaslt_clear_tuning() {
  std::lock_guard<std::mutex> g(g_mu);
  g_tuned.clear();
  g_plans.clear();
}
