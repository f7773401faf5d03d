// Native layer executor for the dense Llama decoder (TP = 1, and TP > 1 with
// the xGMI all-reduce: the two row-parallel outputs of every layer -- o_proj
// and down_proj -- are summed across the TP ranks in place by
// k8s_ar_allreduce_bf16 right after their GEMM, before the residual add +
// RMSNorm that consumes them; HIP-graph capturable like the rest).
//
// An eager engine step (prefill chunks mixed with decode rows: shapes change
// every step, so it cannot replay a HIP graph) issues ~10 kernels per layer.
// Issued op by op from Python each costs ~15-20 us of host time (wrapper
// checks, ctypes marshalling, torch dispatch), ~6 ms for an 8B step: about
// the GPU time of a small mixed step, so the host, not the GPU, set the pace
// and the GPU idled between steps (tools/trace_gaps.py: "last GEMM ->
// next step's upload" gaps).  Here the whole layer stack is issued by one
// call from a per-step descriptor (pointers + sizes + the GEMM kernel chosen
// for this step's M by the measured dispatch table), in exactly the order
// and with exactly the kernels of the Python path (models/llama.py), so the
// results are bit-identical; per-layer weight / KV pointers come from tables
// built once at model init.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>

#include <cstdio>

#include "common.h"

// the kernels' C entry points (other translation units of this library)
extern "C" {
int k8s_rmsnorm(const void* x, void* res, const void* w, void* y, int T, int H, int x_stride, int y_stride, float eps,
                hipStream_t s);
int k8s_splitk_addnorm(const void* part, int splits, void* res, const void* w, void* y, int T, int H, int y_stride,
                       float eps, hipStream_t s);
int k8s_silu_mul(const void* gu, void* out, int T, int I, hipStream_t s);
int k8s_rope_kv(void* qkv, int ld, const int* pos, const float* cos_sin, const int* slots, void* kc, void* vc, int T,
                int nq, int nkv, int BS, hipStream_t s);
int k8s_splitk_rope_kv(const void* part, int splits, void* qkv, int ld, const int* pos, const float* cos_sin,
                       const int* slots, void* kc, void* vc, int T, int nq, int nkv, int BS, hipStream_t s);
int k8s_attn_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                    int bt_stride, const int* ctx_lens, const int* q_start, int S, int nq, int nkv, int BS,
                    float scale, void* out, int out_stride, float* part_o, float* part_ml, int n_parts,
                    int part_size, const int* items, int n_items, const int* d_n_items, int grid_waves,
                    hipStream_t stream);
int k8s_attn_prefill(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                     int bt_stride, const int* ctx_lens, const int* q_start, const int* tile_seq,
                     const int* tile_tok0, const int* tile_len, const int* tile_kv0, const int* tile_kv1,
                     const int* tile_slot, int n_tiles, const int* m_tok0, const int* m_len, const int* m_slot0,
                     const int* m_np, int n_merge, float* pf_o, float* pf_ml, int nq, int nkv, int BS, float scale,
                     void* out, int out_stride, hipStream_t stream);
int k8s_gemm_skinny(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, hipStream_t s);
int k8s_gemm_skinny_rope(const void* x, int ldx, const void* w, void* qkv, int ldq, int M, int N, int K,
                         const int* pos, const float* cos_sin, const int* slots, void* kc, void* vc, int nq, int nkv,
                         int BS, hipStream_t s);
int k8s_gemm_mid(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg, int splits,
                 void* part, hipStream_t s);
int k8s_gemm_mid_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                      int splits, void* part, hipStream_t s);
int k8s_grouped_gemm(const void* a, int lda, const void* w, void* y, int ldy, const int* offsets, int E, int N,
                     int K, int max_tiles, int fuse_silu, int splits, void* part, int total_rows, hipStream_t s);
int k8s_grouped_gemm_part(const void* a, int lda, const void* w, void* y, int ldy, const int* offsets, int E, int N,
                          int K, int max_tiles, int fuse_silu, int splits, void* part, int total_rows, hipStream_t s);
int k8s_blaslt_gemm(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, void* ws,
                    size_t ws_bytes, hipStream_t s);
int k8s_ar_allreduce_bf16(int id, const void* in, void* out, long n, int mode, hipStream_t s);
int k8s_ar_addnorm_bf16(int id, const void* in, void* res, const void* w, void* y, int T, int H, float eps, int mode,
                        hipStream_t s);
int k8s_gemm_stream(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg, int splits,
                    void* part, hipStream_t s);
int k8s_gemm_stream_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                         int splits, void* part, hipStream_t s);
int k8s_gemm_big(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int mode, int pipe,
                 hipStream_t s);
int k8s_gemm_big_split(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int var, int splits,
                       void* part, hipStream_t s);
int k8s_gemm_big_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int var, int splits,
                      void* part, hipStream_t s);
int k8s_gemm_big_rope(const void* x, int ldx, const void* w, void* qkv, int ldq, int M, int N, int K, const int* pos,
                      const float* cos_sin, const int* slots, void* kc, void* vc, int nq, int nkv, int BS, int var,
                      hipStream_t s);
int k8s_gemm_stream_silu(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                         hipStream_t s);
int k8s_gemm_stream_push(const void* x, int ldx, const void* w, int M, int N, int K, int cfg, int splits, void* part,
                         int ar_id, int mode, hipStream_t s);
int k8s_ar_push_addnorm_bf16(int id, void* res, const void* w, void* y, int T, int H, float eps, int mode, int S,
                             hipStream_t s);
int k8s_nonfinite_flag(const void* x, long n, int* flag, hipStream_t s);
int k8s_gemm_skinny_rope_norm(const void* x, int x_stride, const float* part, int splits, const void* res_in,
                              void* res_out, const void* norm_w, float eps, const void* w, void* qkv, int ldq, int M,
                              int N, int K, const int* pos, const float* cos_sin, const int* slots, void* kc, void* vc,
                              int nq, int nkv, int BS, hipStream_t s);
int k8s_gemm_stream_silu_norm(const void* x, int x_stride, const float* part, int splits, const void* res_in,
                              void* res_out, const void* norm_w, float eps, const void* w, void* y, int ldy, int M,
                              int N, int K, int cfg, hipStream_t s);
}

// kind: 0 hipBLASLt, 1 skinny, 2 gemm_mid (cfg, splits), 3 single-expert grouped (splits),
// 4 gemm_stream (cfg = ring depth, splits), 5 gemm_big (cfg = schedule variant, splits);
// fuse: 1 -- a split-K o / down projection may leave its partials to the next norm;
// 2 (gate_up, kinds 4 / 5 with one K split) -- the SwiGLU-epilogue form, which
// writes act directly (gu is never written, no silu_mul launch);
// 3 (qkv, kind 1) -- the skinny kernel's RoPE / KV-write epilogue (no rope_kv launch);
// 4 (qkv, kind 5) -- gemm_big's RoPE / KV-write epilogue (prefill sizes)
struct K8sGemmSel {
  int kind, cfg, splits, fuse;
};

// Mirrors k8s_llm_rca_amd/ops/layer_exec.py:LlamaStep (ctypes, natural alignment).
struct K8sLlamaStep {
  int T, nd, H, nq, nkv, I, L, BS;
  float eps, scale;
  // per-layer tables (host arrays of L pointers)
  const void* const* in_norm;
  const void* const* post_norm;
  const void* const* wqkv;
  const void* const* wo;
  const void* const* wgu;
  const void* const* wdown;
  void* const* kc;
  void* const* vc;
  // activations (row-major, contiguous)
  void* residual;  // [T][H], updated in place
  void* y;         // [T][H]
  void* qkv;       // [T][(nq + 2 nkv) D]
  void* attn;      // [T][nq D]
  void* obuf;      // [T][H]
  void* gu;        // [T][2 I]
  void* act;       // [T][I]
  void* prev;      // [T][H]  (down output of the last layer on return)
  const int* pos;
  const float* cos_sin;
  const int* slots;
  // decode meta (rows [0, nd))
  const int* d_bt;
  const int* d_ctx;
  const int* d_qs;
  float* d_part_o;
  float* d_part_ml;
  const int* d_items;
  const int* d_n_items_dev;
  int d_bt_stride, d_S, d_n_parts, d_part_size, d_n_items, d_grid;
  // prefill meta (rows [nd, T))
  const int* p_bt;
  const int* p_ctx;
  const int* p_qs;
  const int* tile[6];
  const int* merge[4];
  float* pf_o;
  float* pf_ml;
  int p_bt_stride, p_S, n_tiles, n_merge;
  // GEMM choices for this step's M = T: qkv, o, gate_up, down
  K8sGemmSel sel[4];
  void* blaslt_ws;
  size_t blaslt_ws_bytes;
  void* mid_part;
  void* grp_part;
  const int* grp_offs;  // device [0, T]
  // TP: xGMI all-reduce communicator id (-1: TP = 1) and mode (1 one-shot, 2 two-shot);
  // ar_fuse: the all-reduce + residual add + RMSNorm of each row-parallel output in
  // one launch (k8s_ar_addnorm_bf16) instead of all-reduce, then rmsnorm
  int ar_id, ar_mode, ar_fuse;
  // ar_push (with ar_fuse): o / down projections whose choice is the stream GEMM
  // (LDS-DMA cfg, or split-K) store their output straight into the peers'
  // all-reduce slots (k8s_gemm_stream_push) and the fused epilogue waits on
  // per-strip flags (k8s_ar_push_addnorm_bf16): no staging copy
  int ar_push;
  // debug (knob nonfinite_check): nf_flags[l] = 1 when layer l's normed input
  // holds a NaN / inf, nf_flags[L] for the last down output; nullptr = off
  int* nf_flags;
  // norm_fuse (TP = 1, T <= 4; ops/layer_exec.py decides): bit 0 -- the input norm
  // rides in the skinny RoPE qkv GEMM's prologue, bit 1 -- the post-attention norm
  // in the SwiGLU stream gate_up GEMM's (norm_prologue.h).  A fused add-norm
  // writes the new residual to the OTHER of {residual, res2} (its workgroups are
  // still reading the current one), so the current residual alternates.
  void* res2;
  int norm_fuse;
};

namespace {

constexpr int kD = 128;

// A split-K choice (kinds 2 and 3, splits > 1) with `defer` leaves its fp32
// partials in the kind's scratch for the following norm to reduce
// (k8s_splitk_addnorm); deferred() tells the caller where they are.
bool deferred(const K8sGemmSel& g, bool defer) {
  return defer && g.fuse && g.splits > 1 && (g.kind == 2 || g.kind == 3 || g.kind == 4 || g.kind == 5);
}

const void* part_of(const K8sLlamaStep& s, const K8sGemmSel& g) {
  return (g.kind == 2 || g.kind == 4 || g.kind == 5) ? s.mid_part : s.grp_part;
}

int gemm(const K8sLlamaStep& s, const K8sGemmSel& g, const void* x, int ldx, const void* w, void* y, int ldy, int M,
         int N, int K, hipStream_t st, bool defer = false) {
  const bool d = deferred(g, defer);
  switch (g.kind) {
    case 1:
      return k8s_gemm_skinny(x, ldx, w, y, ldy, M, N, K, st);
    case 2:
      return (d ? k8s_gemm_mid_part : k8s_gemm_mid)(x, ldx, w, y, ldy, M, N, K, g.cfg, g.splits, s.mid_part, st);
    case 3:
      return (d ? k8s_grouped_gemm_part : k8s_grouped_gemm)(x, ldx, w, y, ldy, s.grp_offs, 1, N, K,
                                                            (M + 63) / 64 + 1, 0, g.splits, s.grp_part, M, st);
    case 4:
      return (d ? k8s_gemm_stream_part : k8s_gemm_stream)(x, ldx, w, y, ldy, M, N, K, g.cfg, g.splits, s.mid_part,
                                                          st);
    case 5:
      if (g.splits > 1)
        return (d ? k8s_gemm_big_part : k8s_gemm_big_split)(x, ldx, w, y, ldy, M, N, K, g.cfg, g.splits, s.mid_part,
                                                            st);
      return k8s_gemm_big(x, ldx, w, y, ldy, M, N, K, 0, g.cfg, st);
    default:
      return k8s_blaslt_gemm(x, ldx, w, y, ldy, M, N, K, s.blaslt_ws, s.blaslt_ws_bytes, st);
  }
}

// the push epilogue exists on the stream GEMM's LDS-DMA configurations and on
// its split-K reduce pass
bool push_kind(const K8sGemmSel& g) { return g.kind == 4 && (g.cfg >= 13 || g.splits > 1); }

}  // namespace

// a failing op names itself (the step's rc alone does not say which of ~10 per layer it was)
#define K8S_TRY(call)                                                                                     \
  do {                                                                                                    \
    const int rc_ = (call);                                                                               \
    if (rc_) {                                                                                            \
      fprintf(stderr, "k8s_llama_layers: llama_exec.hip:%d failed with %d (T=%d nd=%d sel kinds %d %d %d %d)\n", \
              __LINE__, rc_, s.T, s.nd, s.sel[0].kind, s.sel[1].kind, s.sel[2].kind, s.sel[3].kind);      \
      return rc_;                                                                                         \
    }                                                                                                     \
  } while (0)

// Layers [0, L): on return `y` holds nothing useful and `prev` + `residual`
// are the inputs of the final norm (exactly as after the Python loop).
// Where the step's dispatch picked a split-K kernel for the o or down
// projection, its partials are reduced inside the following residual-add +
// RMSNorm (k8s_splitk_addnorm), and a split-K qkv projection's inside the
// RoPE / KV-write kernel (k8s_splitk_rope_kv): bit-identical, one launch fewer
// per GEMM.
K8S_API int k8s_llama_layers(const K8sLlamaStep* sp, hipStream_t st) {
  const K8sLlamaStep& s = *sp;
  const int T = s.T, H = s.H, nd = s.nd;
  const int qd = s.nq * kD, ld_qkv = (s.nq + 2 * s.nkv) * kD;
  uint16_t* qkv = (uint16_t*)s.qkv;
  uint16_t* attn = (uint16_t*)s.attn;
  bool pend = false;  // the previous layer's down projection is still split-K partials
  const bool tp = s.ar_id >= 0;  // row-parallel outputs are partial sums: all-reduce, never defer split-K
  const bool fuse_an = tp && s.ar_fuse;  // the previous layer's down all-reduce already produced y
  const bool push_o = fuse_an && s.ar_push && push_kind(s.sel[1]);
  const bool push_d = fuse_an && s.ar_push && push_kind(s.sel[3]);
  const long n_out = (long)T * H;
  // current / other residual buffer (norm_fuse ping-pong, see K8sLlamaStep)
  void* rc = s.residual;
  void* ro = s.res2;
  const bool nf_qkv = !tp && (s.norm_fuse & 1) && s.sel[0].kind == 1 && s.sel[0].fuse == 3;
  const bool nf_gu = !tp && (s.norm_fuse & 2) && s.sel[2].kind == 4 && s.sel[2].fuse == 2;
  for (int l = 0; l < s.L; ++l) {
    if (nf_qkv) {  // input norm + qkv GEMM + RoPE / KV write in one launch
      const bool first = l == 0;
      const float* part = pend ? (const float*)part_of(s, s.sel[3]) : nullptr;
      K8S_TRY(k8s_gemm_skinny_rope_norm(first ? rc : (pend ? nullptr : s.prev), H, part, s.sel[3].splits,
                                        first ? nullptr : rc, first ? nullptr : ro, s.in_norm[l], s.eps, s.wqkv[l],
                                        qkv, ld_qkv, T, ld_qkv, H, s.pos, s.cos_sin, s.slots, s.kc[l], s.vc[l], s.nq,
                                        s.nkv, s.BS, st));
      if (!first) {
        void* t = rc;
        rc = ro;
        ro = t;
      }
    } else if (l == 0)
      K8S_TRY(k8s_rmsnorm(rc, nullptr, s.in_norm[l], s.y, T, H, H, H, s.eps, st));
    else if (fuse_an) {
      // y = rmsnorm(all-reduced down_proj + residual): done by the previous layer's fused epilogue
    } else if (pend)
      K8S_TRY(k8s_splitk_addnorm(part_of(s, s.sel[3]), s.sel[3].splits, rc, s.in_norm[l], s.y, T, H, H, s.eps, st));
    else
      K8S_TRY(k8s_rmsnorm(s.prev, rc, s.in_norm[l], s.y, T, H, H, H, s.eps, st));
    if (s.nf_flags && !nf_qkv) K8S_TRY(k8s_nonfinite_flag(s.y, n_out, s.nf_flags + l, st));
    // a split-K qkv projection leaves its partials to the RoPE / KV-write kernel,
    // which reduces them first (k8s_splitk_rope_kv: bit-identical, one launch fewer)
    if (nf_qkv) {
      // done above
    } else if (deferred(s.sel[0], true)) {
      K8S_TRY(gemm(s, s.sel[0], s.y, H, s.wqkv[l], qkv, ld_qkv, T, ld_qkv, H, st, true));
      K8S_TRY(k8s_splitk_rope_kv(part_of(s, s.sel[0]), s.sel[0].splits, qkv, ld_qkv, s.pos, s.cos_sin, s.slots,
                                 s.kc[l], s.vc[l], T, s.nq, s.nkv, s.BS, st));
    } else if (s.sel[0].kind == 5 && s.sel[0].fuse == 4) {  // prefill-size qkv, RoPE / KV write in the epilogue
      K8S_TRY(k8s_gemm_big_rope(s.y, H, s.wqkv[l], qkv, ld_qkv, T, ld_qkv, H, s.pos, s.cos_sin, s.slots, s.kc[l],
                                s.vc[l], s.nq, s.nkv, s.BS, s.sel[0].cfg, st));
    } else if (s.sel[0].kind == 1 && s.sel[0].fuse == 3) {  // skinny qkv with the RoPE / KV-write epilogue
      K8S_TRY(k8s_gemm_skinny_rope(s.y, H, s.wqkv[l], qkv, ld_qkv, T, ld_qkv, H, s.pos, s.cos_sin, s.slots, s.kc[l],
                                   s.vc[l], s.nq, s.nkv, s.BS, st));
    } else {
      K8S_TRY(gemm(s, s.sel[0], s.y, H, s.wqkv[l], qkv, ld_qkv, T, ld_qkv, H, st));
      K8S_TRY(k8s_rope_kv(qkv, ld_qkv, s.pos, s.cos_sin, s.slots, s.kc[l], s.vc[l], T, s.nq, s.nkv, s.BS, st));
    }
    const bool dec = nd > 0 && s.d_bt, pre = nd < T && s.p_bt;
    if (pre)
      K8S_TRY(k8s_attn_prefill(qkv + (size_t)nd * ld_qkv, ld_qkv, s.kc[l], s.vc[l], s.p_bt, s.p_bt_stride, s.p_ctx,
                               s.p_qs, s.tile[0], s.tile[1], s.tile[2], s.tile[3], s.tile[4], s.tile[5], s.n_tiles,
                               s.merge[0], s.merge[1], s.merge[2], s.merge[3], s.n_merge, s.pf_o, s.pf_ml, s.nq,
                               s.nkv, s.BS, s.scale, attn + (size_t)nd * qd, qd, st));
    if (dec)
      K8S_TRY(k8s_attn_decode(qkv, ld_qkv, s.kc[l], s.vc[l], s.d_bt, s.d_bt_stride, s.d_ctx, s.d_qs, s.d_S, s.nq,
                              s.nkv, s.BS, s.scale, attn, qd, s.d_part_o, s.d_part_ml, s.d_n_parts, s.d_part_size,
                              s.d_items, s.d_n_items, s.d_n_items_dev, s.d_grid, st));
    if (push_o) {
      K8S_TRY(k8s_gemm_stream_push(attn, qd, s.wo[l], T, H, qd, s.sel[1].cfg, s.sel[1].splits, s.mid_part, s.ar_id,
                                   s.ar_mode, st));
      K8S_TRY(k8s_ar_push_addnorm_bf16(s.ar_id, s.residual, s.post_norm[l], s.y, T, H, s.eps, s.ar_mode,
                                       k8s::k8s_push_strips(s.sel[1].cfg, s.sel[1].splits, H), st));
    } else {
      K8S_TRY(gemm(s, s.sel[1], attn, qd, s.wo[l], s.obuf, H, T, H, qd, st, !tp));
    }
    if (push_o) {
      // all-reduce + residual add + post-attention norm done above
    } else if (fuse_an)
      K8S_TRY(k8s_ar_addnorm_bf16(s.ar_id, s.obuf, s.residual, s.post_norm[l], s.y, T, H, s.eps, s.ar_mode, st));
    else if (tp)
      K8S_TRY(k8s_ar_allreduce_bf16(s.ar_id, s.obuf, s.obuf, n_out, s.ar_mode, st));
    if (nf_gu) {  // post-attention norm + gate_up + SwiGLU in one launch
      const bool dp = deferred(s.sel[1], true);
      K8S_TRY(k8s_gemm_stream_silu_norm(dp ? nullptr : s.obuf, H, dp ? (const float*)part_of(s, s.sel[1]) : nullptr,
                                        s.sel[1].splits, rc, ro, s.post_norm[l], s.eps, s.wgu[l], s.act, s.I, T, s.I,
                                        H, s.sel[2].cfg, st));
      void* t = rc;
      rc = ro;
      ro = t;
    } else if (fuse_an) {
      // residual add + post-attention norm done above
    } else if (!tp && deferred(s.sel[1], true))
      K8S_TRY(k8s_splitk_addnorm(part_of(s, s.sel[1]), s.sel[1].splits, rc, s.post_norm[l], s.y, T, H, H, s.eps, st));
    else
      K8S_TRY(k8s_rmsnorm(s.obuf, rc, s.post_norm[l], s.y, T, H, H, H, s.eps, st));
    if (nf_gu) {
      // gate_up done above
    } else if (s.sel[2].fuse == 2 && s.sel[2].kind == 5) {  // gate_up + SwiGLU in one launch: gu is never written
      K8S_TRY(k8s_gemm_big(s.y, H, s.wgu[l], s.act, s.I, T, s.I, H, 1, s.sel[2].cfg, st));
    } else if (s.sel[2].fuse == 2 && s.sel[2].kind == 4) {
      K8S_TRY(k8s_gemm_stream_silu(s.y, H, s.wgu[l], s.act, s.I, T, s.I, H, s.sel[2].cfg, st));
    } else {
      K8S_TRY(gemm(s, s.sel[2], s.y, H, s.wgu[l], s.gu, 2 * s.I, T, 2 * s.I, H, st));
      K8S_TRY(k8s_silu_mul(s.gu, s.act, T, s.I, st));
    }
    // the last layer's down output is returned (`prev`) for the final norm
    pend = !tp && deferred(s.sel[3], l + 1 < s.L);
    if (push_d && l + 1 < s.L) {  // the next layer's input norm rides on this all-reduce
      K8S_TRY(k8s_gemm_stream_push(s.act, s.I, s.wdown[l], T, H, s.I, s.sel[3].cfg, s.sel[3].splits, s.mid_part,
                                   s.ar_id, s.ar_mode, st));
      K8S_TRY(k8s_ar_push_addnorm_bf16(s.ar_id, s.residual, s.in_norm[l + 1], s.y, T, H, s.eps, s.ar_mode,
                                       k8s::k8s_push_strips(s.sel[3].cfg, s.sel[3].splits, H), st));
      continue;
    }
    K8S_TRY(gemm(s, s.sel[3], s.act, s.I, s.wdown[l], s.prev, H, T, H, s.I, st, !tp && l + 1 < s.L));
    if (fuse_an && l + 1 < s.L)  // the next layer's input norm rides on this all-reduce
      K8S_TRY(k8s_ar_addnorm_bf16(s.ar_id, s.prev, s.residual, s.in_norm[l + 1], s.y, T, H, s.eps, s.ar_mode, st));
    else if (tp)
      K8S_TRY(k8s_ar_allreduce_bf16(s.ar_id, s.prev, s.prev, n_out, s.ar_mode, st));
  }
  if (s.nf_flags && !pend) K8S_TRY(k8s_nonfinite_flag(s.prev, n_out, s.nf_flags + s.L, st));
  return (int)hipGetLastError();
}

K8S_API int k8s_llama_step_size() { return (int)sizeof(K8sLlamaStep); }
