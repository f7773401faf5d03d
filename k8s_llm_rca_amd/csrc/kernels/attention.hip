// Paged GQA attention for gfx950 (B6 prefill / B7 decode in SURVEY.md §2 Part B).
//
// KV cache layout (per layer), page = BS tokens (BS % 32 == 0):
//   K : [num_blocks][n_kv][BS][128]   row-major keys
//   V : [num_blocks][n_kv][128][BS]   TRANSPOSED per page, so the PV MFMA's
//                                      B operand (8 consecutive keys of one
//                                      d-column) is one 16-byte load.
//
// One wave computes 16 "rows" = (token, q-head) pairs that share a kv head,
// against 32-key chunks, with v_mfma_f32_16x16x32_bf16:
//   * swapped QK^T: S^T = K . Q^T (A = K rows, B = Q^T) so each lane owns ONE
//     query row (lane & 15) and 8 of its key scores -> the online-softmax max
//     is 7 in-lane fmax + 2 shuffles; the row sum stays lane-local until the end.
//   * key permutation: MFMA row rho of key tile t holds key 8*(rho>>2)+4t+(rho&3),
//     so lane half h ends up with keys 8h..8h+7 -- exactly the k-slots 8h+j of
//     the PV MFMA's A operand: P goes from the S accumulator to the PV operand
//     with one bf16 pack and no lane movement.
//   * the 128-wide head dim is split over the 4 MFMA k-steps as dims
//     32c+8h+j: every Q/K fragment is a contiguous 16-byte load and the 4 lanes
//     holding one key read 64 contiguous bytes per instruction (16 half lines
//     per wave instruction instead of 32 scattered pieces).
// Decode (one token / seq): each WAVE owns one (seq, kv head, key partition)
// and streams its pages 64 keys at a time (32 x 16-byte loads in flight per
// lane group before the first MFMA); partitions are merged by attn_reduce
// (flash-decoding split-KV).  No LDS, no barriers.  Prefill / extend (varlen, causal,
// cached prefix): workgroup = (tile of 64/G tokens, kv head); each wave owns 16
// rows and walks the keys its rows can see.
#include <cstdlib>
#include <utility>

#include "common.h"
#include "knobs.h"

namespace k8s {

constexpr int D = 128;
constexpr int ROWS = 16;  // rows per wave
constexpr int CH = 32;    // keys per chunk
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const uint16_t* q;      // [T][q_stride] ; head h at +h*128
  int q_stride;           // elements between consecutive tokens
  const uint16_t* kc;     // K cache
  const uint16_t* vc;     // V cache (transposed pages)
  const int* block_tables;
  int bt_stride;
  const int* ctx_lens;    // [S] total KV length (cached + new)
  const int* q_start;     // [S+1] first q row of each sequence
  int nq, nkv, G, BS;
  float scale_log2;       // softmax scale * log2(e)
  uint16_t* out;          // [T][out_stride]
  int out_stride;
  // decode split-KV
  float* part_o;          // [S][nq][n_parts][128]
  float* part_ml;         // [S][nq][n_parts][2]
  int n_parts, part_size;
  // prefill tiles
  const int* tile_seq;    // [n_tiles]
  const int* tile_tok0;   // [n_tiles] q row of the tile's first token
  const int* tile_len;    // [n_tiles] tokens in the tile
  // prefill split-KV (paged-64 kernel): page range + partial slot per tile
  const int* tile_kv0;    // [n_tiles] first page
  const int* tile_kv1;    // [n_tiles] end page (exclusive, clamped to the causal end)
  const int* tile_slot;   // [n_tiles] -1: write the final rows; else partial slot
  float* pf_o;            // [slots][nkv][128 rows][128] unnormalised partial O
  float* pf_ml;           // [slots][nkv][128 rows][2]   (max, sum) in log2 domain
  const int* m_tok0;      // merge list: q row of the split tile's first token
  const int* m_len;       //   tokens
  const int* m_slot0;     //   first slot; its parts are slot0 .. slot0+np-1
  const int* m_np;
  // decode work list (persistent kernel): int4 (seq, part | -1 = whole row, k1, qrow)
  const int4* items;
  int n_items;
  const int* d_n_items;   // device {item count, part_size} (HIP graphs: the grid stays fixed), or null
  int pf_rows;            // rows per prefill partial slot (128: pg64 kernel, 256: w8 kernel)
  int pf_bf16;            // partials are bf16 O / l (w8 VAR 4) instead of fp32 unnormalised O
};

struct RowState {
  bf16x8 qf[4];
  f32x4 o[8];
  float m;      // running max (log2 domain) of this lane's row
  float l;      // lane-partial row sum
};

__device__ __forceinline__ bf16x8 load16(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
// the decode KV stream's loads: default policy, or non-temporal (NT, knob
// decode_kv_nt) -- MI355X_MICROARCH.md measures nt weight streams at 6.5-6.8
// TB/s against 6.4 with the default policy
template <bool NT>
__device__ __forceinline__ bf16x8 load16k(const uint16_t* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
  else
    return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.0f;
  return z;
}

// Process NSUB consecutive 32-key sub-chunks starting at absolute key `kb`
// (kb % 32 == 0, all inside one page) with ONE online-softmax update.
// All K/V loads of the group are issued before the first MFMA so a wave keeps
// NSUB*16 KB in flight.  `limit` = keys < limit are visible to this lane's row.
template <int NSUB>
__device__ __forceinline__ void chunk(RowState& st, const AttnArgs& a, const int* bt, int kvh, int kb, int limit,
                                      int lane) {
  const int r = lane & 15, h = lane >> 4;
  const int blk = bt[kb / a.BS];
  const int off = kb % a.BS;
  const size_t page = ((size_t)blk * a.nkv + kvh);
  const uint16_t* kp = a.kc + page * (size_t)a.BS * D;
  const uint16_t* vp = a.vc + page * (size_t)D * a.BS;
  // K fragments: sub-chunk u, tile t, row r -> key 32u + 8*(r>>2) + 4t + (r&3); dims 32c+8h..+8
  bf16x8 kf[NSUB][2][4];
#pragma unroll
  for (int u = 0; u < NSUB; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = off + 32 * u + 8 * (r >> 2) + 4 * t + (r & 3);
#pragma unroll
      for (int c = 0; c < 4; ++c) kf[u][t][c] = load16(kp + (size_t)key * D + 32 * c + 8 * h);
    }
  // V fragments: column d = 16*dt + r, keys off + 32u + 8h .. +8 (transposed page)
  bf16x8 vf[NSUB][8];
#pragma unroll
  for (int u = 0; u < NSUB; ++u)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) vf[u][dt] = load16(vp + (size_t)(16 * dt + r) * a.BS + off + 32 * u + 8 * h);

  float p[NSUB][8];
  float cmax = -INFINITY;
#pragma unroll
  for (int u = 0; u < NSUB; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[u][t][c], st.qf[c], s, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kb + 32 * u + 8 * h + 4 * t + i;
        const float v = (key < limit) ? s[i] * a.scale_log2 : -INFINITY;
        p[u][4 * t + i] = v;
        cmax = fmaxf(cmax, v);
      }
    }
  cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
  cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
  const float mnew = fmaxf(st.m, cmax);
  const float alpha = (mnew == -INFINITY) ? 1.f : exp2f(st.m - mnew);
  float psum = 0.f;
  bf16x8 pf[NSUB];
#pragma unroll
  for (int u = 0; u < NSUB; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float e = (mnew == -INFINITY) ? 0.f : exp2f(p[u][j] - mnew);
      psum += e;
      pf[u][j] = (__bf16)e;
    }
  st.l = st.l * alpha + psum;
  st.m = mnew;
  // O rows 4h+i need the alpha of row 4h+i (owned by lane 4h+i)
  float ar[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) ar[i] = __shfl(alpha, 4 * h + i, 64);
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) st.o[dt][i] *= ar[i];
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
      st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[u], vf[u][dt], st.o[dt], 0, 0, 0);
  }
}

__device__ __forceinline__ void init_state(RowState& st, const AttnArgs& a, int qrow, int head, bool valid, int lane) {
  const int h = lane >> 4;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    st.qf[c] = valid ? load16(a.q + (size_t)qrow * a.q_stride + head * D + 32 * c + 8 * h) : zero8();
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) st.o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  st.m = -INFINITY;
  st.l = 0.f;
}

// ---------------------------------------------------------------- decode
// Software-pipelined 64-key stream for paged caches with BS % 64 == 0 (every
// 64-key chunk inside one page).  K registers are refilled with chunk c+1
// right after chunk c's QK^T and V registers right after its PV, so a wave
// always has the next chunk's 16-32 KB in flight while it computes (a plain
// load -> wait -> compute loop leaves the wave's memory pipe idle during
// compute and decode is bound by bytes in flight per CU).
template <bool NT>
__device__ __forceinline__ void dec_load_k(bf16x8 (&kf)[2][2][4], const AttnArgs& a, int blk, int kvh, int kb,
                                           int lane) {
  const int r = lane & 15, h = lane >> 4;
  const size_t page = (size_t)blk * a.nkv + kvh;
  const uint16_t* kp = a.kc + page * (size_t)a.BS * D;
  const int off = kb % a.BS;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = off + 32 * u + 8 * (r >> 2) + 4 * t + (r & 3);
#pragma unroll
      for (int c = 0; c < 4; ++c) kf[u][t][c] = load16k<NT>(kp + (size_t)key * D + 32 * c + 8 * h);
    }
}

template <bool NT>
__device__ __forceinline__ void dec_load_v(bf16x8 (&vf)[2][8], const AttnArgs& a, int blk, int kvh, int kb,
                                           int lane) {
  const int r = lane & 15, h = lane >> 4;
  const size_t page = (size_t)blk * a.nkv + kvh;
  const uint16_t* vp = a.vc + page * (size_t)D * a.BS;
  const int off = kb % a.BS;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) vf[u][dt] = load16k<NT>(vp + (size_t)(16 * dt + r) * a.BS + off + 32 * u + 8 * h);
}

// `blkv`: lane j holds the block id of the partition's j-th page (fetched
// once per work item: a per-chunk block-table load would put a dependent
// memory latency in front of every chunk's K/V loads).
// `k1`: end key of the item (wave-uniform); `lim`: this lane's row sees keys
// < lim (== k1 except for the earlier tokens of a multi-token item);
// `kmin`: the smallest row limit of the wave (tail masking starts there).
template <bool NT>
__device__ __forceinline__ void decode_stream64(RowState& st, const AttnArgs& a, int blkv, int kvh, int k0,
                                                int k1, int kmin, int lim, int lane) {
  const int h = lane >> 4;
  const int nch = (k1 - k0 + 63) >> 6;
  const int pg0 = k0 / a.BS;
  bf16x8 kf[2][2][4], vf[2][8];
  {
    const int b0 = __builtin_amdgcn_readfirstlane(blkv);
    dec_load_k<NT>(kf, a, b0, kvh, k0, lane);
    dec_load_v<NT>(vf, a, b0, kvh, k0, lane);
  }
  for (int c = 0; c < nch; ++c) {
    const int kb = k0 + 64 * c;
    const int kbn = k0 + 64 * min(c + 1, nch - 1);  // unconditional prefetch (last one re-reads)
    const int bn = __builtin_amdgcn_readlane(blkv, kbn / a.BS - pg0);
    f32x4 sc[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[u][t][q], st.qf[q], acc, 0, 0, 0);
        sc[u][t] = acc;
      }
    dec_load_k<NT>(kf, a, bn, kvh, kbn, lane);
    float cmax = -INFINITY;
    if (kb + 64 > kmin) {  // tail chunk: keys >= the row's limit are not visible to it
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (kb + 32 * u + 8 * h + 4 * t + i >= lim) sc[u][t][i] = -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) cmax = fmaxf(cmax, sc[u][t][i]);
    cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
    // deferred max (see the prefill kernel): P <= 2^8
    const float mcand = cmax * a.scale_log2;
    const bool upd = mcand > st.m + 8.f;
    const float mnew = upd ? mcand : st.m;
    const float alpha = upd ? __builtin_amdgcn_exp2f(st.m - mnew) : 1.f;
    const float nmsub = (mnew == -INFINITY) ? 0.f : -mnew;
    bf16x8 pf[2];
    float psum = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(fmaf(sc[u][t][i], a.scale_log2, nmsub));
          psum += e;
          pf[u][4 * t + i] = (__bf16)e;
        }
    st.l = st.l * alpha + psum;
    st.m = mnew;
    if (__ballot(upd)) {
      float ar[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) ar[i] = __shfl(alpha, 4 * h + i, 64);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) st.o[dt][i] *= ar[i];
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int u = 0; u < 2; ++u) st.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[u], vf[u][dt], st.o[dt], 0, 0, 0);
    dec_load_v<NT>(vf, a, bn, kvh, kbn, lane);
  }
}

// grid: S * nkv * n_parts one-wave workgroups.  Each wave owns one
// (seq, kv head, key partition of `part_size` keys) item of a FLAT item list:
// decode is bound by per-CU load throughput, so waves (not 4-wave groups with
// idle members) are what the dispatcher must spread evenly over the CUs.  No LDS, no barriers; a wave writes an
// unnormalised partial (O, m, l) merged by attn_reduce, or the final bf16 row
// when n_parts == 1.
__global__ void __launch_bounds__(64, 2) attn_decode_kernel(AttnArgs a, int S) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x;
  const int part = item % a.n_parts, kvh = (item / a.n_parts) % a.nkv, seq = item / (a.n_parts * a.nkv);
  if (seq >= S) return;
  const int r = lane & 15, h = lane >> 4;
  const int ctx = a.ctx_lens[seq];
  const int k0 = part * a.part_size;
  if (part >= a.n_parts || k0 >= ctx) return;  // wave-uniform exit
  const int k1 = min(ctx, k0 + a.part_size);
  const int qrow = a.q_start[seq];
  const bool valid = r < a.G;
  const int head = kvh * a.G + (valid ? r : 0);
  const int* bt = a.block_tables + (size_t)seq * a.bt_stride;

  RowState st;
  init_state(st, a, qrow, head, valid, lane);
  {
    int kb = k0;
    for (; kb + 64 <= k1 && ((kb % a.BS) + 64 <= a.BS); kb += 64) chunk<2>(st, a, bt, kvh, kb, k1, lane);
    for (; kb < k1; kb += 32) chunk<1>(st, a, bt, kvh, kb, k1, lane);
  }

  float l = st.l + __shfl_xor(st.l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  // rows 4h+i of O belong to lanes 4h+i for m / l
  float mr[4], lr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mr[i] = __shfl(st.m, 4 * h + i, 64);
    lr[i] = __shfl(l, 4 * h + i, 64);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * h + i;
    if (row >= a.G) continue;
    const int qh = kvh * a.G + row;
    if (a.n_parts == 1) {
      const float inv = lr[i] > 0.f ? 1.f / lr[i] : 0.f;
      uint16_t* dst = a.out + (size_t)qrow * a.out_stride + qh * D;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) dst[16 * dt + r] = f2bf(st.o[dt][i] * inv);
    } else {
      const size_t base = ((size_t)seq * a.nq + qh) * a.n_parts + part;
      float* po = a.part_o + base * D;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) po[16 * dt + r] = st.o[dt][i];
      if (r == 0) {
        a.part_ml[base * 2 + 0] = mr[i];
        a.part_ml[base * 2 + 1] = lr[i];
      }
    }
  }
}

// Persistent decode over a host-built work list (BS % 64 == 0): grid = at
// most the resident-wave count (2048 one-wave workgroups: 256 CUs x 4 SIMDs x
// 2); wave g takes work units g, g + grid, ... where unit = item * nkv + kv
// head.  Items come longest-first, so the round-robin assignment is close to
// LPT scheduling, and no wave is ever launched for an empty partition (a
// (seq, parts) grid with the partition count of the longest sequence spent
// most of its waves on nothing when context lengths vary 1k..6k).
// MFMA row rho = qi * G + g: token qi of the item (decode row seq + qi, q row
// qrow + qi), q head g of the kv group.
__device__ __forceinline__ void decode_epilogue(const RowState& st, const AttnArgs& a, int seq, int part, int qrow,
                                                int kvh, bool whole, int nt, int lane) {
  const int r = lane & 15, h = lane >> 4;
  float l = st.l + __shfl_xor(st.l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  float mr[4], lr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mr[i] = __shfl(st.m, 4 * h + i, 64);
    lr[i] = __shfl(l, 4 * h + i, 64);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * h + i;
    if (row >= nt * a.G) continue;
    const int qi = row / a.G;
    const int qh = kvh * a.G + (row - qi * a.G);
    if (whole) {
      const float inv = lr[i] > 0.f ? 1.f / lr[i] : 0.f;
      uint16_t* dst = a.out + (size_t)(qrow + qi) * a.out_stride + qh * D;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) dst[16 * dt + r] = f2bf(st.o[dt][i] * inv);
    } else {
      const size_t base = ((size_t)(seq + qi) * a.nq + qh) * a.n_parts + part;
      float* po = a.part_o + base * D;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) po[16 * dt + r] = st.o[dt][i];
      if (r == 0) {
        a.part_ml[base * 2 + 0] = mr[i];
        a.part_ml[base * 2 + 1] = lr[i];
      }
    }
  }
}

// (Round 2-3 also had an in-kernel split-KV merge by the last-arriving wave of
// each (row group, kv head), K8SRCA_DECODE_MERGE=1: its per-item ticket cost
// what the separate reduce launch saves -- profiles/r2_decode_merge/ -- and it
// was retired in round 4; attn_reduce_kernel merges.)
template <bool NT>
__global__ void __launch_bounds__(64, 2) attn_decode_items_kernel(AttnArgs a) {
  const int lane = threadIdx.x;
  const int r = lane & 15;
  // graphs: {item count, keys per partition} are read on the device, so one
  // captured graph serves every step's plan
  const int n_items = a.d_n_items ? __builtin_amdgcn_readfirstlane(a.d_n_items[0]) : a.n_items;
  const int part_size = a.d_n_items ? __builtin_amdgcn_readfirstlane(a.d_n_items[1]) : a.part_size;
  const int total = n_items * a.nkv;
  for (int w = blockIdx.x; w < total; w += gridDim.x) {
    const int it = w / a.nkv, kvh = w - it * a.nkv;
    const int4 item = a.items[it];
    // item.w = q row | (tokens - 1) << 24: a multi-token item holds up to 16 / G
    // consecutive tokens of one sequence (decode rows seq .. seq + nt - 1, one
    // block table) in the MFMA's 16 rows, so their shared keys are read ONCE
    const int seq = item.x, k1 = item.z, qrow = item.w & 0xFFFFFF, nt = (item.w >> 24) + 1;
    const bool whole = item.y < 0;
    const int part = whole ? 0 : item.y;
    const int k0 = part * part_size;
    const int* bt = a.block_tables + (size_t)seq * a.bt_stride;
    const int pg0 = k0 / a.BS, npg = (k1 - 1) / a.BS - pg0 + 1;
    const int blkv = lane < npg ? bt[pg0 + lane] : 0;
    const int qi = r / a.G;
    const bool valid = qi < nt;
    int lim = k1, kmin = k1;
    if (nt > 1) {  // token qi sees keys < its own context length
      lim = min(k1, a.ctx_lens[seq + min(qi, nt - 1)]);
      kmin = min(k1, __builtin_amdgcn_readfirstlane(a.ctx_lens[seq]));
    }
    RowState st;
    init_state(st, a, qrow + (valid ? qi : 0), kvh * a.G + (valid ? r - qi * a.G : 0), valid, lane);
    decode_stream64<NT>(st, a, blkv, kvh, k0, k1, kmin, lim, lane);
    decode_epilogue(st, a, seq, part, qrow, kvh, whole, nt, lane);
  }
}

// grid: (nq, S); block 128 (one thread per output column).  The (m, l) of the
// row's partitions are loaded ONE PER THREAD and shared through LDS, and the
// partial-O column loads of consecutive partitions are independent (unrolled),
// so a row costs a few memory latencies instead of 2 * n_parts serial ones
// (9.1 us per layer at one decode row with ~12 partitions before, c=1 profile).
// Same max and the same summation order as the serial form.
// PRE: a row of at most kRedPre partitions issues every partition's partial-O
// column load up front (unconditional, clamped to the last partition), beside
// the (m, l) loads, instead of after the max / weights exchange; the exchange
// and the summation are the LDS form's own (bit-identical).  Longer rows take
// the LDS form below.
// Rows of up to 16 partitions (the many-row steps) take the 16-load form; up to
// 32 (one or a few rows over long contexts: 27 at one row x 5k keys, which had
// fallen to the LDS form's serial loads) the 32-load form -- the same arithmetic.
constexpr int kRedPre = 32;
template <int NPRE>
__device__ __forceinline__ void reduce_pre(const AttnArgs& a, size_t base, int np, int qh, int seq, int d, float* sf,
                                           float* sl, float* scratch) {
  // the partial-O column of every partition in flight first (clamped: unconditional),
  // then the LDS form's own max / weights exchange, so the arithmetic is the same
  float po[NPRE];
#pragma unroll
  for (int p = 0; p < NPRE; ++p) po[p] = a.part_o[(base + min(p, np - 1)) * D + d];
  float M = d < np ? a.part_ml[(base + d) * 2] : -INFINITY;
  M = block_max(M, scratch);
  float f = 0.f, lf = 0.f;
  if (d < np) {
    const float m = a.part_ml[(base + d) * 2];
    f = (m == -INFINITY) ? 0.f : exp2f(m - M);
    lf = a.part_ml[(base + d) * 2 + 1] * f;
  }
  sf[d] = f;
  sl[d] = lf;
  __syncthreads();
  float L = 0.f, acc = 0.f;
#pragma unroll
  for (int j = 0; j < NPRE; ++j)
    if (j < np) {
      L += sl[j];
      acc = fmaf(po[j], sf[j], acc);  // explicit: an unrolled, predicated a * b + c may not contract
    }
  const int qrow = a.q_start[seq];
  a.out[(size_t)qrow * a.out_stride + qh * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

template <bool PRE>
__global__ void __launch_bounds__(128) attn_reduce_kernel(AttnArgs a) {
  __shared__ float sf[128], sl[128], scratch[16];
  const int qh = blockIdx.x, seq = blockIdx.y, d = threadIdx.x;
  const int ctx = a.ctx_lens[seq];
  const int part_size = a.d_n_items ? a.d_n_items[1] : a.part_size;
  const int np = min(a.n_parts, (ctx + part_size - 1) / part_size);
  if (np <= 1 && a.items) return;  // work-list mode: whole rows were written by the decode kernel
  const size_t base = ((size_t)seq * a.nq + qh) * a.n_parts;
  if (PRE && np >= 1 && np <= 16) {  // (np == 0, an empty row: the LDS form writes its zero)
    reduce_pre<16>(a, base, np, qh, seq, d, sf, sl, scratch);
    return;
  }
  if (PRE && np > 16 && np <= kRedPre) {
    reduce_pre<kRedPre>(a, base, np, qh, seq, d, sf, sl, scratch);
    return;
  }
  float M = -INFINITY;
  for (int p = d; p < np; p += 128) M = fmaxf(M, a.part_ml[(base + p) * 2]);
  M = block_max(M, scratch);
  float L = 0.f, acc = 0.f;
  for (int p0 = 0; p0 < np; p0 += 128) {
    const int p = p0 + d;
    float f = 0.f, lf = 0.f;
    if (p < np) {
      const float m = a.part_ml[(base + p) * 2];
      f = (m == -INFINITY) ? 0.f : exp2f(m - M);
      lf = a.part_ml[(base + p) * 2 + 1] * f;
    }
    __syncthreads();  // the previous chunk's readers are done with sf / sl
    sf[d] = f;
    sl[d] = lf;
    __syncthreads();
    const int n = min(128, np - p0);
    const float* po = a.part_o + (base + p0) * D + d;
#pragma unroll 8
    for (int j = 0; j < n; ++j) {
      L += sl[j];
      acc = fmaf(po[(size_t)j * D], sf[j], acc);
    }
  }
  const int qrow = a.q_start[seq];
  a.out[(size_t)qrow * a.out_stride + qh * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

// --------------------------------------------------------------- prefill
// grid: (n_tiles, nkv); block 256.  Tile = 64/G tokens of one sequence.
__global__ void __launch_bounds__(256) attn_prefill_kernel(AttnArgs a) {
  const int tile = blockIdx.x, kvh = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int seq = a.tile_seq[tile];
  const int tok0 = a.tile_tok0[tile];
  const int tlen = a.tile_len[tile];
  const int qs = a.q_start[seq];
  const int qlen = a.q_start[seq + 1] - qs;
  const int ctx = a.ctx_lens[seq];
  const int* bt = a.block_tables + (size_t)seq * a.bt_stride;

  const int grow = w * ROWS + r;     // row within the tile
  const int tt = grow / a.G;         // token within the tile
  const int g = grow % a.G;
  const bool valid = tt < tlen;
  const int qrow = tok0 + (valid ? tt : 0);
  const int head = kvh * a.G + g;
  const int pos = ctx - qlen + (qrow - qs);   // absolute position of this row's token
  const int limit = valid ? pos + 1 : 0;       // causal: keys <= pos

  // the wave walks keys up to the last position any of its rows can see
  const int wave_last_tt = min(tlen - 1, (w * ROWS + ROWS - 1) / a.G);
  const int wave_limit = (w * ROWS) / a.G < tlen ? (ctx - qlen + (tok0 + wave_last_tt - qs) + 1) : 0;

  RowState st;
  init_state(st, a, qrow, head, valid, lane);
  int kb = 0;
  for (; kb + 64 <= wave_limit && ((kb % a.BS) + 64 <= a.BS); kb += 64) chunk<2>(st, a, bt, kvh, kb, limit, lane);
  for (; kb < wave_limit; kb += CH) chunk<1>(st, a, bt, kvh, kb, limit, lane);

  float l = st.l + __shfl_xor(st.l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = (l > 0.f) ? 1.f / l : 0.f;
  // O rows 4h+i belong to rows owned by lanes 4h+i
  float inv_r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) inv_r[i] = __shfl(inv, 4 * h + i, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int orow = w * ROWS + 4 * h + i;
    const int ott = orow / a.G, og = orow % a.G;
    if (ott >= tlen) continue;
    uint16_t* dst = a.out + (size_t)(tok0 + ott) * a.out_stride + (kvh * a.G + og) * D;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) dst[16 * dt + r] = f2bf(st.o[dt][i] * inv_r[i]);
  }
}


// ------------------------------------------------------- prefill (paged, BS 64)
// The extend/prefill hot path.  Workgroup = 4 waves x 32 rows = 128 (token,
// q-head) rows of one sequence sharing kv head `kvh` (128/G tokens); one
// 64-key page per iteration, K and V pages staged ONCE per workgroup through
// LDS (register-staged double buffer: the next page's global loads are in
// flight while the current page is computed; one barrier per page).
//
// v_mfma_f32_32x32x16_bf16, swapped QK^T (S^T = K . Q^T): lane (r = l&31,
// hi = l>>5) owns query row r, so the running max / sum / O rescale are
// lane-local (+1 xor-32 shuffle for the max).  Key permutation: MFMA row rho
// of 32-key half kt holds key 32kt + 16*(reg>>3) + 8*hi + (reg&7) with
// reg = (rho&3) + 4*(rho>>3), hi = (rho>>2)&1; S registers 8s..8s+7 of lane
// half h are then keys 16s+8h..+7, exactly the B operand (P^T) of the PV
// MFMA O^T += V^T . P^T for k-step s -> bf16 pack only, no permlane.
// LDS images: K row = 256 B, 16-B chunk c at c ^ (key & 15); V^T row (one
// head dim) = 128 B, chunk c at c ^ ((d >> 1) & 7): every ds_read_b128 lane
// group (4 x 16 lanes) and every ds_write_b128 group (8 lanes) is
// conflict-free for these access patterns.
constexpr int PF_WAVES = 4;
constexpr int PF_ROWS = 32 * PF_WAVES;        // rows per workgroup
constexpr int PF_PAGE = 64;                   // keys per page (== BS)
constexpr int PF_KBYTES = PF_PAGE * D * 2;    // 16 KB
constexpr int PF_VBYTES = D * PF_PAGE * 2;    // 16 KB

__device__ __forceinline__ int pf_key(int reg, int hi) { return 16 * (reg >> 3) + 8 * hi + (reg & 7); }

__global__ void __launch_bounds__(256, 2) attn_prefill_pg64_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2][PF_KBYTES + PF_VBYTES];
  const int kvh = blockIdx.x % a.nkv, tile = blockIdx.x / a.nkv;  // kv head -> XCD (nkv == 8)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hi = lane >> 5;
  const int seq = a.tile_seq[tile];
  const int tok0 = a.tile_tok0[tile];
  const int tlen = a.tile_len[tile];
  const int qs = a.q_start[seq];
  const int qlen = a.q_start[seq + 1] - qs;
  const int ctx = a.ctx_lens[seq];
  const int* bt = a.block_tables + (size_t)seq * a.bt_stride;
  const int base_pos = ctx - qlen + (tok0 - qs);   // position of the tile's first token

  const int grow = w * 32 + r;
  const int tt = grow / a.G, g = grow % a.G;
  const bool valid = tt < tlen;
  const int limit = valid ? base_pos + tt + 1 : 0;  // keys < limit visible to this row
  // wave-uniform key range: rows of wave w are tokens [32w/G, (32w+31)/G]
  const int wt0 = (w * 32) / a.G, wt1 = min(tlen - 1, (w * 32 + 31) / a.G);
  const bool wave_live = wt0 < tlen;
  const int wave_lo = base_pos + wt0 + 1;            // every live row sees keys < wave_lo
  const int wave_hi = wave_live ? base_pos + wt1 + 1 : 0;
  const int kv_end = base_pos + tlen;                // workgroup key range
  const int p_begin = a.tile_kv0[tile];
  const int n_pages = min(a.tile_kv1[tile], (kv_end + PF_PAGE - 1) / PF_PAGE);
  const int slot = a.tile_slot[tile];

  // Q fragments (B operand of S^T): Q[row][16s + 8hi .. +8]
  bf16x8 qf[8];
  {
    const uint16_t* qp = a.q + (size_t)(tok0 + (valid ? tt : 0)) * a.q_stride + (kvh * a.G + g) * D + 8 * hi;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = valid ? load16(qp + 16 * s) : zero8();
  }
  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  // cooperative page staging: 1024 + 1024 16-byte chunks, 4 + 4 per thread
  bf16x8 stg[8];
  auto load_page = [&](int blk) {
    const size_t page = (size_t)blk * a.nkv + kvh;
    const uint16_t* kp = a.kc + page * (size_t)(PF_PAGE * D);
    const uint16_t* vp = a.vc + page * (size_t)(D * PF_PAGE);
#pragma unroll
    for (int i = 0; i < 4; ++i) stg[i] = load16(kp + (size_t)(tid + 256 * i) * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) stg[4 + i] = load16(vp + (size_t)(tid + 256 * i) * 8);
  };
  auto store_page = [&](int b) {
    unsigned char* kl = lds[b];
    unsigned char* vl = lds[b] + PF_KBYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 4, c = q & 15;
      *reinterpret_cast<bf16x8*>(kl + row * 256 + ((c ^ (row & 15)) << 4)) = stg[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, d = q >> 3, c = q & 7;
      *reinterpret_cast<bf16x8*>(vl + d * 128 + ((c ^ ((d >> 1) & 7)) << 4)) = stg[4 + i];
    }
  };

  // this lane's K row per half (A operand row rho = r)
  const int kreg = (r & 3) + 4 * (r >> 3), khi = (r >> 2) & 1;
  const int krow0 = pf_key(kreg, khi);               // key within a 32-key half

  // Q must be resident before the loop: otherwise the waitcnt pass cannot
  // order the Q loads against the in-loop page loads and waits vmcnt(0) at the
  // first QK^T MFMA, serialising the prefetch with compute.
#pragma unroll
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]));
  int blk_next = 0;
  if (p_begin < n_pages) {
    load_page(bt[p_begin]);
    blk_next = bt[min(p_begin + 1, n_pages - 1)];
    store_page(0);
  }
  __syncthreads();
  for (int p = p_begin; p < n_pages; ++p) {
    const int b = (p - p_begin) & 1;
    // block id two pages ahead: its latency hides under this page's compute
    const int blk_after = bt[min(p + 2, n_pages - 1)];
    // unconditional (the last iteration re-reads a valid page): a conditional
    // load would again leave the outstanding-load count ambiguous
    load_page(blk_next);
    const int k0 = p * PF_PAGE;
    if (wave_live && k0 < wave_hi) {
      const unsigned char* kl = lds[b];
      const unsigned char* vl = lds[b] + PF_KBYTES;
      f32x16 sc[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int key = 32 * kt + krow0;
        const unsigned char* kr = kl + key * 256;
        f32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kr + (((2 * s + hi) ^ (key & 15)) << 4));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], acc, 0, 0, 0);
        }
        sc[kt] = acc;
      }
      // causal mask only on pages that cross a row limit (raw scores; scale > 0
      // so the max commutes with it)
      if (k0 + PF_PAGE > wave_lo) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (k0 + 32 * kt + pf_key(i, hi) >= limit) sc[kt][i] = -INFINITY;
      }
      float cmax = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) cmax = fmaxf(cmax, sc[kt][i]);
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      // deferred max (T13): move the reference only when the row max grows by
      // more than 2^8, so P <= 256 (exact in bf16 / fp32 sums) and most pages
      // skip the O rescale entirely.
      const float mcand = cmax * a.scale_log2;
      const bool upd = mcand > m + 8.f;
      const float mnew = upd ? mcand : m;
      const float alpha = upd ? __builtin_amdgcn_exp2f(m - mnew) : 1.f;
      const float nmsub = (mnew == -INFINITY) ? 0.f : -mnew;
      bf16x8 pf[2][2];
      float psum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][8 * s + j], a.scale_log2, nmsub));
            psum += e;
            pf[kt][s][j] = (__bf16)e;
          }
      l = l * alpha + psum;
      m = mnew;
      if (__ballot(upd)) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int d = 32 * dt + r;
        const unsigned char* vr = vl + d * 128;
        const int sw = (d >> 1) & 7;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vr + (((4 * kt + 2 * s + hi) ^ sw) << 4));
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt][s], o[dt], 0, 0, 0);
          }
      }
    }
    store_page(b ^ 1);
    blk_next = blk_after;
    __syncthreads();
  }

  if (!valid) return;
  l += __shfl_xor(l, 32, 64);
  if (slot >= 0) {  // split tile: unnormalised partial, merged by attn_prefill_merge
    const size_t rbase = ((size_t)slot * a.nkv + kvh) * PF_ROWS + grow;
    float* po = a.pf_o + rbase * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        *reinterpret_cast<f32x4*>(po + 32 * dt + 8 * q4 + 4 * hi) =
            f32x4{o[dt][4 * q4], o[dt][4 * q4 + 1], o[dt][4 * q4 + 2], o[dt][4 * q4 + 3]};
    if (hi == 0) {
      a.pf_ml[rbase * 2] = m;
      a.pf_ml[rbase * 2 + 1] = l;
    }
    return;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  // O^T: lane owns query row r; register i of d-tile dt is d = 32dt + (i&3) + 8(i>>2) + 4hi
  uint16_t* dst = a.out + (size_t)(tok0 + tt) * a.out_stride + (kvh * a.G + g) * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      u16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(o[dt][4 * q4 + i] * inv);
      *reinterpret_cast<u16x4*>(dst + 32 * dt + 8 * q4 + 4 * hi) = v;
    }
}

// ------------------------------------------------ prefill (paged, BS 64, 8 waves)
// The 256-row form of the pg64 kernel: workgroup = 8 waves x 32 rows = 256
// (token, q-head) rows of one sequence (256/G tokens), so every staged K/V page
// feeds twice the MFMA work of the 4-wave form (half the staging per query
// token), and pages arrive by LDS-DMA (global_load_lds, no VGPR round trip, no
// ds_write pass) into a 4-page LDS ring: page i+3 is issued right after the
// barrier that retires page i, so three pages (96 KB) are in flight while a
// page is computed.  Synchronisation as the GEMM ring (gemm_stream.hip): one
// __shared__ array, counted vmcnt + raw s_barrier (never __syncthreads inside
// the loop: its fence would drain the DMAs), lgkmcnt(0) after the fragment
// reads.  The LDS images are the pg64 kernel's (XOR-swizzled chunks), written
// lane-linearly with the swizzle moved to the DMA SOURCE address, so the
// per-row arithmetic -- and hence each row's result -- is the pg64 kernel's.
// The tile's page ids are staged in LDS once (no global load in the loop).
constexpr int PF8_WAVES = 8;
constexpr int PF8_ROWS = 32 * PF8_WAVES;            // rows per workgroup
constexpr int PF8_NB = 4;                           // ring pages
constexpr int PF8_STAGE = PF_KBYTES + PF_VBYTES;    // 32 KB
constexpr int PF8_MAXP = 1024;                      // page ids staged in LDS
constexpr int PF8_DMA = 4;                          // DMAs per thread per page (2 K + 2 V)

__device__ __forceinline__ void pf8_glds(const uint16_t* src, unsigned char* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// VAR 6's hand-issued LDS reads with counted waits: lds_rd16 / lgkm_wait (common.h).
// VAR (K8SRCA_PF_W8): 2 = the compiler's schedule of the page loop; 4 = the same
// arithmetic with the page's 16 K fragments read up front (the compiler otherwise
// serialises read -> wait -> MFMA for the first 32 keys: 8 exposed LDS latencies
// per page), the two 32-key score tiles accumulated as interleaved chains, the
// row max as two max3 chains joined across the half-waves by permlane32_swap
// (a VALU exchange instead of a ds_bpermute round trip) and the row sum as four
// partial sums instead of one 32-long dependent add chain.  The measured-loss
// variants (static priority for the younger half: 651 vs 664 TFLOP/s; waves 4-7
// half a page behind: 608) are retired.
template <int VAR>
__global__ void __launch_bounds__(512, 1) attn_prefill_w8_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[PF8_NB * PF8_STAGE + 4 * PF8_MAXP];
  int* s_blk = reinterpret_cast<int*>(lds + PF8_NB * PF8_STAGE);
  const int kvh = blockIdx.x % a.nkv, tile = blockIdx.x / a.nkv;  // kv head -> XCD (nkv == 8)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hi = lane >> 5;
  const int seq = a.tile_seq[tile];
  const int tok0 = a.tile_tok0[tile];
  const int tlen = a.tile_len[tile];
  const int qs = a.q_start[seq];
  const int qlen = a.q_start[seq + 1] - qs;
  const int ctx = a.ctx_lens[seq];
  const int* bt = a.block_tables + (size_t)seq * a.bt_stride;
  const int base_pos = ctx - qlen + (tok0 - qs);

  const int grow = w * 32 + r;
  const int tt = grow / a.G, g = grow % a.G;
  const bool valid = tt < tlen;
  const int limit = valid ? base_pos + tt + 1 : 0;
  const int wt0 = (w * 32) / a.G, wt1 = min(tlen - 1, (w * 32 + 31) / a.G);
  const bool wave_live = wt0 < tlen;
  const int wave_lo = base_pos + wt0 + 1;
  const int wave_hi = wave_live ? base_pos + wt1 + 1 : 0;
  const int kv_end = base_pos + tlen;
  const int p_begin = a.tile_kv0[tile];
  // the planner splits key ranges at PF8_MAXP pages per item (ops/attention.py
  // plan_prefill); the clamp only keeps a foreign plan inside the LDS table
  const int n_pages = min(min(a.tile_kv1[tile], (kv_end + PF_PAGE - 1) / PF_PAGE), p_begin + PF8_MAXP);
  const int np = n_pages - p_begin;
  const int slot = a.tile_slot[tile];

  for (int i = tid; i < np; i += 512) s_blk[i] = bt[p_begin + i];
  bf16x8 qf[8];
  {
    const uint16_t* qp = a.q + (size_t)(tok0 + (valid ? tt : 0)) * a.q_stride + (kvh * a.G + g) * D + 8 * hi;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = valid ? load16(qp + 16 * s) : zero8();
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]));
  __syncthreads();  // page ids visible; every ordinary load retired before the first DMA

  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  // this thread's DMA sources: K pieces 2w, 2w+1 (4 key rows of 256 B each);
  // V pieces 2w, 2w+1 (8 d-rows of 128 B each); lane-linear LDS, swizzled source
  int koff[2], voff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pc = 2 * w + i;
    const int key = 4 * pc + (lane >> 4), kc = (lane & 15) ^ (key & 15);
    koff[i] = key * D + 8 * kc;
    const int d = 8 * pc + (lane >> 3), vc = (lane & 7) ^ ((d >> 1) & 7);
    voff[i] = d * PF_PAGE + 8 * vc;
  }
  auto issue = [&](int stage, int i) {
    const size_t page = (size_t)s_blk[i] * a.nkv + kvh;
    const uint16_t* kp = a.kc + page * (size_t)(PF_PAGE * D);
    const uint16_t* vp = a.vc + page * (size_t)(D * PF_PAGE);
    unsigned char* kl = lds + stage * PF8_STAGE;
    unsigned char* vl = kl + PF_KBYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j) pf8_glds(kp + koff[j], kl + (2 * w + j) * 1024);
#pragma unroll
    for (int j = 0; j < 2; ++j) pf8_glds(vp + voff[j], vl + (2 * w + j) * 1024);
  };

  const int kreg = (r & 3) + 4 * (r >> 3), khi = (r >> 2) & 1;
  const int krow0 = pf_key(kreg, khi);
  constexpr int AHEAD = PF8_NB - 1;  // pages in flight beyond the current one
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds;

  if (np > 0) {
#pragma unroll
    for (int j = 0; j < AHEAD; ++j) issue(j, min(j, np - 1));
  }
  for (int i = 0; i < np; ++i) {
    // this wave's DMAs of page i are done when only the later pages' remain
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((AHEAD - 1) * PF8_DMA) : "memory");
    __builtin_amdgcn_s_barrier();  // every wave's page i landed; every wave is done with the refilled stage
    issue((i + AHEAD) % PF8_NB, min(i + AHEAD, np - 1));  // refill (clamped at the end: an L2 hit)
    const int k0 = (p_begin + i) * PF_PAGE;
    if (wave_live && k0 < wave_hi) {
      const unsigned char* kl = lds + (i % PF8_NB) * PF8_STAGE;
      const unsigned char* vl = kl + PF_KBYTES;
      f32x16 sc[2];
      bf16x8 vq[16];  // VAR 6: the page's V fragments, read during the softmax
      if constexpr (VAR == 6) {
        // K fragments: 16 reads (the second 32-key tile at +8 KB), then each MFMA
        // pair waits only for its own two reads
        const uint32_t ka = lds_base + (uint32_t)((i % PF8_NB) * PF8_STAGE + krow0 * 256);
        bf16x8 kf[2][8];
#define K8S_KRD(S)                                                               \
  {                                                                              \
    const uint32_t a_ = ka + (uint32_t)((((2 * (S) + hi) ^ (krow0 & 15)) << 4)); \
    kf[0][S] = lds_rd16<0>(a_);                                                  \
    kf[1][S] = lds_rd16<8192>(a_);                                               \
  }
        K8S_KRD(0) K8S_KRD(1) K8S_KRD(2) K8S_KRD(3) K8S_KRD(4) K8S_KRD(5) K8S_KRD(6) K8S_KRD(7)
#undef K8S_KRD
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e) sc[kt][e] = 0.f;
#define K8S_KMM(S)                                                                   \
  lgkm_wait<14 - 2 * (S)>(kf[0][S], kf[1][S]);                                       \
  sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[0][S], qf[S], sc[0], 0, 0, 0); \
  sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[1][S], qf[S], sc[1], 0, 0, 0); \
  __builtin_amdgcn_sched_barrier(0); /* the next wait stays behind these MFMAs */
        K8S_KMM(0) K8S_KMM(1) K8S_KMM(2) K8S_KMM(3) K8S_KMM(4) K8S_KMM(5) K8S_KMM(6) K8S_KMM(7)
#undef K8S_KMM
      } else if constexpr (VAR >= 4) {
        // key 32 kt + krow0 has the swizzle of krow0 (32 kt is a multiple of 16):
        // the second tile's reads are the first's at +8 KB
        const unsigned char* kr = kl + krow0 * 256;
        bf16x8 kf[2][8];
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
            kf[kt][s] = *reinterpret_cast<const bf16x8*>(kr + kt * 8192 + (((2 * s + hi) ^ (krow0 & 15)) << 4));
        __builtin_amdgcn_sched_barrier(0);  // all 16 reads issue before the first MFMA (counted waits follow)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e) sc[kt][e] = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kt][s], qf[s], sc[kt], 0, 0, 0);
      } else {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int key = 32 * kt + krow0;
          const unsigned char* kr = kl + key * 256;
          f32x16 acc;
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
          for (int s = 0; s < 8; ++s) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kr + (((2 * s + hi) ^ (key & 15)) << 4));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], acc, 0, 0, 0);
          }
          sc[kt] = acc;
        }
      }
      if (k0 + PF_PAGE > wave_lo) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (k0 + 32 * kt + pf_key(e, hi) >= limit) sc[kt][e] = -INFINITY;
      }
      float cmax;
      if constexpr (VAR >= 4) {
        float c0 = -INFINITY, c1 = -INFINITY;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          c0 = fmaxf(c0, sc[0][e]);
          c1 = fmaxf(c1, sc[1][e]);
        }
        cmax = fmaxf(c0, c1);
        // lanes 0-31 and 32-63 hold the two halves of a row's 64 keys: after the
        // swap one operand has this lane's value and the other the partner's
        const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_uint(cmax), __float_as_uint(cmax), false, false);
        cmax = fmaxf(__uint_as_float(pr[0]), __uint_as_float(pr[1]));
      } else {
        cmax = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int e = 0; e < 16; ++e) cmax = fmaxf(cmax, sc[kt][e]);
        cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      }
      if constexpr (VAR == 6) {
        // V fragments of d-row 32 dt + r: the row's chunk swizzle (d >> 1) & 7 does
        // not depend on dt (32 dt is a multiple of 16), so dt is the +4 KB immediate;
        // issued now, they land while the exps below run
        const uint32_t va = lds_base + (uint32_t)((i % PF8_NB) * PF8_STAGE + PF_KBYTES + r * 128);
        const int sw = (r >> 1) & 7;
#define K8S_VRD(KT, S)                                                            \
  {                                                                               \
    const uint32_t a_ = va + (uint32_t)((((4 * (KT) + 2 * (S) + hi) ^ sw) << 4)); \
    vq[0 + 2 * (KT) + (S)] = lds_rd16<0>(a_);                                     \
    vq[4 + 2 * (KT) + (S)] = lds_rd16<4096>(a_);                                  \
    vq[8 + 2 * (KT) + (S)] = lds_rd16<8192>(a_);                                  \
    vq[12 + 2 * (KT) + (S)] = lds_rd16<12288>(a_);                                \
  }
        K8S_VRD(0, 0) K8S_VRD(0, 1) K8S_VRD(1, 0) K8S_VRD(1, 1)
#undef K8S_VRD
      }
      const float mcand = cmax * a.scale_log2;
      const bool upd = mcand > m + 8.f;
      const float mnew = upd ? mcand : m;
      const float alpha = upd ? __builtin_amdgcn_exp2f(m - mnew) : 1.f;
      const float nmsub = (mnew == -INFINITY) ? 0.f : -mnew;
      bf16x8 pf[2][2];
      float ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][8 * s + j], a.scale_log2, nmsub));
            if constexpr (VAR >= 4)
              ps[j & 3] += e;
            else
              ps[0] += e;
            pf[kt][s][j] = (__bf16)e;
          }
      const float psum = VAR >= 4 ? (ps[0] + ps[1]) + (ps[2] + ps[3]) : ps[0];
      l = l * alpha + psum;
      m = mnew;
      if (__ballot(upd)) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) o[dt][e] *= alpha;
      }
      if constexpr (VAR == 6) {
        // issue order: (kt, s) outer, dt inner -> read q = 4 (2 kt + s) + dt
#define K8S_VMM(KT, S, DT)                                                                                  \
  lgkm_wait<15 - (4 * (2 * (KT) + (S)) + (DT))>(vq[4 * (DT) + 2 * (KT) + (S)]);                             \
  o[DT] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vq[4 * (DT) + 2 * (KT) + (S)], pf[KT][S], o[DT], 0, 0, 0); \
  __builtin_amdgcn_sched_barrier(0);
        K8S_VMM(0, 0, 0) K8S_VMM(0, 0, 1) K8S_VMM(0, 0, 2) K8S_VMM(0, 0, 3)
        K8S_VMM(0, 1, 0) K8S_VMM(0, 1, 1) K8S_VMM(0, 1, 2) K8S_VMM(0, 1, 3)
        K8S_VMM(1, 0, 0) K8S_VMM(1, 0, 1) K8S_VMM(1, 0, 2) K8S_VMM(1, 0, 3)
        K8S_VMM(1, 1, 0) K8S_VMM(1, 1, 1) K8S_VMM(1, 1, 2) K8S_VMM(1, 1, 3)
#undef K8S_VMM
      } else {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int d = 32 * dt + r;
          const unsigned char* vr = vl + d * 128;
          const int sw = (d >> 1) & 7;
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vr + (((4 * kt + 2 * s + hi) ^ sw) << 4));
              o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt][s], o[dt], 0, 0, 0);
            }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS

  if constexpr (VAR >= 5) {
    // Epilogue through LDS (the ring is free once every wave has left the loop):
    // each wave stages its 32 rows x 128 dims as bf16 (O / l) in a private,
    // 272-B-pitch image (conflict-free 8-B writes), then stores 16 B per lane
    // with 16 lanes per row: full 256-B rows (a token's G heads are contiguous
    // in `out`), 8 dwordx4 stores instead of 16 dwordx2 at a 512-B lane stride
    // (cdna_hip_programming.md T21: the row-per-lane store tail is issue-bound).
    // Split tiles store the same bf16 O / l rows plus (m, l): half the fp32
    // partial's bytes, merged by attn_prefill_merge (pf_bf16).
    constexpr int PITCH = 272;
    __syncthreads();
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    unsigned char* wl = lds + w * (32 * PITCH);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][4 * q4 + e] * inv);
        *reinterpret_cast<u16x4*>(wl + r * PITCH + 2 * (32 * dt + 8 * q4 + 4 * hi)) = v;
      }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int c16 = lane & 15;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int rr = 4 * j + (lane >> 4);
      const int gr = w * 32 + rr, tr = gr / a.G, gg = gr % a.G;
      const u16x8 v = *reinterpret_cast<const u16x8*>(wl + rr * PITCH + 16 * c16);
      if (tr < tlen) {
        uint16_t* dst = slot >= 0
            ? reinterpret_cast<uint16_t*>(a.pf_o) + (((size_t)slot * a.nkv + kvh) * PF8_ROWS + gr) * D + 8 * c16
            : a.out + (size_t)(tok0 + tr) * a.out_stride + (kvh * a.G + gg) * D + 8 * c16;
        *reinterpret_cast<u16x8*>(dst) = v;
      }
    }
    if (slot >= 0 && valid && hi == 0) {
      const size_t rbase = ((size_t)slot * a.nkv + kvh) * PF8_ROWS + grow;
      a.pf_ml[rbase * 2] = m;
      a.pf_ml[rbase * 2 + 1] = l;
    }
    return;
  }
  if (!valid) return;
  l += __shfl_xor(l, 32, 64);
  if (slot >= 0) {  // split tile: unnormalised partial, merged by attn_prefill_merge
    const size_t rbase = ((size_t)slot * a.nkv + kvh) * PF8_ROWS + grow;
    float* po = a.pf_o + rbase * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        *reinterpret_cast<f32x4*>(po + 32 * dt + 8 * q4 + 4 * hi) =
            f32x4{o[dt][4 * q4], o[dt][4 * q4 + 1], o[dt][4 * q4 + 2], o[dt][4 * q4 + 3]};
    if (hi == 0) {
      a.pf_ml[rbase * 2] = m;
      a.pf_ml[rbase * 2 + 1] = l;
    }
    return;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  uint16_t* dst = a.out + (size_t)(tok0 + tt) * a.out_stride + (kvh * a.G + g) * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      u16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][4 * q4 + e] * inv);
      *reinterpret_cast<u16x4*>(dst + 32 * dt + 8 * q4 + 4 * hi) = v;
    }
}

// grid: (n_merge * nkv, PF_ROWS / 4); block 256: ONE WAVE PER ROW (a wave
// walking many rows serialises np dependent loads per row).  Two passes:
// M = max_p m_p, then O = sum_p o_p 2^(m_p - M) / sum_p l_p 2^(m_p - M), 2 dims per lane.
__global__ void __launch_bounds__(256) attn_prefill_merge_kernel(AttnArgs a) {
  const int kvh = blockIdx.x % a.nkv, mi = blockIdx.x / a.nkv;
  const int lane = threadIdx.x & 63, row = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int rows = a.m_len[mi] * a.G;
  if (row >= rows) return;
  const int tok0 = a.m_tok0[mi], slot0 = a.m_slot0[mi], np = a.m_np[mi];
  // two passes (the row max, then the rescaled sums) whose per-part loads do
  // not depend on each other, so they are in flight together: the online form
  // chained every part's loads behind the previous part's rescale (11.4 us per
  // merge launch, r2 headline profile)
  float M = -INFINITY;
#pragma unroll 4
  for (int p = 0; p < np; ++p) {
    const size_t rb = ((size_t)(slot0 + p) * a.nkv + kvh) * a.pf_rows + row;
    M = fmaxf(M, a.pf_ml[rb * 2]);
  }
  float L = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll 4
  for (int p = 0; p < np; ++p) {
    const size_t rb = ((size_t)(slot0 + p) * a.nkv + kvh) * a.pf_rows + row;
    const float2 ml = *reinterpret_cast<const float2*>(a.pf_ml + rb * 2);
    // a part that saw no key of the row has m = -inf: weight 0
    const float f = (ml.x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml.x - M);
    L = fmaf(ml.y, f, L);  // explicit fmas: the merge16 form rounds identically
    if (a.pf_bf16) {  // O / l in bf16: the part's O is (O / l) * l
      const uint32_t v = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(a.pf_o) + rb * D + 2 * lane);
      const float fl = f * ml.y;
      o0 = fmaf(bf2f((uint16_t)(v & 0xffffu)), fl, o0);
      o1 = fmaf(bf2f((uint16_t)(v >> 16)), fl, o1);
    } else {
      const float2 v = *reinterpret_cast<const float2*>(a.pf_o + rb * D + 2 * lane);
      o0 += v.x * f;
      o1 += v.y * f;
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int tt = row / a.G, g = row % a.G;
  uint16_t* dst = a.out + (size_t)(tok0 + tt) * a.out_stride + (kvh * a.G + g) * D + 2 * lane;
  dst[0] = f2bf(o0 * inv);
  dst[1] = f2bf(o1 * inv);
}

// The bf16-partial merge (pf_bf16: VAR >= 5) at 16 rows per block: 16 lanes
// per row, 8 dims (one 16-B load) per lane per part, so a block moves 4 KiB
// per part instead of 1 KiB and the launch has a quarter of the waves (the
// 2-dims-per-lane form above ran ~15 us per call on the steady-state replay:
// tens of thousands of waves with 4-byte loads).  Same per-element arithmetic
// in the same order: bit-identical.
constexpr int kMergePre = 8;  // parts prefetched in one round (~97 % of the replay's merges; more: the two-pass loop)
__global__ void __launch_bounds__(256) attn_prefill_merge16_kernel(AttnArgs a) {
  const int kvh = blockIdx.x % a.nkv, mi = blockIdx.x / a.nkv;
  const int c16 = threadIdx.x & 15, row = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int rows = a.m_len[mi] * a.G;
  if (row >= rows) return;
  const int tok0 = a.m_tok0[mi], slot0 = a.m_slot0[mi], np = a.m_np[mi];
  float M = -INFINITY, L = 0.f, o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = 0.f;
  if (np <= kMergePre) {
    // every part's (m, l) and O piece in ONE round of loads (unconditional: parts past
    // np re-read the last one and are never summed), then the two passes from registers
    float2 ml[kMergePre];
    u16x8 v[kMergePre];
#pragma unroll
    for (int p = 0; p < kMergePre; ++p) {
      const size_t rb = ((size_t)(slot0 + min(p, np - 1)) * a.nkv + kvh) * a.pf_rows + row;
      ml[p] = *reinterpret_cast<const float2*>(a.pf_ml + rb * 2);
      v[p] = *reinterpret_cast<const u16x8*>(reinterpret_cast<const uint16_t*>(a.pf_o) + rb * D + 8 * c16);
    }
#pragma unroll
    for (int p = 0; p < kMergePre; ++p)
      if (p < np) M = fmaxf(M, ml[p].x);
#pragma unroll
    for (int p = 0; p < kMergePre; ++p)
      if (p < np) {
        const float f = (ml[p].x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml[p].x - M);
        L = fmaf(ml[p].y, f, L);
        const float fl = f * ml[p].y;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaf(bf2f(v[p][j]), fl, o[j]);
      }
  } else {
#pragma unroll 4
  for (int p = 0; p < np; ++p) {
    const size_t rb = ((size_t)(slot0 + p) * a.nkv + kvh) * a.pf_rows + row;
    M = fmaxf(M, a.pf_ml[rb * 2]);
  }
#pragma unroll 4
  for (int p = 0; p < np; ++p) {
    const size_t rb = ((size_t)(slot0 + p) * a.nkv + kvh) * a.pf_rows + row;
    const float2 ml = *reinterpret_cast<const float2*>(a.pf_ml + rb * 2);
    const float f = (ml.x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml.x - M);
    L = fmaf(ml.y, f, L);
    const u16x8 v = *reinterpret_cast<const u16x8*>(reinterpret_cast<const uint16_t*>(a.pf_o) + rb * D + 8 * c16);
    const float fl = f * ml.y;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(bf2f(v[j]), fl, o[j]);
  }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int tt = row / a.G, g = row % a.G;
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(o[j] * inv);
  *reinterpret_cast<u16x8*>(a.out + (size_t)(tok0 + tt) * a.out_stride + (kvh * a.G + g) * D + 8 * c16) = r;
}

// the decode split-KV reduce's prefetch form for rows of <= kRedPre partitions (default;
// knob decode_reduce_pre=0: the LDS form everywhere, A/B, read per launch).  Bit-identical;
// 8.5 -> 6.4 us per call on the steady-state decode replay (profiles/r4/reduce_pre/)
static bool decode_reduce_pre() { return knob(kKnobDecodeReducePre) != 0; }

// knob pf_merge16=0: the 2-dims-per-lane merge for bf16 partials too (A/B, read per launch)
static bool pf_merge16() { return knob(kKnobPfMerge16) != 0; }

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_attn_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                            int bt_stride, const int* ctx_lens, const int* q_start, int S, int nq, int nkv, int BS,
                            float scale, void* out, int out_stride, float* part_o, float* part_ml, int n_parts,
                            int part_size, const int* items, int n_items, const int* d_n_items, int grid_waves,
                            hipStream_t stream) {
  if (nq % nkv || (nq / nkv) > 16 || BS % 32 || part_size % 32) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const uint16_t*)q;
  a.q_stride = q_stride;
  a.kc = (const uint16_t*)kc;
  a.vc = (const uint16_t*)vc;
  a.block_tables = block_tables;
  a.bt_stride = bt_stride;
  a.ctx_lens = ctx_lens;
  a.q_start = q_start;
  a.nq = nq;
  a.nkv = nkv;
  a.G = nq / nkv;
  a.BS = BS;
  a.scale_log2 = scale * LOG2E;
  a.out = (uint16_t*)out;
  a.out_stride = out_stride;
  a.part_o = part_o;
  a.part_ml = part_ml;
  a.n_parts = n_parts;
  a.part_size = part_size;
  if (items) {  // work-list path (BS % 64 == 0, part_size % 64 == 0, <= 64 pages per item)
    if (BS % 64 || part_size % 64 || part_size / BS > 64 || grid_waves <= 0) return (int)hipErrorInvalidValue;
    a.items = reinterpret_cast<const int4*>(items);
    a.n_items = n_items;
    a.d_n_items = d_n_items;
    if (knob(kKnobDecodeKvNt))
      hipLaunchKernelGGL(attn_decode_items_kernel<true>, dim3(grid_waves), dim3(64), 0, stream, a);
    else
      hipLaunchKernelGGL(attn_decode_items_kernel<false>, dim3(grid_waves), dim3(64), 0, stream, a);
  } else {
    const long nw = (long)S * nkv * n_parts;
    hipLaunchKernelGGL(attn_decode_kernel, dim3((unsigned)nw), dim3(64), 0, stream, a, S);
  }
  if (n_parts > 1) {
    if (decode_reduce_pre())
      hipLaunchKernelGGL(attn_reduce_kernel<true>, dim3(nq, S), dim3(128), 0, stream, a);
    else
      hipLaunchKernelGGL(attn_reduce_kernel<false>, dim3(nq, S), dim3(128), 0, stream, a);
  }
  return (int)hipGetLastError();
}

// K8SRCA_PF_W8: 256-row LDS-DMA prefill workgroups -- unset / 1 / 6: the explicit
// page loop with hand-issued LDS reads (counted waits, V fragments read during the
// softmax) and the LDS-staged bf16 epilogue (VAR 6); 5: the same with hipcc's own
// LDS reads (a full lgkmcnt(0) before every MFMA pair); 4: + per-lane fp32 partial /
// dwordx2 row stores; 2: the compiler's schedule -- and 0: the 128-row pg64 kernel.
// Read per launch, like the planner reads it per plan.  Replayed steady-state mix
// (tools/bench_kernels.py --what replay, profiles/r4/prefill_attn/, interleaved in
// one process): 6 = 711 / 5 = 684 TFLOP/s; earlier pairs 5 = 649 / 4 = 624 / 2 = 628
// and 4 = 669 / 2 = 648, pg64 633 (r3: static priority 651, staggered late waves 608).
static int prefill_w8() {
  const int v = knob(kKnobPfW8);
  return v == 1 ? 6 : v;
}

K8S_API int k8s_attn_prefill(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                             int bt_stride, const int* ctx_lens, const int* q_start, const int* tile_seq,
                             const int* tile_tok0, const int* tile_len, const int* tile_kv0, const int* tile_kv1,
                             const int* tile_slot, int n_tiles, const int* m_tok0, const int* m_len,
                             const int* m_slot0, const int* m_np, int n_merge, float* pf_o, float* pf_ml, int nq,
                             int nkv, int BS, float scale, void* out, int out_stride, hipStream_t stream) {
  if (nq % nkv || (nq / nkv) > 16 || BS % 32) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const uint16_t*)q;
  a.q_stride = q_stride;
  a.kc = (const uint16_t*)kc;
  a.vc = (const uint16_t*)vc;
  a.block_tables = block_tables;
  a.bt_stride = bt_stride;
  a.ctx_lens = ctx_lens;
  a.q_start = q_start;
  a.nq = nq;
  a.nkv = nkv;
  a.G = nq / nkv;
  a.BS = BS;
  a.scale_log2 = scale * LOG2E;
  a.out = (uint16_t*)out;
  a.out_stride = out_stride;
  a.tile_seq = tile_seq;
  a.tile_tok0 = tile_tok0;
  a.tile_len = tile_len;
  a.tile_kv0 = tile_kv0;
  a.tile_kv1 = tile_kv1;
  a.tile_slot = tile_slot;
  a.m_tok0 = m_tok0;
  a.m_len = m_len;
  a.m_slot0 = m_slot0;
  a.m_np = m_np;
  a.pf_o = pf_o;
  a.pf_ml = pf_ml;
  if (n_tiles <= 0) return (int)hipSuccess;
  if (BS == PF_PAGE && PF_ROWS % a.G == 0) {
    if (n_merge > 0 && (!pf_o || !pf_ml)) return (int)hipErrorInvalidValue;
    // the tile size is the planner's: ops/attention.py pf_wg_rows() is the same
    // function of (K8SRCA_PF_W8, G) -- no other condition may pick the 128-row
    // kernel for a plan tiled at 256 rows (its rows 128.. would never be written)
    const int var = prefill_w8();
    const bool w8 = var > 0 && PF8_ROWS % a.G == 0;
    a.pf_rows = w8 ? PF8_ROWS : PF_ROWS;
    a.pf_bf16 = w8 && var >= 5;
    if (w8 && var == 6)
      hipLaunchKernelGGL(attn_prefill_w8_kernel<6>, dim3(n_tiles * nkv), dim3(512), 0, stream, a);
    else if (w8 && var == 5)
      hipLaunchKernelGGL(attn_prefill_w8_kernel<5>, dim3(n_tiles * nkv), dim3(512), 0, stream, a);
    else if (w8 && var == 4)
      hipLaunchKernelGGL(attn_prefill_w8_kernel<4>, dim3(n_tiles * nkv), dim3(512), 0, stream, a);
    else if (w8)
      hipLaunchKernelGGL(attn_prefill_w8_kernel<2>, dim3(n_tiles * nkv), dim3(512), 0, stream, a);
    else
      hipLaunchKernelGGL(attn_prefill_pg64_kernel, dim3(n_tiles * nkv), dim3(256), 0, stream, a);
    if (n_merge > 0 && a.pf_bf16 && pf_merge16())
      hipLaunchKernelGGL(attn_prefill_merge16_kernel, dim3(n_merge * nkv, a.pf_rows / 16), dim3(256), 0, stream, a);
    else if (n_merge > 0)
      hipLaunchKernelGGL(attn_prefill_merge_kernel, dim3(n_merge * nkv, a.pf_rows / 4), dim3(256), 0, stream, a);
  } else {
    if (n_merge > 0) return (int)hipErrorInvalidValue;  // the generic kernel does not split
    hipLaunchKernelGGL(attn_prefill_kernel, dim3(n_tiles, nkv), dim3(256), 0, stream, a);
  }
  return (int)hipGetLastError();
}
