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
#include "common.h"

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
};

struct RowState {
  bf16x8 qf[4];
  f32x4 o[8];
  float m;      // running max (log2 domain) of this lane's row
  float l;      // lane-partial row sum
};

__device__ __forceinline__ bf16x8 load16(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

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
// grid: (n_parts / 4, nkv, S); block 256.  Each WAVE owns one key partition of
// `part_size` keys (a multiple of the page size): no LDS, no barriers; it
// writes an unnormalised partial (O, m, l) merged by attn_reduce, or the final
// bf16 row when n_parts == 1.
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int part = blockIdx.x * 4 + w, kvh = blockIdx.y, seq = blockIdx.z;
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
  int kb = k0;
  for (; kb + 64 <= k1 && ((kb % a.BS) + 64 <= a.BS); kb += 64) chunk<2>(st, a, bt, kvh, kb, k1, lane);
  for (; kb < k1; kb += 32) chunk<1>(st, a, bt, kvh, kb, k1, lane);

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

// grid: (nq, S); block 128 (one thread per output column)
__global__ void __launch_bounds__(128) attn_reduce_kernel(AttnArgs a) {
  const int qh = blockIdx.x, seq = blockIdx.y, d = threadIdx.x;
  const int ctx = a.ctx_lens[seq];
  const int np = min(a.n_parts, (ctx + a.part_size - 1) / a.part_size);
  const size_t base = ((size_t)seq * a.nq + qh) * a.n_parts;
  float M = -INFINITY;
  for (int p = 0; p < np; ++p) M = fmaxf(M, a.part_ml[(base + p) * 2]);
  float L = 0.f, acc = 0.f;
  for (int p = 0; p < np; ++p) {
    const float m = a.part_ml[(base + p) * 2];
    const float f = (m == -INFINITY) ? 0.f : exp2f(m - M);
    L += a.part_ml[(base + p) * 2 + 1] * f;
    acc += a.part_o[(base + p) * D + d] * f;
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

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_attn_decode(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                            int bt_stride, const int* ctx_lens, const int* q_start, int S, int nq, int nkv, int BS,
                            float scale, void* out, int out_stride, float* part_o, float* part_ml, int n_parts,
                            int part_size, hipStream_t stream) {
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
  hipLaunchKernelGGL(attn_decode_kernel, dim3((n_parts + 3) / 4, nkv, S), dim3(256), 0, stream, a);
  if (n_parts > 1) hipLaunchKernelGGL(attn_reduce_kernel, dim3(nq, S), dim3(128), 0, stream, a);
  return (int)hipGetLastError();
}

K8S_API int k8s_attn_prefill(const void* q, int q_stride, const void* kc, const void* vc, const int* block_tables,
                             int bt_stride, const int* ctx_lens, const int* q_start, const int* tile_seq,
                             const int* tile_tok0, const int* tile_len, int n_tiles, int nq, int nkv, int BS,
                             float scale, void* out, int out_stride, hipStream_t stream) {
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
  if (n_tiles > 0) hipLaunchKernelGGL(attn_prefill_kernel, dim3(n_tiles, nkv), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}
