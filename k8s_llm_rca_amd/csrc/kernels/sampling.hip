// Masked sampling over the vocabulary (B9): greedy argmax, temperature, top-k
// and top-p (nucleus), over fp32 (default) or bf16 logits.
//
// Sampling is exact categorical sampling by the Gumbel-max trick:
//   tok = argmax_{i in S}  v_i + G_i,   v_i = logit_i / T,   G_i = -log(-log(U_i)),
// U_i from a counter-based hash of (seed, step, i) -> reproducible and
// graph-capturable (seed/step live in device memory).  The per-request seed
// already includes the sequence id, so the noise does not depend on the row's
// position in the batch.  S is the allowed set:
//   * grammar mask: bitmap mask_table[mask_id[row]] ([V/32] uint32) or an
//     explicit allow-list slice (list_off, list_len);
//   * top-k: the allowed tokens whose v is >= the k-th largest v (ties kept,
//     like HF's `logits < topk_values[..., -1]` filter);
//   * top-p: of those, the smallest highest-v prefix whose softmax mass
//     reaches p (the token that crosses p is kept; ties kept).
// Rows with neither top-k nor top-p take ONE pass over the logits.  Rows with
// either find their thresholds by MSB-first radix select on the order-
// preserving uint32 image of v: 4 byte-passes with a 256-bin LDS histogram of
// counts (top-k) or of softmax mass exp(v - max) (top-p), then one Gumbel-max
// pass over the survivors.  Everything is one 256-thread workgroup per row.
//
// Vocab-parallel (TP) forms: the rank holds columns [vocab_off, vocab_off + V)
// of the vocabulary; noise and masks are keyed by the GLOBAL token id.
//   * out_pair: the rank's (score, id) Gumbel-max winner; the max over ranks
//     is exactly the unsharded kernel's token (B10 without a logits gather).
//   * out_cand (top-k / top-p rows): the rank's highest-v allowed candidates
//     (v, id, v + G), cand_k per row sorted by (v desc, id asc), padded with
//     (-inf, -1, -inf); the ranks' lists are all-gathered and combined (ops/sampling.py):
//     exact for rows with top-k <= cand_k (any top-p: the nucleus lies inside
//     the top-k set); the engine all-gathers the logits of other filtered rows.
#include "common.h"

namespace k8s {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float gumbel(uint32_t seed, uint32_t row, uint32_t step, uint32_t i) {
  uint32_t h = mix32(seed ^ mix32(row * 0x9E3779B9U ^ mix32(step * 0x85EBCA6BU ^ mix32(i + 0x27D4EB2FU))));
  const float u = ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}

// order-preserving map float -> uint32 (larger float -> larger key; -inf > 0)
__device__ __forceinline__ uint32_t okey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct Best {
  float v;
  int i;
};

__device__ __forceinline__ Best better(Best a, Best b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i && b.i >= 0)) return b;
  return a;
}

__device__ __forceinline__ float lg(const uint16_t* p, int i) { return bf2f(p[i]); }
__device__ __forceinline__ float lg(const float* p, int i) { return p[i]; }

// 8 consecutive logits (i0 % 8 == 0): one 16-B (bf16) or two 16-B (f32) loads
__device__ __forceinline__ void lg8(const uint16_t* p, int i0, float* o) {
  const u16x8 x = *reinterpret_cast<const u16x8*>(p + i0);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(x[j]);
}
__device__ __forceinline__ void lg8(const float* p, int i0, float* o) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p + i0);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + i0 + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = a[j];
    o[4 + j] = b[j];
  }
}

// Calls f(global_id, v) for every allowed token of the row held by this
// thread's share (v = logit * inv_temp).
template <typename T, typename F>
__device__ __forceinline__ void for_allowed(const T* lr, int V, int vocab_off, float it, const int* lst, int ll,
                                            const uint32_t* mk, F&& f) {
  if (ll > 0) {
    for (int k = threadIdx.x; k < ll; k += blockDim.x) {
      const int gi = lst[k];
      const int i = gi - vocab_off;
      if (i < 0 || i >= V) continue;
      f(gi, lg(lr, i) * it);
    }
    return;
  }
  const int nv = V >> 3;
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    const int i0 = c * 8, g0 = vocab_off + i0;  // vocab_off % 8 == 0 (host-checked)
    uint32_t bits = 0xFFu;
    if (mk) bits = (mk[g0 >> 5] >> (g0 & 31)) & 0xFFu;
    if (!bits) continue;
    float x[8];
    lg8(lr, i0, x);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((bits >> j) & 1u) f(g0 + j, x[j] * it);
  }
  for (int i = (nv << 3) + threadIdx.x; i < V; i += blockDim.x) {  // tail (V % 8)
    const int gi = vocab_off + i;
    if (mk && !((mk[gi >> 5] >> (gi & 31)) & 1u)) continue;
    f(gi, lg(lr, i) * it);
  }
}

__device__ __forceinline__ Best block_best(Best best, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best other{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, other);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    sv[w] = best.v;
    si[w] = best.i;
  }
  __syncthreads();
  Best b{sv[0], si[0]};
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) b = better(b, Best{sv[k], si[k]});
  return b;
}

// One radix-select byte pass.  Keys whose bytes above `byte` equal `prefix`'s
// and that are >= `floor_key` add `count ? 1 : exp(v - vmax)` to bin (key >>
// 8*byte) & 255.  Then bins are walked from 255 down: the first bin at which
// the running total reaches `*need` is fixed into `*prefix`, and `*need` drops
// by the total of the bins above it.  The mass is accumulated in 2^-24 fixed
// point with 64-bit integer atomics: integer sums do not depend on the order
// the atomics land in, so the bin chosen at the nucleus boundary -- and the
// sampled token -- is the same on every run (float atomics were not).
constexpr float kMassScale = 16777216.0f;  // 2^24

template <typename T>
__device__ void radix_pass(const T* lr, int V, int vocab_off, float it, const int* lst, int ll, const uint32_t* mk,
                           int byte, bool count, float vmax, uint32_t floor_key, uint32_t* prefix, float* need,
                           unsigned long long* hist) {
  for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0ull;
  __syncthreads();
  const uint32_t pre = *prefix;
  const int hs = 8 * (byte + 1);
  for_allowed(lr, V, vocab_off, it, lst, ll, mk, [&](int, float v) {
    const uint32_t k = okey(v);
    if (k < floor_key) return;
    if (hs < 32 && (k >> hs) != (pre >> hs)) return;
    const unsigned long long add =
        count ? (unsigned long long)kMassScale : (unsigned long long)(__expf(v - vmax) * kMassScale + 0.5f);
    atomicAdd(&hist[(k >> (8 * byte)) & 255u], add);
  });
  __syncthreads();
  if (threadIdx.x == 0) {
    float cum = 0.f, rem = *need;
    int pick = -1, lowest = -1;
    for (int b = 255; b >= 0; --b) {
      const float h = (float)((double)hist[b] * (1.0 / kMassScale));
      if (h <= 0.f) continue;
      lowest = b;
      if (cum + h >= rem) {
        pick = b;
        break;
      }
      cum += h;
    }
    if (pick < 0) {  // rounding: the target was never reached -> keep the whole remaining set
      pick = lowest < 0 ? 0 : lowest;
      if (lowest >= 0) cum -= (float)((double)hist[lowest] * (1.0 / kMassScale));  // mass units, like cum
    }
    *need = rem - cum;
    *prefix = pre | ((uint32_t)pick << (8 * byte));
  }
  __syncthreads();
}

constexpr int kNonFinite = -2;

template <typename T>
__global__ void __launch_bounds__(256) sample_kernel(const T* __restrict__ logits, int ld, int V, int vocab_off,
                                                     const float* __restrict__ temperature,
                                                     const uint32_t* __restrict__ seeds,
                                                     const int* __restrict__ steps,
                                                     const int* __restrict__ mask_id,
                                                     const uint32_t* __restrict__ mask_table, int mask_words,
                                                     const int* __restrict__ list_off, const int* __restrict__ list_len,
                                                     const int* __restrict__ lists, const int* __restrict__ top_k,
                                                     const float* __restrict__ top_p, int* __restrict__ out,
                                                     float2* __restrict__ out_pair, float* __restrict__ out_cand,
                                                     int cand_k) {
  __shared__ unsigned long long hist[256];
  __shared__ float sv[4];
  __shared__ int si[4];
  __shared__ uint32_t s_prefix;
  __shared__ float s_need;
  __shared__ int s_nc;
  __shared__ float c_v[256];
  __shared__ int c_i[256];

  const int row = blockIdx.x;
  const T* lr = logits + (size_t)row * ld;
  const float temp = temperature ? temperature[row] : 0.f;
  const bool greedy = !(temp > 0.f);
  const float it = greedy ? 1.f : 1.f / temp;
  const uint32_t seed = seeds ? seeds[row] : 0u;
  const uint32_t step = steps ? (uint32_t)steps[row] : 0u;
  const int ll = list_len ? list_len[row] : 0;
  const int* lst = ll > 0 ? lists + list_off[row] : nullptr;
  const int mid = mask_id ? mask_id[row] : -1;
  const uint32_t* mk = (ll <= 0 && mid >= 0) ? mask_table + (size_t)mid * mask_words : nullptr;
  const int kk = top_k ? top_k[row] : 0;
  const float pp = top_p ? top_p[row] : 1.f;
  const bool cand = out_cand != nullptr && (kk > 0 || pp < 1.f);
  const bool filt = !greedy && (kk > 0 || pp < 1.f);

  uint32_t thr = 0u;  // survivors: okey(v) >= thr
  if (filt || cand) {
    // ---- row max and allowed count
    Best mx{-INFINITY, -1};
    int n_allowed = 0;
    for_allowed(lr, V, vocab_off, it, lst, ll, mk, [&](int gi, float v) {
      mx = better(mx, Best{v, gi});
      ++n_allowed;
    });
    const float vmax = block_best(mx, sv, si).v;
    __syncthreads();
    const float nal = block_sum((float)n_allowed, sv);
    // ---- top-k threshold (cand: the rank-local top-cand_k)
    const int keff = cand ? ((kk > 0 && kk < cand_k) ? kk : cand_k) : kk;
    if (keff > 0 && (float)keff < nal) {
      if (threadIdx.x == 0) {
        s_prefix = 0u;
        s_need = (float)keff;
      }
      __syncthreads();
      for (int byte = 3; byte >= 0; --byte)
        radix_pass(lr, V, vocab_off, it, lst, ll, mk, byte, true, vmax, 0u, &s_prefix, &s_need, hist);
      thr = s_prefix;
    }
    // ---- top-p threshold inside the top-k set (single-rank form only)
    if (!cand && pp < 1.f) {
      float z = 0.f;
      for_allowed(lr, V, vocab_off, it, lst, ll, mk, [&](int, float v) {
        if (okey(v) >= thr) z += __expf(v - vmax);
      });
      __syncthreads();
      z = block_sum(z, sv);
      if (threadIdx.x == 0) {
        s_prefix = 0u;
        s_need = fmaxf(pp, 0.f) * z;
      }
      __syncthreads();
      for (int byte = 3; byte >= 0; --byte)
        radix_pass(lr, V, vocab_off, it, lst, ll, mk, byte, false, vmax, thr, &s_prefix, &s_need, hist);
      thr = s_prefix > thr ? s_prefix : thr;
    }
    __syncthreads();
  }

  if (cand) {
    // ---- rank-local candidates (v >= thr, at most 256 gathered), sorted (v desc, id asc)
    if (threadIdx.x == 0) s_nc = 0;
    for (int k = threadIdx.x; k < 256; k += blockDim.x) {
      c_v[k] = -INFINITY;
      c_i[k] = 0x7fffffff;
    }
    __syncthreads();
    // keys above the threshold (fewer than keff <= 256 of them: every one is
    // kept, and the sort below fixes their order), then the ties AT the
    // threshold into the remaining slots in a fixed order: a block-wide scan of
    // per-thread tie counts, each thread's ties in its own id order (an
    // atomic-arrival fill kept an arbitrary subset when > 256 tokens tie)
    int my_ties = 0;
    for_allowed(lr, V, vocab_off, it, lst, ll, mk, [&](int gi, float v) {
      const uint32_t k = okey(v);
      if (k < thr) return;
      if (k == thr) {
        ++my_ties;
        return;
      }
      const int slot = atomicAdd(&s_nc, 1);
      if (slot < 256) {
        c_v[slot] = v;
        c_i[slot] = gi;
      }
    });
    __syncthreads();
    const int n_above = min(s_nc, 256);
    // exclusive scan of my_ties over the block (wave scan + per-wave totals in LDS)
    int incl = my_ties;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if ((threadIdx.x & 63) >= o) incl += t;
    }
    if ((threadIdx.x & 63) == 63) si[threadIdx.x >> 6] = incl;
    __syncthreads();
    int wave_off = 0;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) wave_off += si[w];
    int pos = n_above + wave_off + incl - my_ties;
    if (my_ties && pos < 256) {
      for_allowed(lr, V, vocab_off, it, lst, ll, mk, [&](int gi, float v) {
        if (okey(v) != thr || pos >= 256) return;
        c_v[pos] = v;
        c_i[pos] = gi;
        ++pos;
      });
    }
    __syncthreads();
    // bitonic sort of 256 (v desc, id asc)
    for (int size = 2; size <= 256; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = threadIdx.x; t < 256; t += blockDim.x) {
          const int o = t ^ stride;
          if (o > t) {
            const bool desc = (t & size) == 0;
            const bool t_first = c_v[t] > c_v[o] || (c_v[t] == c_v[o] && c_i[t] < c_i[o]);
            if (t_first != desc) {
              const float tv = c_v[t];
              c_v[t] = c_v[o];
              c_v[o] = tv;
              const int ti = c_i[t];
              c_i[t] = c_i[o];
              c_i[o] = ti;
            }
          }
        }
        __syncthreads();
      }
    }
    for (int k = threadIdx.x; k < cand_k; k += blockDim.x) {
      const bool ok = k < 256 && c_i[k] != 0x7fffffff;
      float* o = out_cand + ((size_t)row * cand_k + k) * 3;
      o[0] = ok ? c_v[k] : -INFINITY;
      o[1] = ok ? (float)c_i[k] : -1.f;
      o[2] = ok ? (greedy ? c_v[k] : c_v[k] + gumbel(seed, 0u, step, c_i[k])) : -INFINITY;
    }
    if (!out_pair && !out) return;
    __syncthreads();
  }

  // ---- Gumbel-max (or argmax) over the survivors.  A row with a non-finite
  // allowed logit (NaN / +-inf: the model's output went bad) returns kNonFinite
  // (-2), never a token picked from garbage: the engine fails that request
  // loudly (-1 stays "no allowed token").
  Best best{-INFINITY, -1};
  int nonfin = 0;
  for_allowed(lr, V, vocab_off, it, lst, ll, mk, [&](int gi, float v) {
    nonfin |= !(fabsf(v) <= 3.402823466e38f);
    if (filt && okey(v) < thr) return;
    if (!greedy) v += gumbel(seed, 0u, step, gi);
    best = better(best, Best{v, gi});
  });
  const Best b = block_best(best, sv, si);
  const int bad = __syncthreads_or(nonfin);
  if (threadIdx.x == 0) {
    if (out) out[row] = bad ? kNonFinite : b.i;
    // pairs (TP shards): +inf wins the cross-shard max, so the -2 reaches the engine
    if (out_pair) out_pair[row] = bad ? make_float2(INFINITY, (float)kNonFinite) : make_float2(b.v, (float)b.i);
  }
}

}  // namespace k8s

using namespace k8s;

// logits_f32: 1 = fp32 logits, 0 = bf16.  top_k / top_p: per-row (nullptr =
// off; k <= 0 and p >= 1 disable per row).  out_cand [B][cand_k][3] float
// (TP candidate lists, nullptr = off).
K8S_API int k8s_sample(const void* logits, int ld, int B, int V, int vocab_off, const float* temperature,
                       const uint32_t* seeds, const int* steps, const int* mask_id, const uint32_t* mask_table,
                       int mask_words, const int* list_off, const int* list_len, const int* lists, int* out,
                       float* out_pair, hipStream_t s, int logits_f32, const int* top_k, const float* top_p,
                       float* out_cand, int cand_k) {
  if (B <= 0) return 0;
  if (vocab_off % 8 || (vocab_off + V) >= (1 << 24) || (out_cand && (cand_k <= 0 || cand_k > 256)))
    return (int)hipErrorInvalidValue;
  if (logits_f32)
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)logits, ld, V, vocab_off,
                       temperature, seeds, steps, mask_id, mask_table, mask_words, list_off, list_len, lists, top_k,
                       top_p, out, reinterpret_cast<float2*>(out_pair), out_cand, cand_k);
  else
    hipLaunchKernelGGL(sample_kernel<uint16_t>, dim3(B), dim3(256), 0, s, (const uint16_t*)logits, ld, V, vocab_off,
                       temperature, seeds, steps, mask_id, mask_table, mask_words, list_off, list_len, lists, top_k,
                       top_p, out, reinterpret_cast<float2*>(out_pair), out_cand, cand_k);
  return (int)hipGetLastError();
}
