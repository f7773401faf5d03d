// Masked sampling over the vocabulary (B9): greedy argmax or exact softmax
// sampling via the Gumbel-max trick in ONE pass over the logits:
//   tok = argmax_i  logit_i / T + G_i,   G_i = -log(-log(U_i)),
// U_i from a counter-based hash of (seed, step, i) -> reproducible and
// graph-capturable (the seed/step live in device memory).  The per-request
// seed already includes the sequence id, so the noise does not depend on the
// row's position in the batch: a sequence samples the same tokens however the
// scheduler batches it (sync or overlapped steps, any batch mix).
// Constrained decoding masks (grammar states) come in two forms per row:
//   * bitmap: mask_table[mask_id[row]] is a [V/32] uint32 allow-bitmap
//   * list:   an explicit allow-list slice (list_off, list_len) of token ids
// Logits are bf16 [B][ld]; one 256-thread workgroup per row.
// Vocab-parallel (TP) form: the rank holds columns [vocab_off, vocab_off + V)
// of the vocabulary; noise and masks are keyed by the GLOBAL token id, so the
// per-rank (score, id) winners combined by max over ranks give exactly the
// token the unsharded kernel would sample (B10 without a logits all-gather).
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

struct Best {
  float v;
  int i;
};

__device__ __forceinline__ Best better(Best a, Best b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i && b.i >= 0)) return b;
  return a;
}

__global__ void __launch_bounds__(256) sample_kernel(const uint16_t* __restrict__ logits, int ld, int V, int vocab_off,
                                                     const float* __restrict__ temperature,
                                                     const uint32_t* __restrict__ seeds,
                                                     const int* __restrict__ steps,
                                                     const int* __restrict__ mask_id,
                                                     const uint32_t* __restrict__ mask_table, int mask_words,
                                                     const int* __restrict__ list_off, const int* __restrict__ list_len,
                                                     const int* __restrict__ lists, int* __restrict__ out,
                                                     float2* __restrict__ out_pair) {
  const int row = blockIdx.x;
  const uint16_t* lr = logits + (size_t)row * ld;
  const float temp = temperature ? temperature[row] : 0.f;
  const bool greedy = !(temp > 0.f);
  const float it = greedy ? 1.f : 1.f / temp;
  const uint32_t seed = seeds ? seeds[row] : 0u;
  const uint32_t step = steps ? (uint32_t)steps[row] : 0u;
  Best best{-INFINITY, -1};
  const int ll = list_len ? list_len[row] : 0;
  if (ll > 0) {
    const int* lst = lists + list_off[row];
    for (int k = threadIdx.x; k < ll; k += blockDim.x) {
      const int gi = lst[k];
      const int i = gi - vocab_off;
      if (i < 0 || i >= V) continue;
      float v = bf2f(lr[i]) * it;
      if (!greedy) v += gumbel(seed, 0u, step, gi);
      best = better(best, Best{v, gi});
    }
  } else {
    const int mid = mask_id ? mask_id[row] : -1;
    const uint32_t* mk = (mid >= 0) ? mask_table + (size_t)mid * mask_words : nullptr;
    const int nv = V >> 3;
    for (int c = threadIdx.x; c < nv; c += blockDim.x) {
      const int i0 = c * 8, g0 = vocab_off + i0;  // vocab_off % 8 == 0 (host-checked)
      uint32_t bits = 0xFFu;
      if (mk) bits = (mk[g0 >> 5] >> (g0 & 31)) & 0xFFu;
      if (!bits) continue;
      u16x8 x = *reinterpret_cast<const u16x8*>(lr + i0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!((bits >> j) & 1u)) continue;
        float v = bf2f(x[j]) * it;
        if (!greedy) v += gumbel(seed, 0u, step, g0 + j);
        best = better(best, Best{v, g0 + j});
      }
    }
    for (int i = (nv << 3) + threadIdx.x; i < V; i += blockDim.x) {  // tail (V % 8)
      const int gi = vocab_off + i;
      if (mk && !((mk[gi >> 5] >> (gi & 31)) & 1u)) continue;
      float v = bf2f(lr[i]) * it;
      if (!greedy) v += gumbel(seed, 0u, step, gi);
      best = better(best, Best{v, gi});
    }
  }
  // block argmax
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Best other{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, other);
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sv[w] = best.v;
    si[w] = best.i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    Best b{sv[0], si[0]};
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) b = better(b, Best{sv[k], si[k]});
    if (out) out[row] = b.i;
    if (out_pair) out_pair[row] = make_float2(b.v, (float)b.i);  // ids < 2^24: exact in f32
  }
}

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_sample(const void* logits, int ld, int B, int V, int vocab_off, const float* temperature,
                       const uint32_t* seeds, const int* steps, const int* mask_id, const uint32_t* mask_table,
                       int mask_words, const int* list_off, const int* list_len, const int* lists, int* out,
                       float* out_pair, hipStream_t s) {
  if (B <= 0) return 0;
  if (vocab_off % 8 || (vocab_off + V) >= (1 << 24)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(256), 0, s, (const uint16_t*)logits, ld, V, vocab_off, temperature,
                     seeds, steps, mask_id, mask_table, mask_words, list_off, list_len, lists, out,
                     reinterpret_cast<float2*>(out_pair));
  return (int)hipGetLastError();
}
