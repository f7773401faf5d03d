// Mixtral MoE routing kernels (B11 router top-k, B12 permute / combine).
#include "common.h"

namespace k8s {

// One wave per token: softmax over E (<= 64) expert logits, top-k by repeated
// wave argmax, renormalise the k weights.  logits bf16 [T][E].
__global__ void __launch_bounds__(256) route_topk_kernel(const uint16_t* __restrict__ logits, int T, int E, int K,
                                                         float* __restrict__ w_out, int* __restrict__ id_out) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  float v = lane < E ? bf2f(logits[(size_t)t * E + lane]) : -INFINITY;
  const float m = wave_max(v);
  const float e = lane < E ? __expf(v - m) : 0.f;
  const float s = wave_sum(e);
  float p = e / s;
  float chosen_sum = 0.f;
  float wk[8];
  int ik[8];
  for (int k = 0; k < K; ++k) {
    float bv = p;
    int bi = lane < E ? lane : 1 << 30;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    wk[k] = bv;
    ik[k] = bi;
    chosen_sum += bv;
    if (lane == bi) p = -1.f;
  }
  if (lane == 0) {
    for (int k = 0; k < K; ++k) {
      w_out[t * K + k] = wk[k] / chosen_sum;
      id_out[t * K + k] = ik[k];
    }
  }
}

// Single-workgroup counting sort of the T*K (token, k) slots by expert.
// order[pos] = slot, inv[slot] = pos, offsets[E+1].
__global__ void __launch_bounds__(1024) moe_align_kernel(const int* __restrict__ ids, int n, int E,
                                                         int* __restrict__ order, int* __restrict__ inv,
                                                         int* __restrict__ offsets) {
  __shared__ int cnt[256];
  __shared__ int base[257];
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    base[0] = 0;
    for (int e = 0; e < E; ++e) base[e + 1] = base[e] + cnt[e];
    for (int e = 0; e <= E; ++e) offsets[e] = base[e];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // stable within a thread's stride, deterministic enough for the combine (uses inv)
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    const int p = base[e] + atomicAdd(&cnt[e], 1);
    order[p] = i;
    inv[i] = p;
  }
}

// out[t] = sum_k w[t,k] * y[inv[t*K+k]]   (bf16 rows of H, fp32 accumulate)
__global__ void __launch_bounds__(256) moe_combine_kernel(const uint16_t* __restrict__ y, const int* __restrict__ inv,
                                                          const float* __restrict__ w, int T, int K, int H,
                                                          uint16_t* __restrict__ out) {
  const int t = blockIdx.x;
  const int nv = H >> 3;
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < K; ++k) {
      const float wk = w[t * K + k];
      const u16x8 v = *reinterpret_cast<const u16x8*>(y + (size_t)inv[t * K + k] * H + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += wk * bf2f(v[j]);
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<u16x8*>(out + (size_t)t * H + c * 8) = o;
  }
}

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_moe_route(const void* logits, int T, int E, int K, float* w_out, int* id_out, hipStream_t s) {
  if (E > 64 || K > 8 || K > E) return (int)hipErrorInvalidValue;
  if (T <= 0) return 0;
  hipLaunchKernelGGL(route_topk_kernel, dim3((T + 3) / 4), dim3(256), 0, s, (const uint16_t*)logits, T, E, K, w_out,
                     id_out);
  return (int)hipGetLastError();
}

K8S_API int k8s_moe_align(const int* ids, int n, int E, int unused, int* order, int* inv, int* offsets, hipStream_t s) {
  if (E > 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(1024), 0, s, ids, n, E, order, inv, offsets);
  return (int)hipGetLastError();
}

K8S_API int k8s_moe_combine(const void* y, const int* inv, const float* w, int T, int K, int H, void* out,
                            hipStream_t s) {
  if (H % 8) return (int)hipErrorInvalidValue;
  if (T <= 0) return 0;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, s, (const uint16_t*)y, inv, w, T, K, H,
                     (uint16_t*)out);
  return (int)hipGetLastError();
}
