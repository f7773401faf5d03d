// Shared helpers for the CDNA4 (gfx950) kernels of k8s_llm_rca_amd.
// wave64 everywhere; bf16 stored as raw 16-bit words and converted with the
// hardware round-to-nearest-even path (v_cvt_pk_bf16_f32 at -O3).
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#define K8S_API extern "C" __attribute__((visibility("default")))

namespace k8s {

constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

// Weight-stream loads into VGPRs: every weight byte is read once per step and
// never re-read by the launch, so they carry the non-temporal policy (nt), as
// MI355X_MICROARCH.md measures for weight-streaming decode kernels (34.5 ->
// 30.6-30.8 us per Llama-3.2-1B layer).  Measured here, interleaved A/B
// (profiles/r2_nt_ab/): Llama-3-8B per-layer projections at M = 8 / 16 / 32
// 91.8-93.4 / 93.7-95.9 / 98.7-100.1 us vs 98.1-103.6 / 99.6-100.0 /
// 103.5-104.3 us with the default policy.  Activations keep the default policy.
#ifndef K8S_W_NT
#define K8S_W_NT 1
#endif
template <typename V>
__device__ __forceinline__ V ldw_nt(const void* p) {
#if K8S_W_NT
  return __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
#else
  return *reinterpret_cast<const V*>(p);
#endif
}

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// RoPE of one (x[i], x[i + 64]) pair in a fixed operation order -- no choice
// left to the compiler's contraction -- so every kernel that rotates (rope_kv,
// the skinny and the prefill qkv GEMM epilogues) rounds identically.
__device__ __forceinline__ void rope_pair(float a, float b, float co, float si, float& lo, float& hi) {
  lo = fmaf(a, co, -__fmul_rn(b, si));
  hi = fmaf(b, co, __fmul_rn(a, si));
}

// Sum of the `splits` fp32 partials of 8 consecutive outputs, p[s * stride ..
// + 8) for s < splits, in split order (p0 + p1 + p2 ...).  For splits <= 4 every
// load is issued before the first add (unconditional: past the last split the
// address is clamped to it -- an L2 hit that is not added), so a row of a
// split-K consumer pays one memory latency instead of `splits` dependent ones;
// the arithmetic, and hence every bit, is the plain loop's.
__device__ __forceinline__ void sum_splits8(const float* p, size_t stride, int splits, f32x4& a0, f32x4& a1) {
  constexpr int kPre = 4;
  if (splits <= kPre) {
    f32x4 b0[kPre], b1[kPre];
#pragma unroll
    for (int sp = 0; sp < kPre; ++sp) {
      const float* q = p + (size_t)(sp < splits ? sp : splits - 1) * stride;
      b0[sp] = *reinterpret_cast<const f32x4*>(q);
      b1[sp] = *reinterpret_cast<const f32x4*>(q + 4);
    }
    a0 = b0[0];
    a1 = b1[0];
#pragma unroll
    for (int sp = 1; sp < kPre; ++sp)
      if (sp < splits) {
        a0 += b0[sp];
        a1 += b1[sp];
      }
    return;
  }
  a0 = *reinterpret_cast<const f32x4*>(p);
  a1 = *reinterpret_cast<const f32x4*>(p + 4);
  for (int sp = 1; sp < splits; ++sp) {
    a0 += *reinterpret_cast<const f32x4*>(p + sp * stride);
    a1 += *reinterpret_cast<const f32x4*>(p + sp * stride + 4);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x <= 1024 (scratch: >= 16 floats of LDS)
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// Hand-issued LDS fragment reads.  In the LDS-DMA kernels hipcc waits lgkmcnt(0)
// before every MFMA that consumes an LDS fragment (it does not count the reads
// behind the DMA traffic), exposing one LDS latency per fragment group; an asm read is invisible to its
// waitcnt pass, so each consumer gets an explicit counted wait instead, which
// "rewrites" the fragments it covers so the MFMA cannot be hoisted above it
// (cdna_hip_programming.md §5.7: an asm statement's memory traffic is not modelled).
template <int OFF>
// Hand-issued ds_read_b128 for counted lgkmcnt waits (lgkm_wait<N>): the
// caller must keep scalar memory loads out of the window between its reads and
// their waits (lgkmcnt counts them too, out of order) -- a sched_barrier(0)
// before the read block and after the consuming MFMAs (gemm_stream.hip
// glds_strip, attention.hip's page loop).
__device__ __forceinline__ bf16x8 lds_rd16(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}

// TP push epilogue (allreduce.hip "push" section): where a row-parallel GEMM
// (o / down projection at decode sizes) stores its bf16 output tile straight
// into the peers' IPC staging slots instead of its own output buffer, then
// raises one flag per output strip.  Filled on the host by k8s_ar_push_desc;
// the parity half of the slots follows the communicator's device-side epoch,
// read by the kernel itself (HIP-graph capturable).
struct K8sPush {
  unsigned char* base[8];  // every rank's mapped communicator buffer
  int world, rank;
  int two_shot;            // 0: the whole tile to every rank; 1: each strip to the owner of its columns
  int H;                   // row length of the output (= N of the GEMM)
  long slot;               // bytes per (source rank) slot
  long region;             // byte offset of the parity-0 slots; parity 1 follows at + world * slot
  long flags;              // byte offset of the per-(source rank, strip) flags
  long epoch;              // byte offset of the epoch word
};
constexpr int kPushMaxStrips = 256;

// Output strips of a push GEMM (the flag count the consumer waits for): the
// LDS-DMA kernel's strip width (128 columns for cfg 23 / 24, else 64); the
// split-K reduce pass always works on 64-column strips.
__host__ __device__ inline int k8s_push_strips(int cfg, int splits, int N) {
  return N / ((splits == 1 && cfg > 20) ? 128 : 64);
}

__device__ __forceinline__ uint32_t push_epoch(const K8sPush& P) {
  return __hip_atomic_load(reinterpret_cast<uint32_t*>(P.base[P.rank] + P.epoch), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// Store 8 outputs (row m, columns n .. n + 7) of this rank's partial where the
// consumer reads them: one-shot -> slot [rank] of every rank ([T][H] rows);
// two-shot -> slot [rank] of the owner of column n only ([T][H / world] rows
// of the owner's column slice).
__device__ __forceinline__ void push_store8(const K8sPush& P, uint32_t e, int m, int n, const u16x8& v) {
  const size_t par = P.region + (size_t)(e & 1u) * P.world * P.slot + (size_t)P.rank * P.slot;
  if (P.two_shot) {
    const int w = P.H / P.world, o = n / w;
    *reinterpret_cast<u16x8*>(P.base[o] + par + 2 * ((size_t)m * w + (n - o * w))) = v;
  } else {
    for (int p = 0; p < P.world; ++p)
      *reinterpret_cast<u16x8*>(P.base[p] + par + 2 * ((size_t)m * P.H + n)) = v;
  }
}

// After every thread's push_store8 of strip `s` (columns n0 ..): drain the
// stores, ONE system-scope release, then the strip's flag in every rank
// (one-shot) or in the owner (two-shot) -- the all-reduce's ar_publish
// (explicit vmcnt(0) behind the fence, lane-addressed vector stores).
__device__ __forceinline__ void push_publish(const K8sPush& P, uint32_t e, int s, int n0) {
  const int t = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // lane t signals rank t (lane-addressed: a vector store, as in ar_publish)
    if (P.two_shot ? t == n0 / (P.H / P.world) : t < P.world) {
      uint32_t* f = reinterpret_cast<uint32_t*>(P.base[t] + P.flags) + P.rank * kPushMaxStrips + s;
      __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}


}  // namespace k8s
