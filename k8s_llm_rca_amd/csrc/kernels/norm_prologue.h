// RMSNorm prologue for the decode-size projection GEMMs at a few rows.
//
// At concurrency 1-4 a decode layer is ~8 launches of a few microseconds each,
// and every one pays a fixed start / drain latency however little it moves
// (the two residual-add + RMSNorm launches of a layer: ~5 us each at one row,
// profiles/r5/c1/).  A GEMM whose input is a norm's output can compute that
// norm itself: each workgroup normalises the (<= 4) rows it needs into LDS
// while its first weight chunks are already in flight, and reads its X
// operand from LDS instead of L2.  The arithmetic is rmsnorm_kernel's
// (norm_act.hip) step for step -- thread t of the first 256 owns 16-byte
// pieces t, t + 256, ..; the same fp32 order for the square sum, the same
// block_sum tree (the extra waves of a 512-thread block add exact zeros), the
// same bf16 roundings -- so the fused form is bit-identical to
// rmsnorm + GEMM.
//
// The residual: rows of `x` (bf16, stride x_stride) or, with `part`, the
// fp32 split-K partials [splits][M][H] of the producing GEMM (summed in the
// reduce kernels' order, as rmsnorm_kernel<., true>) are added to `res_in`;
// the sum is written to `res_out` by ONE workgroup (`store`).  res_out is a
// different buffer from res_in (the executor ping-pongs two residual
// buffers): every other workgroup is still reading res_in.  res_in == nullptr
// is the first layer's plain norm of `x` (no add, nothing stored).
#pragma once
#include "common.h"

namespace k8s {

constexpr int kNormMaxRows = 4;    // rows a fused-norm launch accepts
constexpr int kNormMaxChunks = 2;  // H <= 2 * 256 * 8 = 4096 (more would cost the skinny kernel its 2nd workgroup per CU)

struct NormIn {
  const uint16_t* x;    // [M][x_stride] bf16, or null with part
  const float* part;    // [splits][M][H] fp32 partials, or null
  const uint16_t* res_in;
  uint16_t* res_out;
  const uint16_t* w;    // norm weight [H]
  int x_stride, splits, H;
  float eps;
};

extern __shared__ __attribute__((aligned(16))) uint16_t k8s_norm_lds[];  // [M][H] bf16 (dynamic LDS)

// all threads of the block call this (it synchronises); rows [0, M) of the
// normed input land in xs[m * H ..].  Two passes over each thread's own
// pieces: the (bf16) sum goes to xs first and is read back after the block
// sum -- bf16-exact, so the same values rmsnorm_kernel keeps in registers,
// without holding a row of fp32 in VGPRs beside the GEMM's weight ring.
__device__ __forceinline__ void norm_rows_to_lds(uint16_t* xs, int M, const NormIn& a, bool store, float* scratch) {
  const int tid = threadIdx.x, nv = a.H >> 3;
  u16x8 wv[kNormMaxChunks];
#pragma unroll
  for (int c = 0; c < kNormMaxChunks; ++c) {
    const int i = tid + c * 256;
    if (tid < 256 && i < nv) wv[c] = *reinterpret_cast<const u16x8*>(a.w + i * 8);
  }
  for (int m = 0; m < M; ++m) {
    float ss = 0.f;
    uint16_t* xr = xs + (size_t)m * a.H;
#pragma unroll
    for (int c = 0; c < kNormMaxChunks; ++c) {
      const int i = tid + c * 256;
      if (tid < 256 && i < nv) {
        u16x8 xa;
        if (a.part) {
          f32x4 a0, a1;
          sum_splits8(a.part + (size_t)m * a.H + i * 8, (size_t)M * a.H, a.splits, a0, a1);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            xa[j] = f2bf(a0[j]);
            xa[j + 4] = f2bf(a1[j]);
          }
        } else {
          xa = *reinterpret_cast<const u16x8*>(a.x + (size_t)m * a.x_stride + i * 8);
        }
        if (a.res_in) {
          const u16x8 b = *reinterpret_cast<const u16x8*>(a.res_in + (size_t)m * a.H + i * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) xa[j] = f2bf(bf2f(xa[j]) + bf2f(b[j]));
          if (store) *reinterpret_cast<u16x8*>(a.res_out + (size_t)m * a.H + i * 8) = xa;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f(xa[j]);
          ss += v * v;
        }
        *reinterpret_cast<u16x8*>(xr + i * 8) = xa;
      }
    }
    const float tot = block_sum(ss, scratch);
    const float inv = rsqrtf(tot / (float)a.H + a.eps);
#pragma unroll
    for (int c = 0; c < kNormMaxChunks; ++c) {
      const int i = tid + c * 256;
      if (tid < 256 && i < nv) {
        const u16x8 sv = *reinterpret_cast<const u16x8*>(xr + i * 8);  // this thread's own pieces
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(sv[j]) * inv * bf2f(wv[c][j]));
        *reinterpret_cast<u16x8*>(xr + i * 8) = o;
      }
    }
    __syncthreads();  // scratch is reused by the next row's block_sum; xs complete for the readers
  }
}

}  // namespace k8s
