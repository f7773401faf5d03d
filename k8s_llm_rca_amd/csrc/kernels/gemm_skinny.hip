// Decode-shape projection GEMM (B4, M <= 128): Y[M][N] = X[M][K] . W[N][K]^T, bf16
// in/out, fp32 accumulate, for the weight-streaming regime where hipBLASLt
// leaves HBM idle at small N (o_proj 4096x4096 ran at 1.65 TB/s).
//
// Workgroup = 16 weight rows x all M, 4 waves split K into contiguous quarters.
// Each wave streams its 16 x K/4 weight slab HBM -> VGPRs (no LDS round trip:
// the slab is read exactly once, cdna_hip_programming.md 'GEMV / M <= 16'),
// issuing U k-steps of loads before the MFMAs, and re-reads the small X from
// L2.  MFMA v_mfma_f32_16x16x32_bf16 with A = W rows, B = X^T: one W fragment
// feeds MT MFMAs (MT = ceil(M/16) m-tiles).  The 4 K-quarters are summed through
// LDS and written as bf16.  Grid = N/16 workgroups (256 for N = 4096: one per CU).
#include "common.h"

namespace k8s {

template <int MT, int U, int NW>
__global__ void __launch_bounds__(NW * 64) gemm_skinny_kernel(const uint16_t* __restrict__ x, int ldx,
                                                              const uint16_t* __restrict__ w,
                                                              uint16_t* __restrict__ y, int ldy, int M, int N, int K) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kq = K / NW;                 // K slice per wave (multiple of 32)
  const int kbeg = wv * kq;
  const uint16_t* wrow = w + (size_t)(n0 + r) * K + kbeg + 8 * h;
  const uint16_t* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = min(mt * 16 + r, M - 1);
    xrow[mt] = x + (size_t)m * ldx + kbeg + 8 * h;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = kq >> 5;
  // software pipeline: block b+1's loads are in flight while block b's MFMAs run
  bf16x8 wa[U], wb[U];
  bf16x8 xa[U][MT], xb[U][MT];
  auto load = [&](bf16x8 (&wf)[U], bf16x8 (&xf)[U][MT], int s0) {
#pragma unroll
    for (int u = 0; u < U; ++u) wf[u] = ldw_nt<bf16x8>(wrow + (s0 + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xf[u][mt] = *reinterpret_cast<const bf16x8*>(xrow[mt] + (s0 + u) * 32);
  };
  auto mma = [&](bf16x8 (&wf)[U], bf16x8 (&xf)[U][MT]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u], xf[u][mt], acc[mt], 0, 0, 0);
  };
  const int nblk = nsteps / U;
  int s = 0;
  if (nblk > 0) {
    load(wa, xa, 0);
    int b = 0;
    for (; b + 2 <= nblk; b += 2) {
      if (b + 1 < nblk) load(wb, xb, (b + 1) * U);
      mma(wa, xa);
      if (b + 2 < nblk) load(wa, xa, (b + 2) * U);
      mma(wb, xb);
    }
    if (b < nblk) mma(wa, xa);
    s = nblk * U;
  }
  for (; s < nsteps; ++s) {
    const bf16x8 wf = ldw_nt<bf16x8>(wrow + s * 32);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xrow[mt] + s * 32);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf, acc[mt], 0, 0, 0);
    }
  }
  // acc[mt][i] = partial C[n = 4h+i][m = 16mt + r]; sum the NW K-slices in LDS
  __shared__ float red[NW][16][16 * MT + 1];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wv][4 * h + i][16 * mt + r] = acc[mt][i];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * 16 * MT; e += NW * 64) {
    const int n = e & 15, m = e >> 4;
    if (m < M) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) v += red[q][n][m];
      y[(size_t)m * ldy + n0 + n] = f2bf(v);
    }
  }
}

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_gemm_skinny(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K,
                            hipStream_t s) {
  if (M <= 0 || M > 128 || N % 16 || K % 256) return (int)hipErrorInvalidValue;
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  dim3 g(N / 16);
  if (M <= 16)
    hipLaunchKernelGGL((gemm_skinny_kernel<1, 4, 8>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K);
  else if (M <= 32)
    hipLaunchKernelGGL((gemm_skinny_kernel<2, 4, 8>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K);
  else if (M <= 64)
    hipLaunchKernelGGL((gemm_skinny_kernel<4, 2, 8>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K);
  else
    hipLaunchKernelGGL((gemm_skinny_kernel<8, 1, 8>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K);
  return (int)hipGetLastError();
}
