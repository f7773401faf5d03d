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
#include "norm_prologue.h"

namespace k8s {

// RoPE + paged KV-write epilogue of the qkv projection (the rope_kv_kernel of
// norm_act.hip folded into the GEMM that produces its input): block b covers
// head b / 8, dims d0 = 8 (b % 8) .. +8 and d0 + 64 .. +8, i.e. its 16 W rows are
// the 8 (i, i + 64) rotation pairs of that head, so the block that finishes a
// pair rotates it, stores it into qkv and (k / v heads) into the KV pages.
// Same arithmetic as rope_kv_kernel on the bf16-rounded GEMM output:
// bit-identical to skinny GEMM + rope_kv.
struct SkinnyRope {
  const int* pos;
  const float* cos_sin;  // [max_pos][128]: cos[0..63] | sin[0..63]
  const int* slots;      // [M] or null (no KV write)
  uint16_t* kc;          // [blocks][nkv][BS][128]
  uint16_t* vc;          // [blocks][nkv][128][BS]
  int nq, nkv, BS;
};

__device__ __forceinline__ int rope_row(int n, int b) {  // W / output row of strip row n in block b
  return (b >> 3) * 128 + (b & 7) * 8 + (n & 7) + (n >= 8 ? 64 : 0);
}

// NORM: X = rmsnorm(nin) computed by the block itself into LDS (norm_prologue.h;
// M <= kNormMaxRows, K == nin.H), after the first U weight loads are issued.
template <int MT, int U, int NW, bool ROPE, bool NORM = false>
__global__ void __launch_bounds__(NW * 64) gemm_skinny_kernel(const uint16_t* __restrict__ x, int ldx,
                                                              const uint16_t* __restrict__ w,
                                                              uint16_t* __restrict__ y, int ldy, int M, int N, int K,
                                                              SkinnyRope rp, NormIn nin = {}) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kq = K / NW;                 // K slice per wave (multiple of 32)
  const int kbeg = wv * kq;
  const uint16_t* wrow = w + (size_t)(ROPE ? rope_row(r, blockIdx.x) : n0 + r) * K + kbeg + 8 * h;
  if constexpr (NORM) {
    x = k8s_norm_lds;
    ldx = K;
  }
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
  if constexpr (NORM) {  // the first weight block in flight while the rows are normalised
    __shared__ float nscr[16];
    if (nblk > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) wa[u] = ldw_nt<bf16x8>(wrow + u * 32);
    }
    norm_rows_to_lds(k8s_norm_lds, M, nin, blockIdx.x == 0, nscr);
    if (nblk > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xa[u][mt] = *reinterpret_cast<const bf16x8*>(xrow[mt] + u * 32);
    }
  }
  if (nblk > 0) {
    if constexpr (!NORM) load(wa, xa, 0);
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
  if constexpr (ROPE) {
    const int hd = blockIdx.x >> 3, d0 = (blockIdx.x & 7) * 8;
    for (int e = threadIdx.x; e < 8 * 16 * MT; e += NW * 64) {
      const int j = e & 7, m = e >> 3;
      if (m >= M) continue;
      float lo = 0.f, hi = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        lo += red[q][j][m];
        hi += red[q][j + 8][m];
      }
      const int d = d0 + j;
      uint16_t a = f2bf(lo), b = f2bf(hi);
      if (hd < rp.nq + rp.nkv) {  // q / k head: rotate-half pair (d, d + 64)
        const float* cs = rp.cos_sin + (size_t)rp.pos[m] * 128;
        const float co = cs[d], si = cs[64 + d], fa = bf2f(a), fb = bf2f(b);
        float ra, rb;
        rope_pair(fa, fb, co, si, ra, rb);
        a = f2bf(ra);
        b = f2bf(rb);
      }
      uint16_t* yr = y + (size_t)m * ldy + hd * 128;
      yr[d] = a;
      yr[d + 64] = b;
      const int slot = rp.slots ? rp.slots[m] : -1;
      if (slot < 0 || hd < rp.nq) continue;
      const int blk = slot / rp.BS, off = slot % rp.BS;
      if (hd < rp.nq + rp.nkv) {
        uint16_t* kp = rp.kc + (((size_t)blk * rp.nkv + (hd - rp.nq)) * rp.BS + off) * 128;
        kp[d] = a;
        kp[d + 64] = b;
      } else {
        uint16_t* vp = rp.vc + ((size_t)blk * rp.nkv + (hd - rp.nq - rp.nkv)) * 128 * rp.BS + off;
        vp[(size_t)d * rp.BS] = a;
        vp[(size_t)(d + 64) * rp.BS] = b;
      }
    }
    return;
  }
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
  const SkinnyRope rp{};
  if (M <= 16)
    hipLaunchKernelGGL((gemm_skinny_kernel<1, 4, 8, false>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K, rp);
  else if (M <= 32)
    hipLaunchKernelGGL((gemm_skinny_kernel<2, 4, 8, false>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K, rp);
  else if (M <= 64)
    hipLaunchKernelGGL((gemm_skinny_kernel<4, 2, 8, false>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K, rp);
  else
    hipLaunchKernelGGL((gemm_skinny_kernel<8, 1, 8, false>), g, dim3(512), 0, s, xx, ldx, ww, yy, ldy, M, N, K, rp);
  return (int)hipGetLastError();
}

// qkv = x . w^T (w = [q heads; k heads; v heads] x 128 rows, N = (nq + 2 nkv) 128)
// with the RoPE + paged KV write of k8s_rope_kv fused into the epilogue
// (M <= 16; bit-identical to k8s_gemm_skinny + k8s_rope_kv).
K8S_API int k8s_gemm_skinny_rope(const void* x, int ldx, const void* w, void* qkv, int ldq, int M, int N, int K,
                                 const int* pos, const float* cos_sin, const int* slots, void* kc, void* vc, int nq,
                                 int nkv, int BS, hipStream_t s) {
  if (M <= 0 || M > 16 || K % 256 || N != (nq + 2 * nkv) * 128 || ldq < N || !pos || !cos_sin || BS <= 0)
    return (int)hipErrorInvalidValue;
  const SkinnyRope rp{pos, cos_sin, slots, (uint16_t*)kc, (uint16_t*)vc, nq, nkv, BS};
  hipLaunchKernelGGL((gemm_skinny_kernel<1, 4, 8, true>), dim3(N / 16), dim3(512), 0, s, (const uint16_t*)x, ldx,
                     (const uint16_t*)w, (uint16_t*)qkv, ldq, M, N, K, rp);
  return (int)hipGetLastError();
}

// k8s_gemm_skinny_rope on X = rmsnorm(x [or the split-K partials `part`] + res_in) * norm_w,
// computed by every workgroup into LDS (norm_prologue.h): bit-identical to
// k8s_rmsnorm / k8s_splitk_addnorm + k8s_gemm_skinny_rope, one launch fewer.  res_in
// null: the plain norm of x (first layer).  Otherwise res_out (!= res_in) <- x + res_in.
K8S_API int k8s_gemm_skinny_rope_norm(const void* x, int x_stride, const float* part, int splits, const void* res_in,
                                      void* res_out, const void* norm_w, float eps, const void* w, void* qkv, int ldq,
                                      int M, int N, int K, const int* pos, const float* cos_sin, const int* slots,
                                      void* kc, void* vc, int nq, int nkv, int BS, hipStream_t s) {
  if (M <= 0 || M > kNormMaxRows || K % 256 || K / 8 > 256 * kNormMaxChunks || N != (nq + 2 * nkv) * 128 ||
      ldq < N || !pos || !cos_sin || BS <= 0 || !norm_w || (!x && !part) || (part && (splits < 1 || !res_in)) ||
      (res_in && (!res_out || res_out == res_in)))
    return (int)hipErrorInvalidValue;
  const SkinnyRope rp{pos, cos_sin, slots, (uint16_t*)kc, (uint16_t*)vc, nq, nkv, BS};
  const NormIn nin{(const uint16_t*)x, part, (const uint16_t*)res_in, (uint16_t*)res_out, (const uint16_t*)norm_w,
                   x_stride, splits, K, eps};
  hipLaunchKernelGGL((gemm_skinny_kernel<1, 4, 8, true, true>), dim3(N / 16), dim3(512), (size_t)M * K * 2, s,
                     nullptr, 0, (const uint16_t*)w, (uint16_t*)qkv, ldq, M, N, K, rp, nin);
  return (int)hipGetLastError();
}
