// MoE grouped GEMM (B13): Y[rows of expert e] = A[rows] . W_e^T, bf16 in/out,
// fp32 accumulate, for every expert e in one launch.  Rows are the permuted
// (token, slot) rows, contiguous per expert: expert e owns rows
// offsets[e] .. offsets[e+1] (device array from moe_align -> no host sync,
// HIP-graph capturable).  W is [E][N][K] row-major.
//
// Grid (N / 128, max_tiles): workgroup (nb, j) finds its (expert, 64-row tile)
// by walking the E tile counts; surplus workgroups exit.  4 waves as 2 (M) x
// 2 (N), 32 x 64 each; k-tiles of 64 through XOR-swizzled LDS (chunk c of row
// r at c ^ (r & 7): conflict-free ds_read_b128 / ds_write_b128 for these
// patterns), register-staged double buffer, one barrier per k-tile.
// v_mfma_f32_16x16x32_bf16 with A = W rows, B = X^T: each lane ends with 4
// consecutive output columns of one row (8-byte stores).
// FUSE_SILU: A[m][k] = silu(G[m][k]) * U[m][k] computed while staging, with
// G|U the gate_up output [rows][2K] (the down projection never materialises
// the activation).
// Split-K (gridDim.z > 1): workgroup z covers k in [z K/Z, (z+1) K/Z) and
// writes fp32 partials part[z][row][n]; grouped_reduce_kernel sums them.  The
// down projection (N = 4096, K = 14336) has only N/128 = 32 column tiles per
// expert, i.e. ~256 workgroups for a decode batch -- one per CU, too few
// loads in flight (3.9 TB/s); Z = 4 gives ~1k workgroups while the partials
// (rows x N x 4 B x Z, a few MB) stay tiny next to the ~0.9 GB of expert
// weights a decode step streams.
#include "common.h"

namespace k8s {

constexpr int GG_BM = 64, GG_BN = 128, GG_BK = 64;

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

template <bool FUSE_SILU>
__global__ void __launch_bounds__(256, 2) grouped_gemm_kernel(const uint16_t* __restrict__ a, int lda,
                                                              const uint16_t* __restrict__ w,
                                                              uint16_t* __restrict__ y, int ldy,
                                                              const int* __restrict__ offsets, int E, int N, int K,
                                                              float* __restrict__ part, int total_rows) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][GG_BM * GG_BK];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][GG_BN * GG_BK];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int r = lane & 15, h = lane >> 4;
  // ---- which (expert, m-tile) is this workgroup?
  int j = blockIdx.y, e = 0, row0 = 0, rows = 0;
  for (; e < E; ++e) {
    const int a0 = offsets[e], a1 = offsets[e + 1];
    const int t = (a1 - a0 + GG_BM - 1) / GG_BM;
    if (j < t) {
      row0 = a0 + j * GG_BM;
      rows = min(GG_BM, a1 - row0);
      break;
    }
    j -= t;
  }
  if (e >= E || rows <= 0) return;  // workgroup-uniform
  const int n0 = blockIdx.x * GG_BN;
  const int kslice = K / gridDim.z, kbase = blockIdx.z * kslice;
  const uint16_t* we = w + ((size_t)e * N + n0) * K + kbase;

  // staging: A 64x64 = 512 chunks (2 / thread), B 128x64 = 1024 chunks (4 / thread)
  bf16x8 sa[FUSE_SILU ? 4 : 2], sb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      const int m = row0 + min(row, rows - 1);
      const uint16_t* p = a + (size_t)m * lda + kbase + k0 + 8 * c;
      if constexpr (FUSE_SILU) {
        sa[2 * i] = *reinterpret_cast<const bf16x8*>(p);          // gate
        sa[2 * i + 1] = *reinterpret_cast<const bf16x8*>(p + K);  // up
      } else {
        sa[i] = *reinterpret_cast<const bf16x8*>(p);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      sb[i] = ldw_nt<bf16x8>(we + (size_t)row * K + k0 + 8 * c);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      bf16x8 v;
      if constexpr (FUSE_SILU) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (__bf16)(silu_f((float)sa[2 * i][t]) * (float)sa[2 * i + 1][t]);
      } else {
        v = sa[i];
      }
      *reinterpret_cast<bf16x8*>(&sA[buf][row * GG_BK + 8 * (c ^ (row & 7))]) = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = q & 7;
      *reinterpret_cast<bf16x8*>(&sB[buf][row * GG_BK + 8 * (c ^ (row & 7))]) = sb[i];
    }
  };

  f32x4 acc[4][2];  // [n-tile][m-tile]: C^T[n][m]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kslice / GG_BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    load(min(kt + 1, nk - 1) * GG_BK);  // unconditional prefetch (last one re-reads)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 4 * ks + h;
      bf16x8 xf[2], wf[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int row = 32 * wm + 16 * mt + r;
        xf[mt] = *reinterpret_cast<const bf16x8*>(&sA[buf][row * GG_BK + 8 * (c ^ (row & 7))]);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int row = 64 * wn + 16 * nt + r;
        wf[nt] = *reinterpret_cast<const bf16x8*>(&sB[buf][row * GG_BK + 8 * (c ^ (row & 7))]);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt], xf[mt], acc[nt][mt], 0, 0, 0);
    }
    store(buf ^ 1);
    __syncthreads();
  }
  // acc[nt][mt][i] = C[m = 32wm + 16mt + r][n = 64wn + 16nt + 4h + i]
  if (gridDim.z > 1) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = 32 * wm + 16 * mt + r;
      if (m >= rows) continue;
      float* pr = part + ((size_t)blockIdx.z * total_rows + row0 + m) * N + n0 + 64 * wn + 4 * h;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) *reinterpret_cast<f32x4*>(pr + 16 * nt) = acc[nt][mt];
    }
    return;
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = 32 * wm + 16 * mt + r;
    if (m >= rows) continue;
    uint16_t* yr = y + (size_t)(row0 + m) * ldy + n0 + 64 * wn + 4 * h;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      u16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(acc[nt][mt][i]);
      *reinterpret_cast<u16x4*>(yr + 16 * nt) = v;
    }
  }
}

// y[row][n] = bf16(sum_z part[z][row][n]) over the rows < offsets[E]
__global__ void __launch_bounds__(256) grouped_reduce_kernel(const float* __restrict__ part, int splits,
                                                             uint16_t* __restrict__ y, int ldy,
                                                             const int* __restrict__ offsets, int E, int N,
                                                             int total_rows) {
  const int used = offsets[E];
  const size_t RN = (size_t)total_rows * N;
  for (size_t idx = (size_t)(blockIdx.x * 256 + threadIdx.x) * 8; idx < (size_t)used * N;
       idx += (size_t)gridDim.x * 256 * 8) {
    const size_t row = idx / N, n = idx % N;
    f32x4 a0 = *reinterpret_cast<const f32x4*>(part + idx);
    f32x4 a1 = *reinterpret_cast<const f32x4*>(part + idx + 4);
    for (int z = 1; z < splits; ++z) {
      a0 += *reinterpret_cast<const f32x4*>(part + z * RN + idx);
      a1 += *reinterpret_cast<const f32x4*>(part + z * RN + idx + 4);
    }
    u16x8 o;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      o[v] = f2bf(a0[v]);
      o[v + 4] = f2bf(a1[v]);
    }
    *reinterpret_cast<u16x8*>(y + row * ldy + n) = o;
  }
}

}  // namespace k8s

using namespace k8s;

// max_tiles >= sum_e ceil(rows_e / 64); ceil(total_rows / 64) + E always is.
// splits > 1: part = splits * total_rows * N fp32 scratch (total_rows = rows
// of `a`, >= offsets[E]); K % (64 * splits) == 0.
static int launch_grouped(const void* a, int lda, const void* w, void* y, int ldy, const int* offsets, int E, int N,
                          int K, int max_tiles, int fuse_silu, int splits, void* part, int total_rows, bool reduce,
                          hipStream_t s) {
  if (N % GG_BN || K % (GG_BK * splits) || E <= 0 || max_tiles <= 0 || splits < 1 || (splits > 1 && !part) ||
      N % 8 || ldy % 8)
    return (int)hipErrorInvalidValue;
  const dim3 grid(N / GG_BN, max_tiles, splits);
  float* pp = (float*)part;
  if (fuse_silu)
    hipLaunchKernelGGL(grouped_gemm_kernel<true>, grid, dim3(256), 0, s, (const uint16_t*)a, lda,
                       (const uint16_t*)w, (uint16_t*)y, ldy, offsets, E, N, K, pp, total_rows);
  else
    hipLaunchKernelGGL(grouped_gemm_kernel<false>, grid, dim3(256), 0, s, (const uint16_t*)a, lda,
                       (const uint16_t*)w, (uint16_t*)y, ldy, offsets, E, N, K, pp, total_rows);
  if (splits > 1 && reduce) {
    const int blocks = min(2048, (int)(((size_t)total_rows * N / 8 + 255) / 256));
    hipLaunchKernelGGL(grouped_reduce_kernel, dim3(max(blocks, 1)), dim3(256), 0, s, (const float*)pp, splits,
                       (uint16_t*)y, ldy, offsets, E, N, total_rows);
  }
  return (int)hipGetLastError();
}

K8S_API int k8s_grouped_gemm(const void* a, int lda, const void* w, void* y, int ldy, const int* offsets, int E,
                             int N, int K, int max_tiles, int fuse_silu, int splits, void* part, int total_rows,
                             hipStream_t s) {
  return launch_grouped(a, lda, w, y, ldy, offsets, E, N, K, max_tiles, fuse_silu, splits, part, total_rows, true, s);
}

// splits > 1: partials [splits][total_rows][N] stay in `part` for a fused consumer
K8S_API int k8s_grouped_gemm_part(const void* a, int lda, const void* w, void* y, int ldy, const int* offsets, int E,
                                  int N, int K, int max_tiles, int fuse_silu, int splits, void* part, int total_rows,
                                  hipStream_t s) {
  return launch_grouped(a, lda, w, y, ldy, offsets, E, N, K, max_tiles, fuse_silu, splits, part, total_rows, false,
                        s);
}
