// Decode-regime projection GEMM, W-shared variant (B4):
//   Y[M][N] = X[M][K] . W[N][K]^T   bf16 in/out, fp32 accumulate, M <= 256.
//
// gemm_mid.hip gives each wave 16*NT output COLUMNS and all M rows, so every
// wave reads every staged X row from LDS per k-step: LDS read traffic grows
// with M (32 KB per 32-deep k-step per 4-wave workgroup at M = 128, 48 KB at
// 192), and that, not HBM, bounds it (profiles/README.md).  Here the roles
// are swapped: a workgroup owns a 64-column strip, and its 4 waves split the
// ROWS (wave w: rows [16*MTW*w, 16*MTW*(w+1))):
//   * W (read once from HBM): each 64-deep k-chunk of the strip (8 KB) is
//     loaded by all 256 threads into a U-chunk register ring (U * 8 KB in
//     flight per workgroup), written once into an XOR-swizzled LDS tile
//     (16-byte piece j of row n at piece j ^ (n & 7): a ds_read_b128 fragment
//     read of 16 rows hits 16 distinct bank slots) and read by the 4 waves:
//     16 KB of LDS reads per 32-deep k-step whatever M is.
//   * X (M x K, a few hundred KB: L2-resident) goes straight from L2 into each
//     wave's own A-fragment registers, prefetched one chunk ahead: no LDS, no
//     sharing needed since each wave owns its rows.
//   * v_mfma_f32_16x16x32_bf16: A = X rows (16 m), B = W^T (16 n); one W
//     fragment read from LDS feeds MTW MFMAs.
//   * split-K over gridDim.y: fp32 partials [split][M][N] reduced by a
//     vectorised kernel, or left for a fused consumer (the next residual add +
//     RMSNorm, k8s_splitk_addnorm) -- the same contract as gemm_mid.
#include "common.h"

namespace k8s {

constexpr int kSC = 64;   // k per chunk
constexpr int kSBN = 64;  // columns per workgroup

__device__ __forceinline__ int sswz(int n, int j) { return j ^ (n & 7); }

template <int MTW, int U>
__global__ void __launch_bounds__(256) gemm_stream_kernel(const uint16_t* __restrict__ x, int ldx,
                                                          const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                          int ldy, float* __restrict__ part, int M, int N, int K,
                                                          int kslice) {
  __shared__ __attribute__((aligned(16))) uint16_t ws[2][kSBN * kSC];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * kSBN;
  const int split = blockIdx.y;
  const int kbeg = split * kslice;
  const int nch = kslice / kSC;
  const int m_base = wv * 16 * MTW;

  // ---- W staging: 512 16-byte pieces per chunk, 2 per thread
  const uint16_t* wsrc[2];
  int wdst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + 256 * i;
    const int n = p >> 3, jl = p & 7;
    wsrc[i] = w + (size_t)(n0 + n) * K + kbeg + 8 * sswz(n, jl);
    wdst[i] = n * kSC + 8 * jl;
  }
  // ---- X fragments: row of frag mt for this lane (clamped; masked at the store)
  const uint16_t* xrow[MTW];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
    const int m = min(m_base + 16 * mt + r, M - 1);
    xrow[mt] = x + (size_t)m * ldx + kbeg + 8 * g;
  }
  const bool active = m_base < M;  // waves past the last row only help stage W

  f32x4 acc[MTW][4];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int cf = 0; cf < 4; ++cf) acc[mt][cf] = f32x4{0.f, 0.f, 0.f, 0.f};

  u16x8 ring[U][2];
  bf16x8 xr[2][2][MTW];
  auto load_w = [&](int slot, int c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ring[slot][i] = *reinterpret_cast<const u16x8*>(wsrc[i] + c * kSC);
  };
  auto store_w = [&](int slot, int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u16x8*>(&ws[buf][wdst[i]]) = ring[slot][i];
  };
  auto load_x = [&](int set, int c) {
    if (!active) return;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
        xr[set][s][mt] = *reinterpret_cast<const bf16x8*>(xrow[mt] + c * kSC + 32 * s);
  };
  auto compute = [&](int buf, int set) {
    if (!active) return;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        const int n = 16 * cf + r;
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(&ws[buf][n * kSC + 8 * sswz(n, 4 * s + g)]);
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
          acc[mt][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xr[set][s][mt], wf, acc[mt][cf], 0, 0, 0);
      }
  };

  // ---- prologue: W chunks 0..U-1 in flight, X chunk 0, W chunk 0 -> LDS
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (u < nch) load_w(u, u);
  load_x(0, 0);
  store_w(0, 0);
  if (U < nch) load_w(0, U);
  __syncthreads();

  // ---- main loop, unrolled by U (even): ring slots and X sets are compile-time
  static_assert(U % 2 == 0, "U must be even");
  for (int c0 = 0; c0 < nch; c0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u;
      if (c < nch) {
        if (c + 1 < nch) load_x((u + 1) & 1, c + 1);
        compute(c & 1, u & 1);
        if (c + 1 < nch) {
          const int slot = (u + 1) % U;
          store_w(slot, (c + 1) & 1);
          if (c + 1 + U < nch) load_w(slot, c + 1 + U);
        }
        __syncthreads();
      }
    }
  }

  // ---- epilogue: acc[mt][cf][v] = C[m = m_base + 16 mt + 4 g + v][n = n0 + 16 cf + r]
  if (!active) return;
  if (gridDim.y == 1) {
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m_base + 16 * mt + 4 * g + v;
        if (m < M) {
#pragma unroll
          for (int cf = 0; cf < 4; ++cf) y[(size_t)m * ldy + n0 + 16 * cf + r] = f2bf(acc[mt][cf][v]);
        }
      }
  } else {
    float* pp = part + (size_t)split * M * N;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m_base + 16 * mt + 4 * g + v;
        if (m < M) {
#pragma unroll
          for (int cf = 0; cf < 4; ++cf) pp[(size_t)m * N + n0 + 16 * cf + r] = acc[mt][cf][v];
        }
      }
  }
}

// Y[m][n] = bf16(sum_s part[s][m][n]); 8 outputs per thread (M * N % 8 == 0).
__global__ void __launch_bounds__(256) gemm_stream_reduce_kernel(const float* __restrict__ part, int splits,
                                                                 uint16_t* __restrict__ y, int ldy, int M, int N) {
  const int idx = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (idx >= M * N) return;
  const int m = idx / N, n = idx % N;
  const size_t MN = (size_t)M * N;
  f32x4 a0 = *reinterpret_cast<const f32x4*>(part + idx);
  f32x4 a1 = *reinterpret_cast<const f32x4*>(part + idx + 4);
  for (int s = 1; s < splits; ++s) {
    a0 += *reinterpret_cast<const f32x4*>(part + s * MN + idx);
    a1 += *reinterpret_cast<const f32x4*>(part + s * MN + idx + 4);
  }
  u16x8 o;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    o[v] = f2bf(a0[v]);
    o[v + 4] = f2bf(a1[v]);
  }
  *reinterpret_cast<u16x8*>(y + (size_t)m * ldy + n) = o;
}

template <int MTW, int U>
static hipError_t launch_stream(dim3 grid, hipStream_t s, const uint16_t* x, int ldx, const uint16_t* w, uint16_t* y,
                                int ldy, float* part, int M, int N, int K, int kslice) {
  hipLaunchKernelGGL((gemm_stream_kernel<MTW, U>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, part, M, N, K, kslice);
  return hipGetLastError();
}

}  // namespace k8s

using namespace k8s;

// cfg: ring depth U (4 or 8).  splits > 1 needs `part` = splits * M * N fp32;
// reduce = 0 leaves the partials for a fused consumer.
static int stream_launch(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                         int splits, void* part, bool reduce, hipStream_t s) {
  if (M <= 0 || M > 256 || N % kSBN || splits < 1 || K % (splits * kSC) || (splits > 1 && part == nullptr) ||
      (cfg != 4 && cfg != 8) || ldx % 8 || (splits > 1 && (M * N) % 8) || (splits == 1 && ldy < N))
    return (int)hipErrorInvalidValue;
  const int kslice = K / splits;
  const int mtw = ((M + 15) / 16 + 3) / 4;  // 16-row fragments per wave (4 waves)
  const dim3 grid(N / kSBN, splits);
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  float* pp = (float*)part;
  hipError_t e;
#define K8S_SL(MT, UU) e = launch_stream<MT, UU>(grid, s, xx, ldx, ww, yy, ldy, pp, M, N, K, kslice)
  if (cfg == 4) {
    switch (mtw) {
      case 1: K8S_SL(1, 4); break;
      case 2: K8S_SL(2, 4); break;
      case 3: K8S_SL(3, 4); break;
      default: K8S_SL(4, 4); break;
    }
  } else {
    switch (mtw) {
      case 1: K8S_SL(1, 8); break;
      case 2: K8S_SL(2, 8); break;
      case 3: K8S_SL(3, 8); break;
      default: K8S_SL(4, 8); break;
    }
  }
#undef K8S_SL
  if (e != hipSuccess) return (int)e;
  if (splits > 1 && reduce) {
    const int blocks = (M * N / 8 + 255) / 256;
    hipLaunchKernelGGL(gemm_stream_reduce_kernel, dim3(blocks), dim3(256), 0, s, (const float*)part, splits, yy, ldy,
                       M, N);
  }
  return (int)hipGetLastError();
}

K8S_API int k8s_gemm_stream(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                            int splits, void* part, hipStream_t s) {
  return stream_launch(x, ldx, w, y, ldy, M, N, K, cfg, splits, part, true, s);
}

K8S_API int k8s_gemm_stream_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                                 int splits, void* part, hipStream_t s) {
  return stream_launch(x, ldx, w, y, ldy, M, N, K, cfg, splits, part, false, s);
}
