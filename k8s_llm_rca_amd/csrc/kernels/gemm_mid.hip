// Decode-regime projection GEMM for 16 < M <= 256 (B4):
//   Y[M][N] = X[M][K] . W[N][K]^T   bf16 in/out, fp32 accumulate.
//
// At these M the projections are weight-bandwidth bound (M flop per weight
// byte), yet hipBLASLt's solutions leave HBM mostly idle on the Llama-3-8B
// decode shapes: o_proj (4096x4096) runs at 1.3-1.8 TB/s for every M, the
// down projection (4096x14336) at 1.5-2.0 TB/s for M = 128-192
// (tools/gemm_mid_sweep.py, profiles/).  The skinny kernel (M <= 16) re-reads
// X from L2 once per 16 weight rows, so its X traffic grows as M/16.
//
// Structure (one workgroup = NW waves = a BN = 16*NT*NW column strip x one
// K slice):
//   * X: the slice is staged through LDS in 64-deep k-chunks (double
//     buffered, one barrier per chunk) and shared by all NW waves, so X is
//     read from L2 once per workgroup instead of once per wave.  Rows are
//     128 B; 16-byte piece j of row m lives at piece j ^ ((m >> 1) & 7): the
//     16 lanes of a ds_read_b128 quarter (rows 0..15, one piece) then hit 16
//     distinct 16-byte bank slots.
//   * W: each wave streams its NT x 16 weight rows HBM -> VGPRs (read exactly
//     once; no LDS round trip) through a U-chunk-deep register ring, so
//     U * NT * 2 KB per wave are in flight while the MFMAs of older chunks run.
//     Each lane loads 16 B of 4 consecutive k-groups -> a 16-row x 128-B tile
//     (whole cache lines) per chunk.
//   * MFMA v_mfma_f32_16x16x32_bf16 with A = W rows (16 n), B = X^T (16 m):
//     one X fragment read from LDS feeds NT MFMAs, one W fragment feeds MT.
//   * split-K over gridDim.y: slices write fp32 partials [split][M][N] that a
//     vectorised reduce kernel sums into bf16; with one slice the epilogue
//     writes bf16 directly.
#include "common.h"

namespace k8s {

constexpr int kChunk = 64;  // k per LDS stage (2 MFMA k-steps)

__device__ __forceinline__ int swz(int m, int j) { return j ^ ((m >> 1) & 7); }

template <int MT, int NT, int NW, int U, bool SILU>
__global__ void __launch_bounds__(NW * 64) gemm_mid_kernel(const uint16_t* __restrict__ x, int ldx,
                                                           const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ y, int ldy,
                                                           float* __restrict__ part, int M, int N, int K,
                                                           int kslice) {
  constexpr int ROWS = 16 * MT;                 // padded M
  constexpr int PIECES = ROWS * (kChunk / 8);   // 16-byte pieces per X chunk
  constexpr int PPT = (PIECES + NW * 64 - 1) / (NW * 64);
  __shared__ __attribute__((aligned(16))) uint16_t xs[2][ROWS * kChunk];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int n0 = blockIdx.x * (16 * NT * NW) + wv * (16 * NT);
  const int split = blockIdx.y;
  const int kbeg = split * kslice;
  const int nchunks = kslice / kChunk;

  // ---- operand pointers
  const uint16_t* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wrow[nt] = w + (size_t)(n0 + 16 * nt + r) * K + kbeg + 8 * h;
  // SILU: x is the gate_up activation [M][2K] (gate | up) and the operand
  // silu(gate) * up is formed while staging (bit-identical to silu_mul_kernel)
  const uint16_t* xsrc[PPT];
  int xdst[PPT];
  bool xok[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int p = tid + i * NW * 64;
    const int m = p >> 3, j = p & 7;
    xok[i] = p < PIECES;
    xsrc[i] = x + (size_t)min(m, M - 1) * ldx + kbeg + 8 * j;
    xdst[i] = m * kChunk + 8 * swz(m, j);
  }

  f32x4 acc[NT][MT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- W register ring: ring[u][nt][ks] holds chunk (c = u mod U)
  bf16x8 ring[U][NT][2];
  auto load_w = [&](int slot, int c) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        ring[slot][nt][ks] = ldw_nt<bf16x8>(wrow[nt] + c * kChunk + 32 * ks);
  };
  // X: register double buffer, loaded two chunks ahead of its MFMAs (one
  // whole iteration of latency slack before the LDS write that needs it)
  u16x8 xr[2][PPT];
  u16x8 xu[SILU ? 2 : 1][SILU ? PPT : 1];
  auto load_x = [&](int set, int c) {
#pragma unroll
    for (int i = 0; i < PPT; ++i)
      if (xok[i]) {
        xr[set][i] = *reinterpret_cast<const u16x8*>(xsrc[i] + c * kChunk);
        if constexpr (SILU) xu[set][i] = *reinterpret_cast<const u16x8*>(xsrc[i] + K + c * kChunk);
      }
  };
  auto store_x = [&](int set, int buf) {
#pragma unroll
    for (int i = 0; i < PPT; ++i)
      if (xok[i]) {
        u16x8 v = xr[set][i];
        if constexpr (SILU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float gv = bf2f(v[j]);
            v[j] = f2bf(gv / (1.f + __expf(-gv)) * bf2f(xu[set][i][j]));
          }
        }
        *reinterpret_cast<u16x8*>(&xs[buf][xdst[i]]) = v;
      }
  };
  auto compute = [&](int slot, int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + r;
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(&xs[buf][m * kChunk + 8 * swz(m, 4 * ks + h)]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[slot][nt][ks], xf, acc[nt][mt], 0, 0, 0);
      }
  };

  // ---- prologue: X chunk 0 -> LDS, X chunk 1 -> registers, W chunks 0..U-1
  load_x(0, 0);
  if (nchunks > 1) load_x(1, 1);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (u < nchunks) load_w(u, u);
  store_x(0, 0);
  __syncthreads();

  // ---- main loop, unrolled by U (even) so ring slots / X sets are compile-time
  static_assert(U % 2 == 0, "U must be even (X register sets alternate per chunk)");
  for (int c0 = 0; c0 < nchunks; c0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u;
      if (c < nchunks) {
        if (c + 2 < nchunks) load_x(u & 1, c + 2);   // set u&1 held X(c), already in LDS
        compute(u, c & 1);
        if (c + U < nchunks) load_w(u, c + U);
        if (c + 1 < nchunks) store_x((u + 1) & 1, (c + 1) & 1);
        __syncthreads();
      }
    }
  }

  // ---- epilogue: acc[nt][mt][v] = C[n = n0 + 16 nt + 4h + v][m = 16 mt + r]
  if (gridDim.y == 1) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + r;
        if (m < M) {
          u16x4 o;
#pragma unroll
          for (int v = 0; v < 4; ++v) o[v] = f2bf(acc[nt][mt][v]);
          *reinterpret_cast<u16x4*>(y + (size_t)m * ldy + n0 + 16 * nt + 4 * h) = o;
        }
      }
  } else {
    float* pp = part + (size_t)split * M * N;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + r;
        if (m < M) *reinterpret_cast<f32x4*>(pp + (size_t)m * N + n0 + 16 * nt + 4 * h) = acc[nt][mt];
      }
  }
}

// Y[m][n] = bf16(sum_s part[s][m][n]); 8 outputs per thread.
__global__ void __launch_bounds__(256) gemm_mid_reduce_kernel(const float* __restrict__ part, int splits,
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

struct MidCfg {
  int mt, nt, nw, u, silu;
  const void* fn;
};

#define K8S_MID(MT, NT, NW, U) {MT, NT, NW, U, 0, (const void*)gemm_mid_kernel<MT, NT, NW, U, false>}
#define K8S_MIDS(MT, NT, NW, U) {MT, NT, NW, U, 1, (const void*)gemm_mid_kernel<MT, NT, NW, U, true>}
// variant table (index = the `cfg` argument of k8s_gemm_mid)
static const MidCfg kMidCfgs[] = {
    K8S_MID(2, 1, 4, 4),  K8S_MID(2, 2, 4, 4),  K8S_MID(4, 1, 4, 4),  K8S_MID(4, 2, 4, 4),
    K8S_MID(8, 1, 4, 4),  K8S_MID(8, 2, 4, 4),  K8S_MID(16, 1, 4, 4), K8S_MID(16, 2, 4, 2),
    K8S_MID(8, 2, 4, 2),  K8S_MID(4, 2, 4, 8),  K8S_MID(8, 1, 8, 4),  K8S_MID(16, 1, 8, 4),
    // SwiGLU-fused down projections (x = gate_up)
    K8S_MIDS(2, 1, 4, 4), K8S_MIDS(4, 1, 4, 4), K8S_MIDS(8, 1, 4, 4), K8S_MIDS(8, 1, 8, 4), K8S_MIDS(16, 1, 8, 4),
    // M tiles matched to the decode batch buckets 48 / 96 / 160 / 192 / 224:
    // every wave reads all 16*MT staged X rows from LDS per chunk (the LDS
    // reads, not HBM, bound this kernel -- profiles/README.md), so padding
    // M = 96 to 128 rows or 192 to 256 costs 25-33 % of that traffic and of the
    // MFMAs.  Appended so the indices above (dispatch tables) stay valid.
    K8S_MID(3, 1, 4, 4),  K8S_MID(3, 2, 4, 4),  K8S_MID(6, 1, 4, 4),  K8S_MID(6, 1, 8, 4),
    K8S_MID(6, 2, 4, 4),  K8S_MID(10, 1, 8, 4), K8S_MID(12, 1, 4, 4), K8S_MID(12, 1, 8, 4),
    K8S_MID(14, 1, 8, 4),
};
#undef K8S_MID
#undef K8S_MIDS
constexpr int kNumMidCfgs = sizeof(kMidCfgs) / sizeof(kMidCfgs[0]);

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_gemm_mid_num_cfgs() { return kNumMidCfgs; }

K8S_API int k8s_gemm_mid_cfg(int cfg, int* out5) {
  if (cfg < 0 || cfg >= kNumMidCfgs) return (int)hipErrorInvalidValue;
  out5[0] = kMidCfgs[cfg].mt;
  out5[1] = kMidCfgs[cfg].nt;
  out5[2] = kMidCfgs[cfg].nw;
  out5[3] = kMidCfgs[cfg].u;
  out5[4] = kMidCfgs[cfg].silu;
  return 0;
}

// splits > 1 needs `part` = splits * M * N fp32 scratch.  SwiGLU variants
// read x as [M][2K] gate|up (ldx = row stride of that buffer).
static int launch_mid(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                      int splits, void* part, bool reduce, hipStream_t s) {
  if (cfg < 0 || cfg >= kNumMidCfgs || splits < 1) return (int)hipErrorInvalidValue;
  const MidCfg& c = kMidCfgs[cfg];
  const int bn = 16 * c.nt * c.nw;
  if (M <= 0 || M > 16 * c.mt || N % bn || K % (splits * kChunk) || (splits > 1 && part == nullptr) ||
      (M * N) % 8 || ldx % 8 || ldy % 8)
    return (int)hipErrorInvalidValue;
  const int kslice = K / splits;
  dim3 g(N / bn, splits);
  void* args[] = {(void*)&x, (void*)&ldx, (void*)&w, (void*)&y, (void*)&ldy, (void*)&part,
                  (void*)&M, (void*)&N, (void*)&K, (void*)&kslice};
  // the kernel parameters above are all 4- or 8-byte scalars/pointers, in order
  hipError_t e = hipLaunchKernel(c.fn, g, dim3(c.nw * 64), args, 0, s);
  if (e != hipSuccess) return (int)e;
  if (splits > 1 && reduce) {
    const int blocks = (M * N / 8 + 255) / 256;
    hipLaunchKernelGGL(gemm_mid_reduce_kernel, dim3(blocks), dim3(256), 0, s, (const float*)part, splits,
                       (uint16_t*)y, ldy, M, N);
  }
  return (int)hipGetLastError();
}

K8S_API int k8s_gemm_mid(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                         int splits, void* part, hipStream_t s) {
  return launch_mid(x, ldx, w, y, ldy, M, N, K, cfg, splits, part, true, s);
}

// splits > 1: leaves the fp32 partials [splits][M][N] in `part` for a fused
// consumer (k8s_splitk_addnorm) instead of launching the reduce kernel.
K8S_API int k8s_gemm_mid_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                              int splits, void* part, hipStream_t s) {
  return launch_mid(x, ldx, w, y, ldy, M, N, K, cfg, splits, part, false, s);
}
