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
//     wave's own A-fragment registers, in the same U-chunk ring as W (a
//     chunk's W and X loads are issued together, so the in-order vmcnt wait
//     for one chunk never drains the later ones): no LDS, no sharing needed
//     since each wave owns its rows.
//   * v_mfma_f32_16x16x32_bf16: A = X rows (16 m), B = W^T (16 n); one W
//     fragment read from LDS feeds MTW MFMAs.
//   * split-K over gridDim.y: fp32 partials [split][M][N] reduced by a
//     vectorised kernel, or left for a fused consumer (the next residual add +
//     RMSNorm, k8s_splitk_addnorm) -- the same contract as gemm_mid.
#include <cstdlib>

#include "common.h"
#include "knobs.h"
#include "norm_prologue.h"

namespace k8s {

constexpr int kSC = 64;   // k per chunk
constexpr int kSBN = 64;  // columns per workgroup

__device__ __forceinline__ int sswz(int n, int j) { return j ^ (n & 7); }

// W row (relative to the strip's first row) of strip row n, 16-row fragment
// f = n / 16 of NF.  Plain: n.  SwiGLU form (silu_i = I > 0, W = [Wg; Wu] of
// 2I rows, strip base = the first gate row of the strip's 8 NF act columns):
// fragments [0, NF/2) are gate rows, [NF/2, NF) the up rows of the same act
// columns, so fragment f and f + NF/2 of one lane hold gate and up of one
// (row, column) of the product.
template <int NF>
__device__ __forceinline__ int strip_row(int n, int silu_i) {
  if (!silu_i) return n;
  const int f = n >> 4, half = NF / 2;
  return (f >= half ? silu_i : 0) + (f % half) * 16 + (n & 15);
}

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// NORM: X = rmsnorm(nin) computed by the workgroup into LDS (norm_prologue.h;
// M <= kNormMaxRows, one K split, K == nin.H) while its first U chunks of W
// are in flight; the X fragments are then read from LDS.
template <int MTW, int U, bool NORM = false>
__global__ void __launch_bounds__(256) gemm_stream_kernel(const uint16_t* __restrict__ x, int ldx,
                                                          const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                          int ldy, float* __restrict__ part, int M, int N, int K,
                                                          int kslice, int silu_i, NormIn nin = {}) {
  __shared__ __attribute__((aligned(16))) uint16_t ws[2][kSBN * kSC];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  // strip: 64 W rows (plain: output columns n0 ..; SwiGLU: 32 act columns n0 ..)
  const int n0 = blockIdx.x * (silu_i ? kSBN / 2 : kSBN);
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
    wsrc[i] = w + (size_t)(n0 + strip_row<4>(n, silu_i)) * K + kbeg + 8 * sswz(n, jl);
    wdst[i] = n * kSC + 8 * jl;
  }
  // ---- X fragments: row of frag mt for this lane (clamped; masked at the store)
  if constexpr (NORM) {
    x = k8s_norm_lds;
    ldx = K;
  }
  const uint16_t* xrow[MTW];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
    const int m = min(m_base + 16 * mt + r, M - 1);
    xrow[mt] = x + (size_t)m * ldx + kbeg + 8 * g;
  }
  // every wave computes (a wave past the last row works on clamped rows and
  // stores nothing): no wave-dependent branch around a load, see below
  const bool active = m_base < M;

  f32x4 acc[MTW][4];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int cf = 0; cf < 4; ++cf) acc[mt][cf] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ring slot c % U holds chunk c: its W pieces (written to LDS one iteration
  // before chunk c is computed) and this wave's X fragments of it (read
  // straight from the registers by chunk c's MFMAs).  W and X of a chunk are
  // issued together, U chunks ahead, so loads are consumed in issue order and
  // the in-order vmcnt never drains the ring early: (U-1) chunks stay in flight
  // while one is computed.
  u16x8 ring[U][2];
  bf16x8 xq[U][2][MTW];
  auto load_w = [&](int slot, int c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ring[slot][i] = ldw_nt<u16x8>(wsrc[i] + c * kSC);
  };
  auto load_x = [&](int slot, int c) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
        xq[slot][s][mt] = *reinterpret_cast<const bf16x8*>(xrow[mt] + c * kSC + 32 * s);
  };
  auto load_chunk = [&](int slot, int c) {
    load_w(slot, c);
    load_x(slot, c);
  };
  auto store_w = [&](int slot, int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u16x8*>(&ws[buf][wdst[i]]) = ring[slot][i];
  };
  auto compute = [&](int buf, int slot) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        const int n = 16 * cf + r;
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(&ws[buf][n * kSC + 8 * sswz(n, 4 * s + g)]);
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
          acc[mt][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xq[slot][s][mt], wf, acc[mt][cf], 0, 0, 0);
      }
  };

  // ---- prologue: chunks 0..U-1 in flight, chunk 0's W -> LDS
  // (nch % U == 0 and nch >= U: checked at launch)
  if constexpr (NORM) {
    __shared__ float nscr[16];
#pragma unroll
    for (int u = 0; u < U; ++u) load_w(u, u);
    norm_rows_to_lds(k8s_norm_lds, M, nin, blockIdx.x == 0 && blockIdx.y == 0, nscr);
#pragma unroll
    for (int u = 0; u < U; ++u) load_x(u, u);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) load_chunk(u, u);
  }
  store_w(0, 0);
  __syncthreads();

  // ---- main loop, unrolled by U (ring slots compile-time).  EVERY load is
  // unconditional: one past the slice is clamped to the last chunk (an L2
  // hit) -- a conditional load makes hipcc wait vmcnt(0) before every ring
  // ds_write, which left ONE chunk in flight per workgroup (7.5 GB/s per
  // workgroup: 0.95 TB/s at 128 workgroups, profiles/r2_gemm_probe_m128*.txt).
  for (int c0 = 0; c0 < nch; c0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u;
      compute(c & 1, u);
      store_w((u + 1) % U, (c + 1) & 1);
      load_chunk(u, min(c + U, nch - 1));
      __syncthreads();
    }
  }

  // ---- epilogue: acc[mt][cf][v] = C[m = m_base + 16 mt + 4 g + v][n = n0 + 16 cf + r]
  if (!active) return;
  if (silu_i) {  // act = silu(gate) * up, with the unfused path's bf16 rounding of both
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m_base + 16 * mt + 4 * g + v;
        if (m < M) {
#pragma unroll
          for (int cf = 0; cf < 2; ++cf)
            y[(size_t)m * ldy + n0 + 16 * cf + r] =
                f2bf(silu_f(bf2f(f2bf(acc[mt][cf][v]))) * bf2f(f2bf(acc[mt][cf + 2][v])));
        }
      }
  } else if (gridDim.y == 1) {
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

// ---------------------------------------------------------------- LDS-DMA
// Same decomposition (64-column strip x all M rows x one K slice per
// workgroup, 4 waves splitting the rows), both operands staged by
// global_load_lds (16-byte LDS-DMA, no VGPR round trip) into an NB-stage LDS
// ring.  X arrives as full 128-byte row pieces instead of the fragment-shaped
// L2 loads of the register-ring kernel (16 rows x 64 B per instruction, the
// TA-bound pattern).  Both images are lane-linear per DMA instruction with
// the XOR swizzle applied on the SOURCE address (piece j of row n lands in
// slot j ^ (n & 7)), so every ds_read_b128 fragment read is the same as the
// register-ring kernel's.  Synchronisation (cdna_hip_programming.md,
// "Pipelining across barriers"): one __shared__ array, a counted
// s_waitcnt vmcnt((NB-2) * DMAs per chunk) + raw s_barrier per chunk (never
// __syncthreads, whose fence would drain the DMAs in flight), lgkmcnt(0)
// after the fragment reads so the stage can be re-filled after the next
// barrier.
typedef __attribute__((address_space(3))) void lds_void_t;

// a __device__ function: with the builtin written in the kernel template's own
// body, hipcc's host pass silently dropped the kernels' launch stubs
__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_dst, 16, 0, 0);
}

// Weight stream of the LDS-DMA kernel: default cache policy.  The non-temporal
// policy (nt, bit 2) that speeds the register-path weight loads (ldw_nt, M <= 32:
// 4-6 % per layer) made this kernel 2-3 % SLOWER at M = 96-192, measured
// interleaved nt / off / nt / off (profiles/r2_nt_ab/).  K8S_GLDS_W_NT=1 restores it.
#ifndef K8S_GLDS_W_NT
#define K8S_GLDS_W_NT 0
#endif
__device__ __forceinline__ void glds16_w(const uint16_t* src, uint16_t* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_dst, 16, 0, K8S_GLDS_W_NT ? 2 : 0);
}

// NF: 16-column fragments per strip (4: 64-column strips, 8: 128-column strips,
// which halve the X re-reads per weight byte at M ~ 100-256: every workgroup
// stages all M rows of X for its strip, so X -- not W -- was the larger
// stream through L2 -> LDS there).
template <int MTW, int NB, int NF = 4>
constexpr int glds_lds_elems() {
  return NB * (16 * NF * kSC + 64 * MTW * kSC);
}

// One workgroup's 64-column strip over one K slice: acc += X[0..M) . W[strip]^T.
// x: the tile's first row (rows past M are clamped, never stored); wstrip: the
// strip's first W row ([N][K] row-major, K-slice offset already applied);
// nch: 64-deep chunks in the slice; sm: the kernel's one __shared__ array of
// glds_lds_elems<MTW, NB>() elements.
// HAND: the stage's MTW X and NF W fragments per 32-deep half are read by
// hand-issued ds_read_b128 (common.h lds_rd16) and each fragment column's MFMAs
// wait only for the reads they consume (hipcc's own schedule waits lgkmcnt(0)
// before every group: one LDS latency per NF group; K8SRCA_GLDS_HAND=0 restores it).
template <int MTW, int NF, int CF>
__device__ __forceinline__ void glds_mm(f32x4 (&acc)[MTW][NF], bf16x8 (&xf)[MTW], bf16x8 (&wf)[NF]) {
  if constexpr (CF < NF) {
    if constexpr (CF == 0) {
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) lgkm_wait<NF - 1>(xf[mt]);
    }
    lgkm_wait<NF - 1 - CF>(wf[CF]);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[mt][CF] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[mt], wf[CF], acc[mt][CF], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // the next column's wait stays behind these MFMAs
    glds_mm<MTW, NF, CF + 1>(acc, xf, wf);
  }
}

template <int MTW, int NB, int NF = 4, bool HAND = false>
__device__ __forceinline__ void glds_strip(const uint16_t* __restrict__ x, int ldx, int M,
                                           const uint16_t* __restrict__ wstrip, int K, int nch, uint16_t* sm,
                                           f32x4 (&acc)[MTW][NF], int silu_i = 0) {
  constexpr int MP = 64 * MTW;         // X rows staged: 4 waves x MTW 16-row fragments
  constexpr int WST = 16 * NF * kSC;   // W stage: 16 NF rows x 64 k
  constexpr int STG = WST + MP * kSC;  // elements per stage
  constexpr int XPT = MP * 8 / 256;    // X pieces (DMAs) per thread per chunk
  constexpr int WPT = NF / 2;          // W pieces (DMAs) per thread per chunk
  constexpr int LPC = WPT + XPT;       // DMAs per thread per chunk
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int m_base = wv * 16 * MTW;

  const uint16_t* wsrc[WPT];
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int p = 256 * i + tid, n = p >> 3, jl = p & 7;
    wsrc[i] = wstrip + (size_t)strip_row<NF>(n, silu_i) * K + 8 * (jl ^ (n & 7));
  }
  const uint16_t* xsrc[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int p = 256 * i + tid, m = p >> 3, jl = p & 7;
    xsrc[i] = x + (size_t)min(m, M - 1) * ldx + 8 * (jl ^ (m & 7));
  }
  auto issue = [&](int stage, int c) {
    uint16_t* st = sm + stage * STG;
#pragma unroll
    for (int i = 0; i < WPT; ++i) glds16_w(wsrc[i] + c * kSC, st + (256 * i + 64 * wv) * 8);
#pragma unroll
    for (int i = 0; i < XPT; ++i) glds16(xsrc[i] + c * kSC, st + WST + (256 * i + 64 * wv) * 8);
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)sm;
  auto compute = [&](int stage) {
    const uint16_t* ws = sm + stage * STG;
    const uint16_t* xs = ws + WST;
    if constexpr (HAND) {
      const uint32_t wb = lds0 + 2u * (uint32_t)(stage * STG), xb = wb + 2u * WST;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // the counted lgkmcnt waits of glds_mm assume every lgkm operation
        // between these reads and their waits is one of these ds_reads: a scalar
        // load scheduled into the window (it also counts on lgkmcnt, and returns
        // out of order) would let a wait pass before its fragment landed.  No
        // instruction from before the block may move into it (this barrier), and
        // none from after it (glds_mm's barrier behind each column's MFMAs);
        // the reads' own addresses are VALU / SALU arithmetic.
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 xf[MTW], wf[NF];
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) {
          const int m = m_base + 16 * mt + r;
          xf[mt] = lds_rd16<0>(xb + 2u * (uint32_t)(m * kSC + 8 * ((4 * s + g) ^ (m & 7))));
        }
#pragma unroll
        for (int cf = 0; cf < NF; ++cf) {
          const int n = 16 * cf + r;
          wf[cf] = lds_rd16<0>(wb + 2u * (uint32_t)(n * kSC + 8 * ((4 * s + g) ^ (n & 7))));
        }
        glds_mm<MTW, NF, 0>(acc, xf, wf);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 xf[MTW];
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) {
        const int m = m_base + 16 * mt + r;
        xf[mt] = *reinterpret_cast<const bf16x8*>(xs + m * kSC + 8 * ((4 * s + g) ^ (m & 7)));
      }
#pragma unroll
      for (int cf = 0; cf < NF; ++cf) {
        const int n = 16 * cf + r;
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(ws + n * kSC + 8 * ((4 * s + g) ^ (n & 7)));
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
          acc[mt][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[mt], wf, acc[mt][cf], 0, 0, 0);
      }
    }
  };

  // prologue: chunks 0..NB-2 in flight (clamped to the slice's last chunk)
#pragma unroll
  for (int c = 0; c < NB - 1; ++c) issue(c, min(c, nch - 1));
  for (int c0 = 0; c0 < nch; c0 += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int c = c0 + u;
      // this wave's DMAs of chunk c are done when at most the NB-2 later chunks' remain
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 2) * LPC) : "memory");
      __builtin_amdgcn_s_barrier();  // every wave's chunk c landed; every wave is done reading chunk c-1
      issue((u + NB - 1) % NB, min(c + NB - 1, nch - 1));  // re-fill chunk c-1's stage (clamped: an L2 hit)
      // the last trip may run past the slice (nch % NB != 0): those steps skip
      // only the MFMAs -- every DMA, wait and barrier stays unconditional
      if (c < nch) compute(u);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS
}

// acc[mt][cf][v] = C[m_base + 16 mt + 4 g + v][16 cf + r] of the tile: bf16 rows
// of y (final) or fp32 rows of `part` (split-K partial), rows < M only.
template <int MTW, int NF = 4>
__device__ __forceinline__ void glds_store(const f32x4 (&acc)[MTW][NF], int M, uint16_t* __restrict__ y, int ldy,
                                           float* __restrict__ pp, int ldp, bool silu = false) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int m_base = wv * 16 * MTW;
  if (m_base >= M) return;
  if (silu) {  // fragments [0, NF/2) gate, [NF/2, NF) up: act columns 16 cf + r of the strip
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m_base + 16 * mt + 4 * g + v;
        if (m < M) {
#pragma unroll
          for (int cf = 0; cf < NF / 2; ++cf)
            y[(size_t)m * ldy + 16 * cf + r] =
                f2bf(silu_f(bf2f(f2bf(acc[mt][cf][v]))) * bf2f(f2bf(acc[mt][cf + NF / 2][v])));
        }
      }
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int m = m_base + 16 * mt + 4 * g + v;
      if (m < M) {
#pragma unroll
        for (int cf = 0; cf < NF; ++cf) {
          if (pp)
            pp[(size_t)m * ldp + 16 * cf + r] = acc[mt][cf][v];
          else
            y[(size_t)m * ldy + 16 * cf + r] = f2bf(acc[mt][cf][v]);
        }
      }
    }
}

// Push epilogue (TP row-parallel output, common.h K8sPush): the tile goes
// through LDS (bf16, 16-B padded rows) so each thread pushes whole 16-byte row
// pieces -- full 128- / 256-byte row segments per strip over xGMI, not the
// accumulator layout's 32-byte pieces -- then the strip's flag is raised.
template <int MTW, int NF>
__device__ __forceinline__ void glds_push_store(const f32x4 (&acc)[MTW][NF], int M, uint16_t* sm, const K8sPush& P,
                                                int n0, int strip) {
  constexpr int BN = 16 * NF, PITCH = BN + 8, CPR = BN / 8;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int m_base = wv * 16 * MTW;
  __syncthreads();  // every wave is done reading the ring's last stage
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int cf = 0; cf < NF; ++cf) sm[(m_base + 16 * mt + 4 * g + v) * PITCH + 16 * cf + r] = f2bf(acc[mt][cf][v]);
  __syncthreads();
  const uint32_t e = push_epoch(P);
  for (int i = threadIdx.x; i < M * CPR; i += 256) {
    const int m = i / CPR, c = i % CPR;
    push_store8(P, e, m, n0 + 8 * c, *reinterpret_cast<const u16x8*>(sm + m * PITCH + 8 * c));
  }
  push_publish(P, e, strip, n0);
}

template <int MTW, int NB, int NF, bool HAND, bool PUSH = false>
__global__ void __launch_bounds__(256) gemm_glds_kernel(const uint16_t* __restrict__ x, int ldx,
                                                        const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                        int ldy, float* __restrict__ part, int M, int N, int K,
                                                        int kslice, int silu_i, K8sPush push) {
  __shared__ __attribute__((aligned(16))) uint16_t sm[glds_lds_elems<MTW, NB, NF>()];
  // strip: 16 NF W rows (plain: output columns n0 ..; SwiGLU: 8 NF act columns n0 ..)
  const int n0 = blockIdx.x * (silu_i ? 8 : 16) * NF, split = blockIdx.y, kbeg = split * kslice;
  f32x4 acc[MTW][NF];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int cf = 0; cf < NF; ++cf) acc[mt][cf] = f32x4{0.f, 0.f, 0.f, 0.f};
  glds_strip<MTW, NB, NF, HAND>(x + kbeg, ldx, M, w + (size_t)n0 * K + kbeg, K, kslice / kSC, sm, acc, silu_i);
  static_assert(64 * MTW * (16 * NF + 8) <= glds_lds_elems<MTW, NB, NF>(), "push tile must fit the ring's LDS");
  if constexpr (PUSH)
    glds_push_store<MTW, NF>(acc, M, sm, push, n0, blockIdx.x);
  else if (silu_i)
    glds_store<MTW, NF>(acc, M, y + n0, ldy, nullptr, 0, true);
  else if (gridDim.y == 1)
    glds_store<MTW, NF>(acc, M, y + n0, ldy, nullptr, 0);
  else
    glds_store<MTW, NF>(acc, M, nullptr, 0, part + (size_t)split * M * N + n0, N);
}

// MoE grouped form (B13, decode batches): rows offsets[e] .. offsets[e+1] of x
// times W_e^T for every expert e in one launch (w [E][N][K]).  Grid (N / 64,
// max_tiles, splits): workgroup (nb, j, z) walks the per-expert counts of
// 64-row tiles to find its (expert, tile); surplus workgroups exit.  Split-K
// partials are [splits][total_rows][N] (gemm_stream_reduce_kernel's layout).
template <int NB>
__global__ void __launch_bounds__(256) grouped_glds_kernel(const uint16_t* __restrict__ x, int ldx,
                                                           const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                           int ldy, float* __restrict__ part,
                                                           const int* __restrict__ offsets, int E, int N, int K,
                                                           int kslice, int total_rows) {
  __shared__ __attribute__((aligned(16))) uint16_t sm[glds_lds_elems<1, NB>()];
  int j = blockIdx.y, e = 0, row0 = 0, rows = 0;
  for (; e < E; ++e) {
    const int a0 = offsets[e], a1 = offsets[e + 1];
    const int t = (a1 - a0 + 63) / 64;
    if (j < t) {
      row0 = a0 + 64 * j;
      rows = min(64, a1 - row0);
      break;
    }
    j -= t;
  }
  if (e >= E || rows <= 0) return;  // workgroup-uniform: before any DMA or barrier
  const int n0 = blockIdx.x * kSBN, split = blockIdx.z, kbeg = split * kslice;
  f32x4 acc[1][4];
#pragma unroll
  for (int cf = 0; cf < 4; ++cf) acc[0][cf] = f32x4{0.f, 0.f, 0.f, 0.f};
  glds_strip<1, NB>(x + (size_t)row0 * ldx + kbeg, ldx, rows, w + ((size_t)e * N + n0) * K + kbeg, K, kslice / kSC,
                    sm, acc);
  if (gridDim.z == 1)
    glds_store<1>(acc, rows, y + (size_t)row0 * ldy + n0, ldy, nullptr, 0);
  else
    glds_store<1>(acc, rows, nullptr, 0, part + ((size_t)split * total_rows + row0) * N + n0, N);
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

// The split-K form of the push epilogue: gemm_stream_reduce_kernel's sums (same
// order: bit-identical) for one 64-column strip of all M rows per workgroup,
// pushed into the peers' slots, then the strip's flag.
__global__ void __launch_bounds__(256) gemm_stream_reduce_push_kernel(const float* __restrict__ part, int splits,
                                                                      int M, int N, K8sPush P) {
  const int strip = blockIdx.x, n0 = 64 * strip;
  const size_t MN = (size_t)M * N;
  const uint32_t e = push_epoch(P);
  for (int i = threadIdx.x; i < M * 8; i += 256) {
    const int m = i >> 3, n = n0 + 8 * (i & 7);
    const size_t idx = (size_t)m * N + n;
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
    push_store8(P, e, m, n, o);
  }
  push_publish(P, e, strip, n0);
}

// the hand-issued LDS reads of glds_strip (default; knob glds_hand=0: hipcc's
// own reads, A/B, read per launch).  Bit-identical; 0-5 % faster per projection
// at M = 64-192 (tools/glds_hand_ab.py, profiles/r4/glds_hand/): the decode GEMMs
// are bound by their DMA stream more than by the exposed LDS latency.
static bool glds_hand() { return knob(kKnobGldsHand) != 0; }

// push != nullptr: the push-epilogue form (splits == 1, plain output; hand reads)
template <int MTW, int NB, int NF = 4>
static hipError_t launch_glds(dim3 grid, hipStream_t s, const uint16_t* x, int ldx, const uint16_t* w, uint16_t* y,
                              int ldy, float* part, int M, int N, int K, int kslice, int silu_i,
                              const K8sPush* push = nullptr) {
  const K8sPush none{};
  if (push)
    hipLaunchKernelGGL((gemm_glds_kernel<MTW, NB, NF, true, true>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, part, M,
                       N, K, kslice, 0, *push);
  else if (glds_hand())
    hipLaunchKernelGGL((gemm_glds_kernel<MTW, NB, NF, true>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, part, M, N,
                       K, kslice, silu_i, none);
  else
    hipLaunchKernelGGL((gemm_glds_kernel<MTW, NB, NF, false>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, part, M, N,
                       K, kslice, silu_i, none);
  return hipGetLastError();
}

template <int MTW, int U>
static hipError_t launch_stream(dim3 grid, hipStream_t s, const uint16_t* x, int ldx, const uint16_t* w, uint16_t* y,
                                int ldy, float* part, int M, int N, int K, int kslice, int silu_i) {
  hipLaunchKernelGGL((gemm_stream_kernel<MTW, U>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, part, M, N, K, kslice,
                     silu_i);
  return hipGetLastError();
}

}  // namespace k8s

using namespace k8s;

// cfg: register-ring depth U (4 or 8), or 10 + NB for the LDS-DMA kernel (NB = 3..6
// stages; 5 and 6 for M <= 64), or 20 + NB for the LDS-DMA kernel on 128-column
// strips (NB = 3, or 4 for M <= 192; N % 128 == 0).  splits > 1 needs `part` =
// splits * M * N fp32; reduce = 0 leaves the partials for a fused consumer.
// silu: w is the gate_up weight [2N][K] (gate rows first) and y[M][N] = silu(x Wg^T) * (x Wu^T)
// (splits == 1 only: the nonlinearity needs the whole K sum).
static int stream_launch(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                         int splits, void* part, bool reduce, hipStream_t s, bool silu = false,
                         const K8sPush* push = nullptr) {
  // push (splits == 1): the LDS-DMA kernel's own epilogue pushes; splits > 1: the reduce pass does
  const K8sPush* gpush = (push && splits == 1) ? push : nullptr;
  if (push && (silu || !reduce || (splits == 1 && cfg < 13))) return (int)hipErrorInvalidValue;
  const int bn = (cfg > 20 ? 128 : kSBN) / (silu ? 2 : 1);  // output columns per strip
  if (M <= 0 || M > 256 || N % bn || splits < 1 || K % (splits * kSC) || (splits > 1 && part == nullptr) ||
      (cfg != 4 && cfg != 8 && (cfg < 13 || cfg > 16) && cfg != 23 && cfg != 24) || ldx % 8 ||
      (splits > 1 && (M * N) % 8) || ((splits == 1 || reduce) && ldy < N) || (silu && splits != 1))
    return (int)hipErrorInvalidValue;
  const int silu_i = silu ? N : 0;
  const int kslice = K / splits;
  // the register-ring loop is unrolled by U chunks with no partial trip
  if (cfg < 10 && (kslice / kSC) % cfg) return (int)hipErrorInvalidValue;
  const int mtw = ((M + 15) / 16 + 3) / 4;  // 16-row fragments per wave (4 waves)
  // LDS-DMA stages of (64 + 64 * mtw) x 64 bf16 must fit the 160 KB of LDS
  if ((cfg == 14 && mtw > 3) || (cfg > 14 && cfg < 20 && mtw > 1) || (cfg == 24 && mtw > 3))
    return (int)hipErrorInvalidValue;
  if (cfg == 8 && mtw > 2) return (int)hipErrorInvalidValue;  // an 8-deep X ring would not fit the VGPRs
  const dim3 grid(N / bn, splits);
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  float* pp = (float*)part;
  hipError_t e;
#define K8S_SL(MT, UU) e = launch_stream<MT, UU>(grid, s, xx, ldx, ww, yy, ldy, pp, M, N, K, kslice, silu_i)
#define K8S_GL(MT, NB) e = launch_glds<MT, NB>(grid, s, xx, ldx, ww, yy, ldy, pp, M, N, K, kslice, silu_i, gpush)
#define K8S_GW(MT, NB) e = launch_glds<MT, NB, 8>(grid, s, xx, ldx, ww, yy, ldy, pp, M, N, K, kslice, silu_i, gpush)
  if (cfg == 23) {
    switch (mtw) {
      case 1: K8S_GW(1, 3); break;
      case 2: K8S_GW(2, 3); break;
      case 3: K8S_GW(3, 3); break;
      default: K8S_GW(4, 3); break;
    }
  } else if (cfg == 24) {
    switch (mtw) {
      case 1: K8S_GW(1, 4); break;
      case 2: K8S_GW(2, 4); break;
      default: K8S_GW(3, 4); break;
    }
  } else if (cfg == 13) {
    switch (mtw) {
      case 1: K8S_GL(1, 3); break;
      case 2: K8S_GL(2, 3); break;
      case 3: K8S_GL(3, 3); break;
      default: K8S_GL(4, 3); break;
    }
  } else if (cfg == 14) {
    switch (mtw) {
      case 1: K8S_GL(1, 4); break;
      case 2: K8S_GL(2, 4); break;
      default: K8S_GL(3, 4); break;
    }
  } else if (cfg == 15) {
    K8S_GL(1, 5);
  } else if (cfg == 16) {
    K8S_GL(1, 6);
  } else if (cfg == 4) {
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
      default: return (int)hipErrorInvalidValue;
    }
  }
#undef K8S_SL
#undef K8S_GL
#undef K8S_GW
  if (e != hipSuccess) return (int)e;
  if (splits > 1 && push) {
    hipLaunchKernelGGL(gemm_stream_reduce_push_kernel, dim3(N / 64), dim3(256), 0, s, (const float*)part, splits, M, N,
                       *push);
  } else if (splits > 1 && reduce) {
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

extern "C" int k8s_ar_push_desc(int id, int N, int T, int mode, K8sPush* out);

// A TP row-parallel projection with the push epilogue: x . w^T is stored into
// the xGMI communicator `ar_id`'s slots (mode 1 one-shot / 2 two-shot layout)
// instead of a y buffer, with one flag per output strip (k8s_push_strips(cfg,
// splits, N) of them); k8s_ar_push_addnorm_bf16 consumes it.  cfg: the LDS-DMA
// configurations (13-16, 23, 24), or any stream cfg with splits > 1 (the
// split-K reduce pass pushes).
K8S_API int k8s_gemm_stream_push(const void* x, int ldx, const void* w, int M, int N, int K, int cfg, int splits,
                                 void* part, int ar_id, int mode, hipStream_t s) {
  K8sPush P;
  const int rc = k8s_ar_push_desc(ar_id, N, M, mode, &P);
  if (rc) return rc;
  if (k8s_push_strips(cfg, splits, N) > kPushMaxStrips) return (int)hipErrorInvalidValue;
  return stream_launch(x, ldx, w, nullptr, N, M, N, K, cfg, splits, part, true, s, false, &P);
}

// y[M][N] = silu(x . w[0:N]^T) * (x . w[N:2N]^T): the gate_up projection with its
// SwiGLU epilogue (the [M][2N] gate_up activation is never written); splits == 1.
K8S_API int k8s_gemm_stream_silu(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K,
                                 int cfg, hipStream_t s) {
  return stream_launch(x, ldx, w, y, ldy, M, N, K, cfg, 1, nullptr, true, s, true);
}

// k8s_gemm_stream_silu (register-ring cfg 4 / 8) on X = rmsnorm(x [or the split-K
// partials `part`] + res_in) * norm_w computed by every workgroup into LDS
// (norm_prologue.h): bit-identical to k8s_rmsnorm / k8s_splitk_addnorm +
// k8s_gemm_stream_silu, one launch fewer.  res_out (!= res_in) <- x + res_in.
K8S_API int k8s_gemm_stream_silu_norm(const void* x, int x_stride, const float* part, int splits, const void* res_in,
                                      void* res_out, const void* norm_w, float eps, const void* w, void* y, int ldy,
                                      int M, int N, int K, int cfg, hipStream_t s) {
  if (M <= 0 || M > kNormMaxRows || K % kSC || K / 8 > 256 * kNormMaxChunks || (cfg != 4 && cfg != 8) ||
      (K / kSC) % cfg || N % (kSBN / 2) || ldy < N || !norm_w || (!x && !part) || (part && (splits < 1 || !res_in)) ||
      (res_in && (!res_out || res_out == res_in)))
    return (int)hipErrorInvalidValue;
  const NormIn nin{(const uint16_t*)x, part, (const uint16_t*)res_in, (uint16_t*)res_out, (const uint16_t*)norm_w,
                   x_stride, splits, K, eps};
  const dim3 grid(N / (kSBN / 2), 1);
  const size_t lds = (size_t)M * K * 2;
  if (cfg == 4)
    hipLaunchKernelGGL((gemm_stream_kernel<1, 4, true>), grid, dim3(256), lds, s, nullptr, 0, (const uint16_t*)w,
                       (uint16_t*)y, ldy, nullptr, M, N, K, K, N, nin);
  else
    hipLaunchKernelGGL((gemm_stream_kernel<1, 8, true>), grid, dim3(256), lds, s, nullptr, 0, (const uint16_t*)w,
                       (uint16_t*)y, ldy, nullptr, M, N, K, K, N, nin);
  return (int)hipGetLastError();
}

K8S_API int k8s_gemm_stream_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int cfg,
                                 int splits, void* part, hipStream_t s) {
  return stream_launch(x, ldx, w, y, ldy, M, N, K, cfg, splits, part, false, s);
}

// MoE grouped GEMM on the LDS-DMA strip kernel (decode batches: every expert's
// rows fit one or a few 64-row tiles).  cfg = 10 + NB (NB 3..6 stages);
// max_tiles >= sum_e ceil(rows_e / 64) (ceil(total_rows / 64) + E always is);
// splits > 1 needs `part` = splits * total_rows * N fp32 and reduces into y
// unless reduce == 0.
static int grouped_glds_launch(const void* x, int ldx, const void* w, void* y, int ldy, const int* offsets, int E,
                               int N, int K, int max_tiles, int cfg, int splits, void* part, int total_rows,
                               bool reduce, hipStream_t s) {
  if (total_rows <= 0) return (int)hipSuccess;
  if (E <= 0 || N % kSBN || splits < 1 || K % (splits * kSC) || (splits > 1 && part == nullptr) || cfg < 13 ||
      cfg > 16 || ldx % 8 || max_tiles <= 0 || (splits > 1 && ((size_t)total_rows * N) % 8))
    return (int)hipErrorInvalidValue;
  const int kslice = K / splits;
  const dim3 grid(N / kSBN, max_tiles, splits);
  const uint16_t* xx = (const uint16_t*)x;
  const uint16_t* ww = (const uint16_t*)w;
  uint16_t* yy = (uint16_t*)y;
  float* pp = (float*)part;
#define K8S_GG(NB)                                                                                               \
  hipLaunchKernelGGL((grouped_glds_kernel<NB>), grid, dim3(256), 0, s, xx, ldx, ww, yy, ldy, pp, offsets, E, N, K, \
                     kslice, total_rows)
  switch (cfg) {
    case 13: K8S_GG(3); break;
    case 14: K8S_GG(4); break;
    case 15: K8S_GG(5); break;
    default: K8S_GG(6); break;
  }
#undef K8S_GG
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (splits > 1 && reduce) {
    const int blocks = (int)(((size_t)total_rows * N / 8 + 255) / 256);
    hipLaunchKernelGGL(gemm_stream_reduce_kernel, dim3(blocks), dim3(256), 0, s, (const float*)part, splits, yy, ldy,
                       total_rows, N);
  }
  return (int)hipGetLastError();
}

K8S_API int k8s_grouped_glds(const void* x, int ldx, const void* w, void* y, int ldy, const int* offsets, int E, int N,
                             int K, int max_tiles, int cfg, int splits, void* part, int total_rows, hipStream_t s) {
  return grouped_glds_launch(x, ldx, w, y, ldy, offsets, E, N, K, max_tiles, cfg, splits, part, total_rows, true, s);
}
