// Prefill-size projection GEMM (B4, M >= ~1k):
//   Y[M][N] = X[M][K] . W[N][K]^T   bf16 in/out, fp32 accumulate
// with an optional SwiGLU epilogue for the gate_up projection:
//   act[M][I] = silu(X . Wg^T) * (X . Wu^T),  W = [Wg; Wu] ([2I][K], gate rows first)
// so the [M][2I] gate_up activation is never written nor re-read.
//
// Structure (cdna_hip_programming.md §5, "glds vs register staging" and
// "Pipelining across barriers"):
//   * 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N),
//     128 x 64 per wave: 8 x 4 accumulators of v_mfma_f32_16x16x32_bf16), one
//     workgroup per CU (128 KB of LDS).
//   * K in 32-deep chunks; chunk c = A[256][32] + B[256][32] (32 KB), staged by
//     global_load_lds (16-byte LDS-DMA, lane-linear) into a 4-stage ring: two
//     chunks are in flight while one is computed.  One __shared__ array, a
//     counted `s_waitcnt vmcnt` and a raw s_barrier per chunk (never
//     __syncthreads, whose fence would drain the DMAs in flight).
//   * LDS image: 64-byte rows of 4 16-byte pieces, piece p of row n stored in
//     slot p ^ g((n >> 2) & 3), g = {0, 2, 3, 1}.  Applied on the DMA SOURCE
//     address (the LDS side is lane-linear) and on the fragment read; with the
//     ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS ({0-3,12-15,20-27},
//     {4-11,16-19,28-31}, ...) every 16-lane group of a fragment read hits 16
//     distinct 16-byte bank slots.
//   * PIPE = 1: the fragments of chunk c+1 are read from LDS while chunk c's
//     MFMAs issue (one register set per operand plus a second B set), so the
//     barrier of chunk c+1 finds its operands already in registers; PIPE = 0 is
//     the plain form (read after the barrier).  Both are kept for A/B.
//   * Tile order: XCD-aware bijective remap of the workgroup id (each XCD's L2
//     sees a contiguous range of tiles), then groups of 4 M tiles x all N tiles
//     so the ~32 tiles an XCD runs at once share 4 X panels and 8 W panels.
//
// Rows past M are clamped on load (an L2 hit) and never stored.
// Reference parity: replaces the hipBLASLt call on the prefill path of
// models/llama.py (the reference's GPT-4 prompt processing of the whole thread
// history, /root/reference/common/openai_generic_assistant.py:45-51).
#include "common.h"

namespace k8s {
namespace big {

constexpr int BM = 256, BN = 256, BK = 32, NB = 4;
constexpr int STAGE = (BM + BN) * BK;  // bf16 elements per stage (32 KB)
constexpr int LPC = STAGE * 2 / (512 * 16);  // DMAs per thread per chunk (4)
constexpr int GM = 4;  // M tiles per tile group

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_dst, 16, 0, 0);
}

// slot XOR of a 64-byte row n: g((n >> 2) & 3), g = {0, 2, 3, 1}
__device__ __forceinline__ int gx(int q) { return (0x78 >> (2 * q)) & 3; }

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// MODE 0: plain (N output columns = W rows); MODE 1: SwiGLU (N = I output
// columns, W has 2I rows).  In MODE 1 an output tile covers 128 act columns
// j0 .. j0+127: wave column wc's 64 B rows are gate rows j0 + 32 wc + [0, 32)
// (fragments 0, 1) and the matching up rows (fragments 2, 3), so fragment f and
// f + 2 of one lane hold gate and up of the same (row, column).
template <int MODE, int PIPE>
__global__ void __launch_bounds__(512) gemm_big_kernel(const uint16_t* __restrict__ x, int ldx,
                                                       const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                       int ldy, int M, int N, int K, int n_mt, int n_nt) {
  __shared__ __attribute__((aligned(16))) uint16_t sm[NB * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 2, wc = wv & 3;

  // ---- tile of this workgroup: XCD-contiguous remap, then grouped order
  const int nwg = n_mt * n_nt;
  int t;
  {
    const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int gsz = GM * n_nt, gid = t / gsz, first_m = gid * GM;
  const int gm = min(n_mt - first_m, GM);
  const int tm = first_m + (t % gsz) % gm, tn = (t % gsz) / gm;
  const int m0 = tm * BM;

  // ---- DMA sources: instruction i of this wave stages combined rows
  // [16 ci, 16 ci + 16) of the [A; B] stage image, ci = 8 i + wv
  const int piece = (lane & 3) ^ gx(lane >> 4);
  const uint16_t* src[LPC];
#pragma unroll
  for (int i = 0; i < LPC; ++i) {
    const int ci = 8 * i + wv;
    const int row = 16 * ci + (lane >> 2);
    if (row < BM) {
      src[i] = x + (size_t)min(m0 + row, M - 1) * ldx + 8 * piece;
    } else {
      const int rb = row - BM;
      int gn;
      if (MODE == 0) {
        gn = tn * BN + rb;
      } else {
        const int f = (rb >> 4) & 3;
        gn = (f >= 2 ? N : 0) + tn * 128 + (rb >> 6) * 32 + (f & 1) * 16 + (rb & 15);
      }
      src[i] = w + (size_t)gn * K + 8 * piece;
    }
  }
  auto issue = [&](int stage, int c) {
    uint16_t* st = sm + stage * STAGE;
#pragma unroll
    for (int i = 0; i < LPC; ++i) glds16(src[i] + c * BK, st + (8 * i + wv) * 512);
  };

  // ---- fragment reads: lane's row (r = lane & 15) and swizzled piece
  const int foff = (lane & 15) * BK + 8 * ((lane >> 4) ^ gx((lane >> 2) & 3));
  const int a_off = (wr * 128) * BK + foff;
  const int b_off = (BM + wc * 64) * BK + foff;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = K / BK;
  // prologue: chunks 0 .. NB-2 in flight (clamped: short K re-reads its last chunk)
#pragma unroll
  for (int c = 0; c < NB - 1; ++c) issue(c, min(c, nch - 1));

  if (PIPE == 0) {
    // iteration c: wait for chunk c, barrier, refill chunk c-1's stage, compute c
    for (int c0 = 0; c0 < nch; c0 += NB) {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int c = c0 + u;
        // this wave's DMAs of chunk c are done when only the NB-2 later chunks' remain
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 2) * LPC) : "memory");
        __builtin_amdgcn_s_barrier();  // all of chunk c landed; all waves done reading chunk c-1
        asm volatile("" ::: "memory");
        issue((u + NB - 1) % NB, min(c + NB - 1, nch - 1));  // refill chunk c-1's stage
        if (c < nch) {
          const uint16_t* st = sm + u * STAGE;
          bf16x8 fb[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(st + b_off + 16 * j * BK);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const bf16x8 fa = *reinterpret_cast<const bf16x8*>(st + a_off + 16 * i * BK);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
  } else if (PIPE == 2) {
    // two explicit fragment sets: chunk c's MFMAs run on set c & 1 while chunk
    // c+1's fragments stream into the other set, interleaved by
    // sched_group_barrier (hipcc otherwise sinks every ds_read below the MFMAs,
    // so each barrier exposed the full LDS latency: PIPE 1 ran at the PIPE 0 rate)
    issue(NB - 1, min(NB - 1, nch - 1));
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 1) * LPC) : "memory");  // chunk 0 (this wave's part)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 fa[2][8], fb[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[0][j] = *reinterpret_cast<const bf16x8*>(sm + b_off + 16 * j * BK);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[0][i] = *reinterpret_cast<const bf16x8*>(sm + a_off + 16 * i * BK);
    for (int c0 = 0; c0 < nch; c0 += NB) {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int c = c0 + u, cur = u & 1, nxt = cur ^ 1;
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NB - 2) * LPC) : "memory");
        __builtin_amdgcn_s_barrier();  // all of chunk c+1 landed; every wave holds chunk c in registers
        asm volatile("" ::: "memory");
        if (c < nch) {
          issue(u, min(c + NB, nch - 1));  // chunk c's stage is free: refill it with chunk c + NB
          const uint16_t* nx = sm + ((u + 1) % NB) * STAGE;  // chunk c+1 (a clamped re-read past the end)
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[nxt][j] = *reinterpret_cast<const bf16x8*>(nx + b_off + 16 * j * BK);
#pragma unroll
          for (int i = 0; i < 8; ++i) fa[nxt][i] = *reinterpret_cast<const bf16x8*>(nx + a_off + 16 * i * BK);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
          // issue order: the 4 DMAs between the first MFMAs, then one fragment
          // read per two MFMAs, then the remaining MFMAs
#pragma unroll
          for (int k = 0; k < LPC; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
          }
#pragma unroll
          for (int k = 0; k < 12; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 32 - LPC - 24, 0);
        } else {
          issue(u, nch - 1);
        }
      }
    }
  } else {
    // chunk c's fragments are read during chunk c-1's MFMAs.  Stage of chunk c
    // is refilled (chunk c+NB) right after iteration c's barrier: every wave
    // finished reading it (lgkmcnt(0) before that barrier).  At the top of
    // iteration c chunks c+1 .. c+NB-1 are in flight, so the last stage is
    // filled in the prologue too.
    issue(NB - 1, min(NB - 1, nch - 1));
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 1) * LPC) : "memory");  // chunk 0 (this wave's part)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 fa[8], fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(sm + b_off + 16 * j * BK);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(sm + a_off + 16 * i * BK);
    for (int c0 = 0; c0 < nch; c0 += NB) {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int c = c0 + u;
        // chunk c's fragments are in registers; chunk c+1 has landed (this wave's part)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NB - 2) * LPC) : "memory");
        __builtin_amdgcn_s_barrier();  // all of chunk c+1 landed; every wave holds chunk c in registers
        asm volatile("" ::: "memory");
        issue(u, min(c + NB, nch - 1));  // chunk c's stage is free: refill it with chunk c + NB
        if (c < nch) {
          const uint16_t* nx = sm + ((u + 1) % NB) * STAGE;  // chunk c+1 (a clamped re-read past the end)
          bf16x8 fbn[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) fbn[j] = *reinterpret_cast<const bf16x8*>(nx + b_off + 16 * j * BK);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            fa[i] = *reinterpret_cast<const bf16x8*>(nx + a_off + 16 * i * BK);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j] = fbn[j];
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS

  // ---- epilogue: acc[i][j][v] = C[row 128 wr + 16 i + 4 (lane >> 4) + v][col 64 wc + 16 j + (lane & 15)]
  const int rbase = m0 + wr * 128 + 4 * (lane >> 4);
  if (MODE == 0) {
    uint16_t* yb = y + tn * BN + wc * 64 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = rbase + 16 * i + v;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < 4; ++j) yb[(size_t)m * ldy + 16 * j] = f2bf(acc[i][j][v]);
        }
      }
  } else {
    uint16_t* yb = y + tn * 128 + wc * 32 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = rbase + 16 * i + v;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // the unfused path's rounding: gate and up rounded to bf16 first (silu_mul_kernel)
            const float g = bf2f(f2bf(acc[i][j][v])), u = bf2f(f2bf(acc[i][j + 2][v]));
            yb[(size_t)m * ldy + 16 * j] = f2bf(silu(g) * u);
          }
        }
      }
  }
}

template <int MODE, int PIPE>
static int launch(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, hipStream_t s) {
  const int n_mt = (M + BM - 1) / BM, n_nt = MODE == 0 ? N / BN : N / 128;
  hipLaunchKernelGGL((gemm_big_kernel<MODE, PIPE>), dim3(n_mt * n_nt), dim3(512), 0, s, (const uint16_t*)x, ldx,
                     (const uint16_t*)w, (uint16_t*)y, ldy, M, N, K, n_mt, n_nt);
  return (int)hipGetLastError();
}

}  // namespace big
}  // namespace k8s

// mode 0: y[M][N] = x . w^T (w [N][K], N % 256 == 0);
// mode 1: y[M][N] = silu(x . w[0:N]^T) * (x . w[N:2N]^T) (w [2N][K], N % 128 == 0).
// pipe: 0 plain loop, 1 fragment prefetch across the barrier, 2 the same with two explicit
// fragment sets and a forced read / MFMA interleave.
// K % 32 == 0, ldx % 8 == 0, 16-byte aligned x / w; y row stride ldy >= N.
K8S_API int k8s_gemm_big(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int mode,
                         int pipe, hipStream_t s) {
  using namespace k8s::big;
  if (M <= 0) return 0;
  if (K % BK || K < BK || ldx % 8 || ldx < K || ldy < N || N <= 0 || (mode == 0 && N % BN) ||
      (mode == 1 && N % 128) || (mode != 0 && mode != 1) ||
      ((uintptr_t)x % 16) || ((uintptr_t)w % 16))
    return (int)hipErrorInvalidValue;
  if (pipe < 0 || pipe > 2) return (int)hipErrorInvalidValue;
  if (mode == 0) {
    if (pipe == 2) return launch<0, 2>(x, ldx, w, y, ldy, M, N, K, s);
    return pipe ? launch<0, 1>(x, ldx, w, y, ldy, M, N, K, s) : launch<0, 0>(x, ldx, w, y, ldy, M, N, K, s);
  }
  // the SwiGLU form of pipe 2 spills 24 VGPRs inside the loop (2 x 48 fragment
  // registers + the gate/up epilogue): 978 vs 1204 TFLOP/s at M = 4096
  // (profiles/r3/gemm_big/ab_v2_pipe2.jsonl) -- it runs the pipe-1 loop
  return pipe ? launch<1, 1>(x, ldx, w, y, ldy, M, N, K, s) : launch<1, 0>(x, ldx, w, y, ldy, M, N, K, s);
}
