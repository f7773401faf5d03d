// Prefill-size projection GEMM (B4, M >= ~1k):
//   Y[M][N] = X[M][K] . W[N][K]^T   bf16 in/out, fp32 accumulate
// with an optional SwiGLU epilogue for the gate_up projection:
//   act[M][I] = silu(X . Wg^T) * (X . Wu^T),  W = [Wg; Wu] ([2I][K], gate rows first)
// so the [M][2I] gate_up activation is never written nor re-read.
//
// Structure: the 256 x 256 x 64 eight-phase schedule of
// cdna_hip_programming.md §5 ("The 256² 8-phase template", T1-T5), built
// for this engine's operand layouts and epilogues:
//   * one 512-thread workgroup per CU, 256 x 256 output tile, K in 64-deep
//     tiles.  LDS = 2 buffers x {X rows 0-127, X rows 128-255, W rows 0-127,
//     W rows 128-255} half-tiles of 128 x 64 bf16 (16 KB each) = 128 KB, one
//     __shared__ array.
//   * a K-tile is four phases, one per 128 x 128 C quadrant (q = (X half,
//     W half) = (0,0) (0,1) (1,1) (1,0)); in every phase each of the 8 waves
//     (2 along M x 4 along N inside the quadrant) issues 16
//     v_mfma_f32_16x16x32_bf16 for its 64 x 32 piece of the quadrant.  The
//     fragments of a quadrant are read in the phase's load segment (X half: 8
//     ds_read_b128, W half: 4), so over a K-tile a wave reads every fragment
//     once (24 reads): the X half of the previous quadrant and the W halves
//     stay in registers.
//   * ping-pong: waves 4-7 (the second wave of every SIMD) run one barrier
//     behind waves 0-3, so on each SIMD one wave issues its MFMA cluster while
//     its partner reads fragments and issues DMAs (MI355X_MICROARCH.md "Two
//     waves per SIMD"); the MFMA cluster sits between s_setprio(1)/(0) (T5).
//   * every phase stages one half-tile by 16-byte LDS-DMA (global_load_lds,
//     2 per thread): W half 1 / X half 1 of tile u+1 in phases 1 / 2, X half 0
//     / W half 0 of tile u+2 in phases 3 / 4 -- each at least two phases after
//     its buffer's last fragment read (the WAR rule, with the stagger), and a
//     counted `s_waitcnt vmcnt(8)` (four half-tiles in flight, never 0 in the
//     loop) in the load segment of the phase before the first read (the RAW
//     rule: wait, then a barrier both groups pass, then read).  Raw s_barrier
//     only: __syncthreads' fence would drain the DMAs in flight.
//   * LDS image: 128-byte rows of 8 16-byte chunks, chunk c of row r stored at
//     c ^ ((r >> 1) & 7).  The swizzle is applied on the DMA SOURCE address
//     (the LDS side is lane-linear, rule 21) and on the fragment read; every
//     16-lane group of a ds_read_b128 then hits 16 distinct 16-byte bank slots.
//   * the MFMA computes Y^T (A operand = W fragment, B = X fragment), so a lane
//     holds 4 consecutive output COLUMNS of one row; W rows are staged in a
//     permuted order so that the lane's two N fragments are columns 8g .. 8g+7:
//     the epilogue stores 16 contiguous bytes per lane (8 for SwiGLU), no LDS.
//     In the SwiGLU form the two fragments are the gate and up rows of the
//     same 4 act columns.
//   * tile order: XCD-aware bijective remap of the workgroup id (each XCD's L2
//     sees a contiguous range of tiles), then groups of GM M tiles x all N tiles
//     (the ~32 tiles an XCD runs at once share 4 X panels and 8 W panels).
//   * split tail (stream-K's role): when the tile count leaves a partial last
//     wave (T = 256 f + r, r < 256), the r tiles of that wave run as r x S work
//     units of K / S each (S <= 4, r S <= 256), so the last wave takes 1/S of a
//     tile's time instead of a whole one.  A unit writes its fp32 partial tile
//     (256 KB, lane-contiguous) to a workspace; the last of a tile's S units to
//     arrive (agent-scope release -> ticket add; acquire -> read the other S-1
//     partials, cdna_hip_programming.md "Projection GEMM at M = 256" item 2)
//     sums them in slice order -- deterministic -- and runs the normal
//     epilogue (SwiGLU included); it resets the ticket for the next launch.
//     The S units of a tile are consecutive after an XCD remap of the units
//     (same XCD, same L2 under round-robin placement; speed only).
//   * grouped (MoE experts, B13 at prefill sizes): G groups of rows
//     goffs[g] .. goffs[g+1] (device offsets, e.g. the token permutation's
//     expert offsets), group g multiplied by weight g; the grid covers
//     ceil(R / 256) + G M tiles (an upper bound computed from the row count R,
//     no host read of the offsets), each workgroup maps its M tile to (group,
//     local tile) from the offsets and the surplus ones exit at once.
//   * split-K (MODE 0, grids of less than one wave: M <= 2048 at N = 4096):
//     `splits` workgroups per tile, consecutive after the remap (one XCD), each
//     over K / splits, writing fp32 partials [splits][M][N] (32 contiguous bytes
//     per lane) that the consumer reduces: the following residual add + RMSNorm
//     or RoPE / KV write in the layer executor (k8s_splitk_addnorm /
//     k8s_splitk_rope_kv, as for the other split-K kernels), else the reduce
//     kernel below.
//
// Rows past M are clamped on load (an L2 hit) and never stored.
// Reference parity: replaces the hipBLASLt call on the prefill path of
// models/llama.py (the reference's GPT-4 prompt processing of the whole thread
// history, /root/reference/common/openai_generic_assistant.py:45-51).
#include <mutex>
#include <type_traits>

#include "common.h"

namespace k8s {
namespace big {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HALF_B = 128 * BK * 2;  // bytes per half-tile (16 KB)
constexpr int BUF_B = 4 * HALF_B;     // one K-tile (64 KB)
constexpr int OX0 = 0, OX1 = HALF_B, OW0 = 2 * HALF_B, OW1 = 3 * HALF_B;
constexpr int GM = 4;  // M tiles per tile group

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const uint16_t* src, unsigned char* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds_dst, 16, 0, 0);
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
using ic = std::integral_constant<int, N>;

// Per-shape MFMA geometry of a wave's 64 x 32 piece of a quadrant.
//   SH 16: v_mfma_f32_16x16x32_bf16, 4 M x 2 N fragments, 2 k-steps of 32
//   SH 32: v_mfma_f32_32x32x16_bf16, 2 M x 1 N fragments, 4 k-steps of 16 (half
//          the register operand bytes per FLOP: MI355X_MICROARCH.md "DVFS
//          give-back" -- the chip may hold a higher clock on one shape)
template <int SH>
struct Geo {
  static constexpr int XT = SH == 16 ? 4 : 2, WT = SH == 16 ? 2 : 1, KS = SH == 16 ? 2 : 4;
  typedef typename std::conditional<SH == 16, f32x4, f32x16>::type acc_t;
  static constexpr int NC = SH == 16 ? 1 : 4;  // f32x4 chunks per accumulator
};

template <int SH>
__device__ __forceinline__ typename Geo<SH>::acc_t mfma(const bf16x8& w, const bf16x8& x,
                                                        const typename Geo<SH>::acc_t& c) {
  if constexpr (SH == 16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, x, c, 0, 0, 0);
}

// chunk c (4 floats) of an accumulator, and its write-back
template <int C>
__device__ __forceinline__ f32x4 chunk(const f32x4& v) {
  return v;
}
template <int C>
__device__ __forceinline__ f32x4 chunk(const f32x16& v) {
  return f32x4{v[4 * C], v[4 * C + 1], v[4 * C + 2], v[4 * C + 3]};
}
template <int C>
__device__ __forceinline__ void set_chunk(f32x4& v, const f32x4& t) {
  v = t;
}
template <int C>
__device__ __forceinline__ void set_chunk(f32x16& v, const f32x4& t) {
  v[4 * C] = t[0];
  v[4 * C + 1] = t[1];
  v[4 * C + 2] = t[2];
  v[4 * C + 3] = t[3];
}

// W row of slab row rho (0..31) of W half h of tile tn: the order that puts a
// lane's output columns next to each other (see the header comment)
// MODE 2 (qkv + RoPE): W half h of tile tn is head 2 tn + h; a wave slab holds 16
// rotation pairs (dims 16 slab + [0, 16) and their partners + 64) laid out like
// SwiGLU's gate / up, so a lane holds whole pairs.
template <int MODE, int SH>
__device__ __forceinline__ int w_row(int tn, int h, int slab, int rho, int N) {
  if constexpr (SH == 16) {
    if constexpr (MODE == 0)  // lane group g of the fragment pair <- columns 8g .. 8g+7
      return tn * BN + 128 * h + 32 * slab + 8 * ((rho >> 2) & 3) + 4 * (rho >> 4) + (rho & 3);
    else if constexpr (MODE == 1)  // fragment 0: gate rows, fragment 1: the up rows of the same act columns
      return (rho >> 4 ? N : 0) + tn * 128 + 64 * h + 16 * slab + (rho & 15);
    else  // fragment 0: dims 16 slab + (rho & 15), fragment 1: their rotation partners
      return tn * BN + 128 * h + (rho >> 4 ? 64 : 0) + 16 * slab + (rho & 15);
  } else {
    // 32x32 accumulator: register r of lane half hh holds fragment row
    // (r & 3) + 8 (r >> 2) + 4 hh; rho -> (r, hh)
    const int r = (rho & 3) + 4 * (rho >> 3), hh = (rho >> 2) & 1;
    if constexpr (MODE == 0)  // lane half hh <- columns 16 hh .. 16 hh + 15 (register order)
      return tn * BN + 128 * h + 32 * slab + 16 * hh + r;
    else if constexpr (MODE == 1)  // registers 0-7: gate of act columns 8 hh .. +7, registers 8-15: their up rows
      return (r >= 8 ? N : 0) + tn * 128 + 64 * h + 16 * slab + 8 * hh + (r & 7);
    else  // registers 0-7: dims 16 slab + 8 hh + [0, 8), registers 8-15: their partners (+ 64)
      return tn * BN + 128 * h + (r >= 8 ? 64 : 0) + 16 * slab + 8 * hh + (r & 7);
  }
}

// MODE 2 epilogue arguments (the unfused path: k8s_rope_kv in norm_act.hip)
struct RopeArgs {
  const int* pos;        // [M] positions
  const float* cos_sin;  // [max_pos][128]: cos of the 64 frequencies, then sin
  const int* slots;      // [M] paged-KV slot (-1: none)
  uint16_t* kc;          // [blocks][nkv][BS][128]
  uint16_t* vc;          // [blocks][nkv][128][BS]
  int nq, nkv, BS;
};

// MODE 0: plain (N output columns = W rows); MODE 1: SwiGLU (N = I output
// act columns, W has 2I rows, I = N); MODE 2: the qkv projection with RoPE on q
// and k and the paged K / V write in the epilogue (N = (nq + 2 nkv) 128; the
// rope_kv_kernel's arithmetic and rounding: bit-identical to GEMM + k8s_rope_kv).
// VAR bit 0: ping-pong stagger of waves
// 4-7; bit 1: s_setprio(1) around the MFMA clusters; bit 2: the 32x32x16 MFMA
// (1 = the default).
template <int MODE, int VAR>
__global__ void __launch_bounds__(512, 1) gemm_big_kernel(const uint16_t* __restrict__ x, int ldx,
                                                          const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                                                          int ldy, int M, int N, int K, int n_mt, int n_nt, int splits,
                                                          float* __restrict__ part, int tail_tiles, int tail_split,
                                                          float* __restrict__ tws, int* __restrict__ tick,
                                                          const int* __restrict__ goffs, int G, RopeArgs ra) {
  constexpr int SH = (VAR & 4) ? 32 : 16;
  using GG = Geo<SH>;
  using acc_t = typename GG::acc_t;
  constexpr int XT = GG::XT, WT = GG::WT, KS = GG::KS;
  __shared__ __attribute__((aligned(1024))) unsigned char sm[2 * BUF_B];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wv >> 2, wc = wv & 3;

  // ---- tile of this workgroup: XCD-contiguous remap, then grouped order
  int tm, tn, slice, nsl = splits, tt = -1;  // tt: tail tile index (split tail), else -1
  {
    // bijective XCD remap of id b within [0, n): blocks b, b+8, ... (one XCD under
    // round-robin placement) get a contiguous id range
    auto remap = [](int b, int n) {
      const int xcd = b & 7, q = n >> 3, r = n & 7;
      return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    };
    const int T = n_mt * n_nt, F = T - tail_tiles, b = blockIdx.x;
    int t;
    if (splits > 1) {  // uniform split-K: units of one tile consecutive
      const int t0 = remap(b, T * splits);
      slice = t0 % splits;
      t = t0 / splits;
    } else if (b < F) {
      t = remap(b, F);
      slice = 0;
      nsl = 1;
    } else {
      const int u = remap(b - F, tail_tiles * tail_split);
      tt = u / tail_split;
      slice = u % tail_split;
      nsl = tail_split;
      t = F + tt;
    }
    const int gsz = GM * n_nt, gid = t / gsz, first_m = gid * GM;
    const int gm = min(n_mt - first_m, GM);
    tm = first_m + (t % gsz) % gm;
    tn = (t % gsz) / gm;
  }
  if (G > 0) {  // grouped: M tile tm -> (group, local tile); rows and weights of that group
    int lm = tm, e = -1;
    for (int gi = 0; gi < G; ++gi) {
      const int a = __builtin_amdgcn_readfirstlane(goffs[gi]), bnd = __builtin_amdgcn_readfirstlane(goffs[gi + 1]);
      const int c = (bnd - a + BM - 1) / BM;
      if (lm < c) {
        e = gi;
        x += (size_t)a * ldx;
        y += (size_t)a * ldy;
        M = bnd - a;
        break;
      }
      lm -= c;
    }
    if (e < 0) return;  // past the last group's tiles (the grid is an upper bound)
    w += (size_t)e * (MODE == 0 ? N : 2 * N) * K;
    tm = lm;
  }
  const int m0 = tm * BM;

  // ---- DMA sources: instruction i of this wave stages half-tile rows
  // 16 wv + 8 i + (lane >> 3), lane's LDS chunk (lane & 7) <- source chunk
  // (lane & 7) ^ ((row >> 1) & 7)
  const uint16_t* xs[2][2];
  const uint16_t* wsrc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int R = 16 * wv + 8 * i + (lane >> 3);
    const int lch = (lane & 7) ^ ((R >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      xs[h][i] = x + (size_t)min(m0 + 128 * h + R, M - 1) * ldx + 8 * lch;
      wsrc[h][i] = w + (size_t)w_row<MODE, SH>(tn, h, R >> 5, R & 31, N) * K + 8 * lch;
    }
  }
  const int nt = K / BK / nsl, kt0 = slice * nt;  // this workgroup's K tiles
  auto issue = [&](const uint16_t* const* src, int lds_off, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(src[i] + (kt0 + kt) * BK, sm + lds_off + (2 * wv + i) * 1024);
  };

  // ---- fragment reads: row (lane & (SH-1)) of an SH-row block, 16-byte k-chunk
  // (lane / SH) + (64 / SH) ks, stored at chunk ^ ((row >> 1) & 7)
  const int frow = lane & (SH - 1), fhi = lane / SH;
  const int f0 = frow * 128 + 16 * (fhi ^ ((frow >> 1) & 7));
  auto fo = [&](int ks) { return f0 ^ (ks * (SH == 16 ? 64 : 32)); };
  const int xoff = 64 * wr * 128, woff = 32 * wc * 128;

  acc_t acc[4][XT][WT];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < XT; ++i)
#pragma unroll
      for (int j = 0; j < WT; ++j) acc[q][i][j] = acc_t{};
  bf16x8 xf[XT][KS], wf0[WT][KS], wf1[WT][KS];

  // prologue: tile 0 whole, tile 1's X half 0 and W half 0 (the main loop's issue order)
  issue(xs[0], OX0, 0);
  issue(wsrc[0], OW0, 0);
  issue(wsrc[1], OW1, 0);
  issue(xs[1], OX1, 0);
  issue(xs[0], BUF_B + OX0, 1);
  issue(wsrc[0], BUF_B + OW0, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's part of X0h(0), W0h(0)
  bar();
  if ((VAR & 1) && wr == 1) bar();  // waves 4-7 run one barrier behind

  auto phase = [&](auto PHc, auto BUFc, int u) {
    constexpr int PH = decltype(PHc)::value, BUF = decltype(BUFc)::value;
    constexpr int B0 = BUF * BUF_B, B1 = (BUF ^ 1) * BUF_B;
    // ---- load segment: this quadrant's new fragments, one half-tile of DMAs
    if constexpr (PH == 1) {
#pragma unroll
      for (int j = 0; j < WT; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          wf0[j][ks] = *reinterpret_cast<const bf16x8*>(sm + B0 + OW0 + woff + SH * j * 128 + fo(ks));
#pragma unroll
      for (int i = 0; i < XT; ++i)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          xf[i][ks] = *reinterpret_cast<const bf16x8*>(sm + B0 + OX0 + xoff + SH * i * 128 + fo(ks));
      issue(wsrc[1], B1 + OW1, min(u + 1, nt - 1));
    } else if constexpr (PH == 2) {
#pragma unroll
      for (int j = 0; j < WT; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          wf1[j][ks] = *reinterpret_cast<const bf16x8*>(sm + B0 + OW1 + woff + SH * j * 128 + fo(ks));
      issue(xs[1], B1 + OX1, min(u + 1, nt - 1));
    } else if constexpr (PH == 3) {
#pragma unroll
      for (int i = 0; i < XT; ++i)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          xf[i][ks] = *reinterpret_cast<const bf16x8*>(sm + B0 + OX1 + xoff + SH * i * 128 + fo(ks));
      issue(xs[0], B0 + OX0, min(u + 2, nt - 1));
    } else {
      issue(wsrc[0], B0 + OW0, min(u + 2, nt - 1));
    }
    // RAW: the half-tile the next phase reads first (X0h/W0h of tile u+1 in
    // phase 4, W1h(u) in phase 1, X1h(u) in phase 2) has landed once at most
    // the four later half-tiles of this wave are in flight
    if constexpr (PH != 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    bar();
    // ---- compute segment: quadrant (X half, W half) = (0,0) (0,1) (1,1) (1,0)
    constexpr int Q = PH - 1;
    if constexpr (VAR & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < XT; ++i)
#pragma unroll
        for (int j = 0; j < WT; ++j) {
          const bf16x8 wfr = (PH == 1 || PH == 4) ? wf0[j][ks] : wf1[j][ks];
          acc[Q][i][j] = mfma<SH>(wfr, xf[i][ks], acc[Q][i][j]);
        }
    if constexpr (VAR & 2) __builtin_amdgcn_s_setprio(0);
    bar();
  };

  for (int u = 0; u < nt; u += 2) {
    phase(ic<1>{}, ic<0>{}, u);
    phase(ic<2>{}, ic<0>{}, u);
    phase(ic<3>{}, ic<0>{}, u);
    phase(ic<4>{}, ic<0>{}, u);
    phase(ic<1>{}, ic<1>{}, u + 1);
    phase(ic<2>{}, ic<1>{}, u + 1);
    phase(ic<3>{}, ic<1>{}, u + 1);
    phase(ic<4>{}, ic<1>{}, u + 1);
  }
  if ((VAR & 1) && wr == 0) bar();                          // equal barrier counts in both groups
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS

  // accumulator chunk k (0..31) of this lane, in a fixed flat order (split-tail partials)
  constexpr int NC = GG::NC;
  auto for_chunks = [&](auto&& fn) {
#pragma unroll
    for (int Q = 0; Q < 4; ++Q)
#pragma unroll
      for (int i = 0; i < XT; ++i)
#pragma unroll
        for (int j = 0; j < WT; ++j) {
          const int k0 = ((Q * XT + i) * WT + j) * NC;
          fn(acc[Q][i][j], k0);
        }
  };

  if (tt >= 0) {
    // split tail: publish this unit's partial; the last of the tile's units sums them
    float* mine = tws + ((size_t)tt * nsl + slice) * (BM * BN) + (size_t)(wv * 32 * 64 + lane) * 4;
    for_chunks([&](acc_t& a, int k0) {
      *reinterpret_cast<f32x4*>(mine + (k0 + 0) * 256) = chunk<0>(a);
      if constexpr (NC == 4) {
        *reinterpret_cast<f32x4*>(mine + (k0 + 1) * 256) = chunk<1>(a);
        *reinterpret_cast<f32x4*>(mine + (k0 + 2) * 256) = chunk<2>(a);
        *reinterpret_cast<f32x4*>(mine + (k0 + 3) * 256) = chunk<3>(a);
      }
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(sm);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(tick + tt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == nsl - 1;
      if (last) {
        __hip_atomic_store(tick + tt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // every partial (this unit's too, from memory: one uniform path) summed in
    // slice order; 16 independent 16-byte loads in flight per slice and half
    // (a per-slice "register or load" branch would wait for each load alone)
    const float* base = tws + (size_t)tt * nsl * (BM * BN) + (size_t)(wv * 32 * 64 + lane) * 4;
#pragma unroll
    for (int hk = 0; hk < 2; ++hk) {
      f32x4 s[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) s[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int sl = 0; sl < nsl; ++sl) {
        f32x4 t[16];
#pragma unroll
        for (int c = 0; c < 16; ++c)
          t[c] = *reinterpret_cast<const f32x4*>(base + (size_t)sl * (BM * BN) + (16 * hk + c) * 256);
#pragma unroll
        for (int c = 0; c < 16; ++c) s[c] += t[c];
      }
      for_chunks([&](acc_t& a, int k0) {
        if (k0 >= 16 * hk && k0 < 16 * hk + 16) {
          set_chunk<0>(a, s[k0 - 16 * hk]);
          if constexpr (NC == 4) {
            set_chunk<1>(a, s[k0 - 16 * hk + 1]);
            set_chunk<2>(a, s[k0 - 16 * hk + 2]);
            set_chunk<3>(a, s[k0 - 16 * hk + 3]);
          }
        }
      });
    }
  }

  // ---- epilogue.  SH 16: acc[Q][i][j][v] = Y[m][n], m = m0 + 128 qx + 64 wr + 16 i + (lane & 15),
  // n = tn*256 + 128 qw + 32 wc + 8 g + 4 j + v (g = lane >> 4).  SH 32: acc[Q][i][0][r],
  // m = m0 + 128 qx + 64 wr + 32 i + (lane & 31), n = tn*256 + 128 qw + 32 wc + 16 hh + r
  // (hh = lane >> 5).  SwiGLU: the two halves of a lane's values are gate and up.
#pragma unroll
  for (int Q = 0; Q < 4; ++Q) {
    const int qx = (Q == 2 || Q == 3) ? 1 : 0, qw = (Q == 1 || Q == 2) ? 1 : 0;
#pragma unroll
    for (int i = 0; i < XT; ++i) {
      const int m = m0 + 128 * qx + 64 * wr + SH * i + (lane & (SH - 1));
      if (m >= M) continue;
      // this lane's values in column order: 8 (SH 16) or 16 (SH 32)
      float v[2 * 4 * WT * GG::NC];
      if constexpr (SH == 16) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[Q][i][0][e];
          v[4 + e] = acc[Q][i][1][e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = acc[Q][i][0][e];
      }
      constexpr int NV = SH == 16 ? 8 : 16;
      if (MODE == 0 && part != nullptr) {  // split-K: fp32 partials [splits][M][N]
        float* o = part + (size_t)slice * M * N + (size_t)m * N + tn * BN + 128 * qw + 32 * wc + NV * fhi;
#pragma unroll
        for (int e = 0; e < NV; e += 4) *reinterpret_cast<f32x4*>(o + e) = f32x4{v[e], v[e + 1], v[e + 2], v[e + 3]};
      } else if (MODE == 2) {
        // head 2 tn + qw; this lane's NA dims d0 .. and their partners d0 + 64
        constexpr int NA = NV / 2;
        const int hd = 2 * tn + qw, d0 = 16 * wc + NA * fhi;
        uint16_t* o = y + (size_t)m * ldy + hd * 128 + d0;
        const int slot = ra.slots ? ra.slots[m] : -1;
        const int blk = slot >= 0 ? slot / ra.BS : 0, off = slot >= 0 ? slot % ra.BS : 0;
        float lo[NA], hi[NA];
        if (hd < ra.nq + ra.nkv) {
          const float* cs = ra.cos_sin + (size_t)ra.pos[m] * 128;
#pragma unroll
          for (int c = 0; c < NA; ++c) {
            const float co = cs[d0 + c], si = cs[64 + d0 + c];
            const float a = bf2f(f2bf(v[c])), b = bf2f(f2bf(v[NA + c]));
            rope_pair(a, b, co, si, lo[c], hi[c]);
          }
        } else {
#pragma unroll
          for (int c = 0; c < NA; ++c) {
            lo[c] = v[c];
            hi[c] = v[NA + c];
          }
        }
        typedef typename std::conditional<NA == 4, u16x4, u16x8>::type ovec;
        ovec olo, ohi;
#pragma unroll
        for (int c = 0; c < NA; ++c) {
          olo[c] = f2bf(lo[c]);
          ohi[c] = f2bf(hi[c]);
        }
        *reinterpret_cast<ovec*>(o) = olo;
        *reinterpret_cast<ovec*>(o + 64) = ohi;
        if (slot >= 0 && hd >= ra.nq) {
          if (hd < ra.nq + ra.nkv) {  // K page row: dims contiguous
            uint16_t* kp = ra.kc + (((size_t)blk * ra.nkv + (hd - ra.nq)) * ra.BS + off) * 128 + d0;
            *reinterpret_cast<ovec*>(kp) = olo;
            *reinterpret_cast<ovec*>(kp + 64) = ohi;
          } else {  // V page: [dim][token]
            uint16_t* vp = ra.vc + ((size_t)blk * ra.nkv + (hd - ra.nq - ra.nkv)) * 128 * ra.BS + off;
#pragma unroll
            for (int c = 0; c < NA; ++c) {
              vp[(size_t)(d0 + c) * ra.BS] = olo[c];
              vp[(size_t)(d0 + 64 + c) * ra.BS] = ohi[c];
            }
          }
        }
      } else if (MODE == 0) {
        uint16_t* o = y + (size_t)m * ldy + tn * BN + 128 * qw + 32 * wc + NV * fhi;
#pragma unroll
        for (int e = 0; e < NV; e += 8) {
          u16x8 ov;
#pragma unroll
          for (int c = 0; c < 8; ++c) ov[c] = f2bf(v[e + c]);
          *reinterpret_cast<u16x8*>(o + e) = ov;
        }
      } else {
        constexpr int NA = NV / 2;  // act outputs of this lane
        uint16_t* o = y + (size_t)m * ldy + tn * 128 + 64 * qw + 16 * wc + NA * fhi;
        // the unfused path's rounding: gate and up rounded to bf16 first (silu_mul_kernel)
        float a[NA];
#pragma unroll
        for (int c = 0; c < NA; ++c) {
          const float gt = bf2f(f2bf(v[c])), up = bf2f(f2bf(v[NA + c]));
          a[c] = silu(gt) * up;
        }
        if constexpr (NA == 4) {
          u16x4 ov;
#pragma unroll
          for (int c = 0; c < 4; ++c) ov[c] = f2bf(a[c]);
          *reinterpret_cast<u16x4*>(o) = ov;
        } else {
          u16x8 ov;
#pragma unroll
          for (int c = 0; c < 8; ++c) ov[c] = f2bf(a[c]);
          *reinterpret_cast<u16x8*>(o) = ov;
        }
      }
    }
  }
}

// Y[m][n] = bf16(sum_s part[s][m][n]) (slice order); 8 outputs per thread.
__global__ void __launch_bounds__(256) big_reduce_kernel(const float* __restrict__ part, int splits,
                                                         uint16_t* __restrict__ y, int ldy, int M, int N) {
  const long idx = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (idx >= (long)M * N) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
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

// Split-tail workspace (per device, set once by the host: k8s_gemm_big_set_ws):
// 256 partial tiles of 256 KB + 256 tickets, zeroed at allocation.  One GEMM at
// a time per workspace: two launches in flight on different streams would mix
// their partials and leave tickets non-zero, and every later launch would then
// sum the wrong slices.  So the workspace belongs to ONE stream: the first
// launch that uses it claims it (g_tail_owner), and a launch on any other
// stream runs without the split tail (whole-tile last wave: slower, never
// wrong).  k8s_gemm_big_set_ws releases the claim.    The engine
// claims it explicitly for its compute stream at init (k8s_gemm_big_claim_ws,
// ADVICE r5), so a short-lived stream that happens to launch first (a capture's
// warm-up, a tuning side stream) can no longer take it; claims are serialised
// by g_tail_mu, so two host threads never both own it.
constexpr int kTailUnits = 256;
constexpr size_t kTailWsBytes = (size_t)kTailUnits * BM * BN * 4 + kTailUnits * 4;
static void* g_tail_ws[16] = {};
static hipStream_t g_tail_owner[16] = {};
static bool g_tail_claimed[16] = {};
static long g_tail_foreign[16] = {};  // launches that skipped the tail (another stream owns it)
static std::mutex g_tail_mu;

// (tail tiles r, split S) for T tiles of nt K-tiles on 256 CUs: the last partial
// wave's r tiles in r x S units (S in {4, 2}: r S <= 256, nt % (2 S) == 0, >= 8 K-tiles each).
static void tail_plan(int T, int nt, int& r, int& S) {
  r = T % 256;
  S = 1;
  if (r == 0) return;
  for (int c : {4, 2})
    if (r * c <= kTailUnits && nt % (2 * c) == 0 && nt / c >= 8) {
      S = c;
      break;
    }
  if (S == 1) r = 0;
}

// MODE 2's epilogue arguments for the next launch (set by k8s_gemm_big_rope;
// host state of the issuing thread, like the executor's launch sequence)
static thread_local RopeArgs g_rope{};

template <int MODE, int VAR>
static int launch(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int splits,
                  float* part, hipStream_t s) {
  const int n_mt = (M + BM - 1) / BM, n_nt = MODE == 1 ? N / 128 : N / BN;
  const int T = n_mt * n_nt;
  int tr = 0, ts = 1;
  float* tws = nullptr;
  int* tick = nullptr;
  if (splits == 1) {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 16 && g_tail_ws[dev]) {
      bool mine;
      {
        std::lock_guard<std::mutex> g(g_tail_mu);
        if (!g_tail_claimed[dev]) {
          g_tail_claimed[dev] = true;
          g_tail_owner[dev] = s;
        }
        mine = g_tail_owner[dev] == s;
      }
      if (!mine) {
        ++g_tail_foreign[dev];
      } else {
        tail_plan(T, K / BK, tr, ts);
        tws = (float*)g_tail_ws[dev];
        tick = (int*)((char*)g_tail_ws[dev] + (size_t)kTailUnits * BM * BN * 4);
      }
    }
  }
  const int grid = splits > 1 ? T * splits : T - tr + tr * ts;
  hipLaunchKernelGGL((gemm_big_kernel<MODE, VAR>), dim3(grid), dim3(512), 0, s, (const uint16_t*)x, ldx,
                     (const uint16_t*)w, (uint16_t*)y, ldy, M, N, K, n_mt, n_nt, splits, part, tr, ts, tws, tick,
                     (const int*)nullptr, 0, g_rope);
  return (int)hipGetLastError();
}

template <int MODE, int VAR>
static int launch_grouped(const void* x, int ldx, const void* w, void* y, int ldy, const int* offs, int G, int R, int N,
                          int K, hipStream_t s) {
  const int n_mt = (R + BM - 1) / BM + G, n_nt = MODE == 0 ? N / BN : N / 128;
  hipLaunchKernelGGL((gemm_big_kernel<MODE, VAR>), dim3(n_mt * n_nt), dim3(512), 0, s, (const uint16_t*)x, ldx,
                     (const uint16_t*)w, (uint16_t*)y, ldy, R, N, K, n_mt, n_nt, 1, (float*)nullptr, 0, 1,
                     (float*)nullptr, (int*)nullptr, offs, G, RopeArgs{});
  return (int)hipGetLastError();
}

}  // namespace big
}  // namespace k8s

static int big_launch(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int mode,
                      int var, int splits, float* part, bool reduce, hipStream_t s) {
  using namespace k8s::big;
  if (M <= 0) return 0;
  if (splits < 1 || K % (2 * BK * splits) || K < 2 * BK || ldx % 8 || ldx < K || ldy < N || N <= 0 ||
      ((mode == 0 || mode == 2) && N % BN) || (mode == 1 && N % 128) || mode < 0 || mode > 2 ||
      ((uintptr_t)x % 16) || ((uintptr_t)w % 16) || (mode != 1 && (ldy % 8 || (uintptr_t)y % 16)) ||
      (mode == 1 && (ldy % 4 || (uintptr_t)y % 8)) || (splits > 1 && (mode != 0 || part == nullptr)))
    return (int)hipErrorInvalidValue;
  if (var != 1 && var != 3 && var != 5 && var != 7) return (int)hipErrorInvalidValue;
  float* pp = splits > 1 ? part : nullptr;
  int rc;
  if (mode == 0) {
    switch (var) {
      case 1: rc = launch<0, 1>(x, ldx, w, y, ldy, M, N, K, splits, pp, s); break;
      case 3: rc = launch<0, 3>(x, ldx, w, y, ldy, M, N, K, splits, pp, s); break;
      case 5: rc = launch<0, 5>(x, ldx, w, y, ldy, M, N, K, splits, pp, s); break;
      default: rc = launch<0, 7>(x, ldx, w, y, ldy, M, N, K, splits, pp, s); break;
    }
  } else if (mode == 1) {
    rc = (var & 4) ? launch<1, 5>(x, ldx, w, y, ldy, M, N, K, 1, nullptr, s)
                   : launch<1, 1>(x, ldx, w, y, ldy, M, N, K, 1, nullptr, s);
  } else {
    rc = (var & 4) ? launch<2, 5>(x, ldx, w, y, ldy, M, N, K, 1, nullptr, s)
                   : launch<2, 1>(x, ldx, w, y, ldy, M, N, K, 1, nullptr, s);
  }
  if (rc || splits == 1 || !reduce) return rc;
  const long blocks = ((long)M * N / 8 + 255) / 256;
  hipLaunchKernelGGL(big_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)part, splits,
                     (uint16_t*)y, ldy, M, N);
  return (int)hipGetLastError();
}

// Grouped (MoE experts): y rows goffs[g] .. goffs[g+1] = x rows of group g times
// weight g (w = [G][N or 2N][K] contiguous; mode 1 = SwiGLU, y = [R][N] act).
// R = rows of x / y (>= goffs[G]); rows past goffs[G] are never read or written.
K8S_API int k8s_gemm_big_grouped(const void* x, int ldx, const void* w, void* y, int ldy, const int* offs, int G, int R,
                                 int N, int K, int mode, int var, hipStream_t s) {
  using namespace k8s::big;
  if (R <= 0) return 0;
  if (G <= 0 || !offs || K % (2 * BK) || ldx % 8 || ldx < K || ldy < N || N <= 0 || (mode == 0 && N % BN) ||
      (mode == 1 && N % 128) || (mode != 0 && mode != 1) || ((uintptr_t)x % 16) || ((uintptr_t)w % 16) ||
      (mode == 0 && (ldy % 8 || (uintptr_t)y % 16)) || (mode == 1 && (ldy % 4 || (uintptr_t)y % 8)))
    return (int)hipErrorInvalidValue;
  const bool sh32 = var & 4;
  if (mode == 0)
    return sh32 ? launch_grouped<0, 5>(x, ldx, w, y, ldy, offs, G, R, N, K, s)
                : launch_grouped<0, 1>(x, ldx, w, y, ldy, offs, G, R, N, K, s);
  return sh32 ? launch_grouped<1, 5>(x, ldx, w, y, ldy, offs, G, R, N, K, s)
              : launch_grouped<1, 1>(x, ldx, w, y, ldy, offs, G, R, N, K, s);
}

// Split-tail workspace of the calling thread's current device: `ws` (device
// memory of k8s_gemm_big_ws_bytes() bytes, ZEROED) or nullptr to disable.
K8S_API long k8s_gemm_big_ws_bytes() { return (long)k8s::big::kTailWsBytes; }
K8S_API int k8s_gemm_big_set_ws(void* ws) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return (int)hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(k8s::big::g_tail_mu);
  k8s::big::g_tail_ws[dev] = ws;
  k8s::big::g_tail_claimed[dev] = false;  // the next launch that uses it claims it for its stream
  return 0;
}
// Give the current device's split-tail workspace to stream `s` (the engine's
// compute stream); launches on every other stream run without the tail.
K8S_API int k8s_gemm_big_claim_ws(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return (int)hipErrorInvalidValue;
  std::lock_guard<std::mutex> g(k8s::big::g_tail_mu);
  if (!k8s::big::g_tail_ws[dev]) return (int)hipErrorInvalidValue;
  k8s::big::g_tail_claimed[dev] = true;
  k8s::big::g_tail_owner[dev] = s;
  return 0;
}
// launches on this device that ran without the split tail because another
// stream owns the workspace (test / diagnostics)
K8S_API long k8s_gemm_big_tail_foreign() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -1;
  return k8s::big::g_tail_foreign[dev];
}

// mode 0: y[M][N] = x . w^T (w [N][K], N % 256 == 0);
// mode 1: y[M][N] = silu(x . w[0:N]^T) * (x . w[N:2N]^T) (w [2N][K], N % 128 == 0).
// var: schedule variant (bit 0: ping-pong stagger, bit 1: s_setprio around the
// MFMA clusters, bit 2: 32x32x16 MFMA; 1 / 3 / 5 / 7 are built).
// K % 128 == 0, ldx % 8 == 0, ldy % 8 (mode 0) / 4 (mode 1) == 0, 16-byte
// aligned x / w / y (8 for y in mode 1); y row stride ldy >= N.
K8S_API int k8s_gemm_big(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int mode,
                         int var, hipStream_t s) {
  return big_launch(x, ldx, w, y, ldy, M, N, K, mode, var, 1, nullptr, true, s);
}

// The qkv projection with its RoPE + paged KV-write epilogue (mode 2): qkv =
// x . w^T with q and k rotated (cos_sin [max_pos][128]) and k / v written to
// their pages (slots[m] < 0: none) -- k8s_gemm_big + k8s_rope_kv in one launch,
// bit-identical.  N = (nq + 2 nkv) * 128, N % 256 == 0.
K8S_API int k8s_gemm_big_rope(const void* x, int ldx, const void* w, void* qkv, int ldq, int M, int N, int K,
                              const int* pos, const float* cos_sin, const int* slots, void* kc, void* vc, int nq,
                              int nkv, int BS, int var, hipStream_t s) {
  using namespace k8s::big;
  if (N != (nq + 2 * nkv) * 128 || !pos || !cos_sin || BS <= 0 || (slots && (!kc || !vc)))
    return (int)hipErrorInvalidValue;
  g_rope = RopeArgs{pos, cos_sin, slots, (uint16_t*)kc, (uint16_t*)vc, nq, nkv, BS};
  const int rc = big_launch(x, ldx, w, qkv, ldq, M, N, K, 2, var, 1, nullptr, true, s);
  g_rope = RopeArgs{};
  return rc;
}

// split-K (mode 0): `splits` K slices (K % (128 splits) == 0) into the fp32
// scratch `part` [splits][M][N], then reduced into y
K8S_API int k8s_gemm_big_split(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int var,
                               int splits, void* part, hipStream_t s) {
  return big_launch(x, ldx, w, y, ldy, M, N, K, 0, var, splits, (float*)part, true, s);
}

// the same, leaving the partials in `part` for a fused consumer (no reduce launch)
K8S_API int k8s_gemm_big_part(const void* x, int ldx, const void* w, void* y, int ldy, int M, int N, int K, int var,
                              int splits, void* part, hipStream_t s) {
  return big_launch(x, ldx, w, y, ldy, M, N, K, 0, var, splits, (float*)part, false, s);
}
