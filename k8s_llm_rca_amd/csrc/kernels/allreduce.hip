// Custom all-reduce over xGMI peer memory (B14 in SURVEY.md §2 Part B; §5.8).
//
// For the latency-bound TP all-reduces of decode (16 KiB .. a few MiB, two per
// layer) RCCL's ring pays per-step launch + protocol latency; on a full xGMI
// mesh every GPU can instead READ all its peers directly (7 links at once).
// Each rank owns one IPC-exported, uncached buffer:
//
//   [FLAGS_A 8x256 u32][FLAGS_B 8x256 u32][EPOCH 256 u32][STATUS][DATA 2 x max][RES 2 x max][A2A 2 x 2max]
//
// and every rank maps every peer's buffer (hipIpcOpenMemHandle).  Work is
// split into per-block slices; block b of every rank only ever synchronises
// with block b of the other ranks, through per-(source rank, block) flags, so
// there is no grid-wide barrier:
//   one-shot : stage own slice -> signal(A) -> wait(A) -> sum the slice from all
//              ranks (fixed rank order: bit-identical results on every rank)
//   two-shot : stage -> A -> reduce my 1/N part of the slice into RES ->
//              signal(B) -> wait(B) -> gather the N reduced parts
// (two-shot moves 2(N-1)/N of the data per rank instead of N-1: mid sizes).
// The epoch lives in device memory, so the kernel is HIP-graph capturable:
// ONE counter per rank, read by every block at launch and advanced once per
// call by the last block to finish (an arrival counter), so every block of a
// call -- whatever the call's block count -- uses the same epoch and parity.
// (A per-block counter raced: a call with fewer blocks left the higher blocks'
// epochs behind, and a later call's high block could re-write a parity buffer
// a peer was still reading.)  DATA / RES are double buffered by epoch parity:
// a rank starts call E only after its call E-1 waited for every peer to
// signal E-1, i.e. after every peer's call E-2 -- the last reader of parity
// E & 1 -- had completed (stream order).
// Signals are system-scope release stores into the PEER's flag array, waits
// are system-scope acquire loads of our own; spins are bounded (wall clock)
// and record a timeout in STATUS instead of hanging the GPU.  Once STATUS is
// set every later wait falls through at once (the communicator is dead: its
// epochs no longer match the peers'), so a fault costs one timeout, not one
// per collective; the engine reads STATUS with every sampled step
// (k8s_ar_status_async, ordered before the token copy) and fails its runs.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "knobs.h"

namespace k8s {

constexpr int AR_MAX_WORLD = 8;
constexpr int AR_MAX_BLOCKS = 256;
constexpr int AR_THREADS = 512;
constexpr size_t AR_FLAGS_A = 0;
constexpr size_t AR_FLAGS_B = AR_FLAGS_A + 4 * AR_MAX_WORLD * AR_MAX_BLOCKS;
constexpr size_t AR_EPOCH = AR_FLAGS_B + 4 * AR_MAX_WORLD * AR_MAX_BLOCKS;
constexpr size_t AR_STATUS = AR_EPOCH + 4 * AR_MAX_BLOCKS;  // AR_EPOCH: [0] epoch, [1] arrivals
constexpr size_t AR_FLAGS_P = 20480;  // push epilogue: [source rank][strip] u32 (kPushMaxStrips per rank)
constexpr size_t AR_DATA = 32768;
static_assert(AR_STATUS + 4 <= AR_FLAGS_P && AR_FLAGS_P + 4 * AR_MAX_WORLD * kPushMaxStrips <= AR_DATA,
              "header layout");
// push slots follow DATA / RES / A2A: [parity][source rank][slot], 2 x max_bytes in all
__host__ __device__ inline size_t push_region(long max_bytes) { return AR_DATA + 8 * (size_t)max_bytes; }
static long push_slot(long max_bytes, int world) { return (max_bytes / world) / 16 * 16; }

struct ARPeers {
  unsigned char* base[AR_MAX_WORLD];
};

struct ARCtx {
  ARPeers peers;
  int world, rank;
  long max_bytes;
  uint64_t timeout_ticks;
  bool used;
  int sim;          // loopback stand-in (tp-sim): every "peer" buffer is local, waits are skipped
  void* own_alloc;  // loopback: the one allocation holding all `world` buffers
  int max_blocks;   // grid cap of every collective (the same on every rank; k8s_ar_set_max_blocks)
};

static ARCtx g_ctx[16];

// knob ar_fence_all: the old publish (a system fence in every wave), for A/B (per launch)
static int fence_all() { return knob(kKnobArFenceAll) ? 1 : 0; }

// Publish this block's stores, then raise its flag in every rank's buffer.
// Every storing wave drains its own stores (vmcnt(0)) before the barrier; ONE
// wave then issues ONE system-scope release (the L2 write-back) and the flag
// stores behind an explicit vmcnt(0) (hipcc can drop the fence's own wait:
// MI355X_MICROARCH.md "Compiler hazard").  fence_all = the previous form, a
// system fence in every wave (8 L2 write-backs per block; A/B only).
__device__ __forceinline__ void ar_publish(const ARPeers& P, size_t flags, int world, int rank, int b, uint32_t e,
                                           int fence_all) {
  const int t = threadIdx.x;
  if (fence_all) __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t < world) {
      uint32_t* f = reinterpret_cast<uint32_t*>(P.base[t] + flags) + rank * AR_MAX_BLOCKS + b;
      __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__device__ __forceinline__ void ar_wait(unsigned char* own, size_t flags, int world, int b, uint32_t e,
                                        uint64_t timeout_ticks, int sim) {
  const int t = threadIdx.x;
  if (t < world && !sim) {
    uint32_t* f = reinterpret_cast<uint32_t*>(own + flags) + t * AR_MAX_BLOCKS + b;
    uint32_t* status = reinterpret_cast<uint32_t*>(own + AR_STATUS);
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
      if (wall_clock64() - t0 > timeout_ticks) {
        __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// Push-epilogue consumer wait: the flags of strips [s0, s0 + ns) from every
// source rank, spread over the block's threads (world * ns flags), each spin
// bounded like ar_wait's; then a barrier, so every thread's reads follow every
// thread's acquire.
__device__ __forceinline__ void push_wait(unsigned char* own, int world, int s0, int ns, uint32_t e,
                                          uint64_t timeout_ticks, int sim) {
  if (!sim) {
    uint32_t* status = reinterpret_cast<uint32_t*>(own + AR_STATUS);
    for (int i = threadIdx.x; i < world * ns; i += blockDim.x) {
      uint32_t* f = reinterpret_cast<uint32_t*>(own + AR_FLAGS_P) + (i / ns) * kPushMaxStrips + s0 + i % ns;
      const uint64_t t0 = wall_clock64();
      while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
        if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
        if (wall_clock64() - t0 > timeout_ticks) {
          __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
}

// Sum of `world` bf16 vectors in source-rank order (fp32, then one bf16
// rounding).  WN > 0 (world == WN, the launchers' 2 / 4 / 8 instantiations):
// the WN loads are unconditional and all issued before the first add, so a
// chunk costs ONE memory latency -- an uncached local or xGMI peer read --
// instead of `world` of them in a chain (the runtime-world loop, WN = 0,
// waits for each load before the next: hipcc's waitcnt pass puts a vmcnt(0)
// behind every conditional load; the fused epilogue measured 9-21 us for
// 0.5-4 MiB that way).
template <int WN, typename Addr>
__device__ __forceinline__ u16x8 sum8_ranks(int world, Addr addr) {
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if constexpr (WN > 0) {
    u16x8 v[WN];
#pragma unroll
    for (int p = 0; p < WN; ++p) v[p] = *reinterpret_cast<const u16x8*>(addr(p));
#pragma unroll
    for (int p = 0; p < WN; ++p)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[p][j]);
  } else {
    for (int p = 0; p < world; ++p) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(addr(p));
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
  }
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(acc[j]);
  return r;
}

// sum of the `world` pushed bf16 vectors at byte offset `off` of slot 0 of THIS
// rank's buffer (slots `slot` bytes apart)
template <int WN>
__device__ __forceinline__ u16x8 push_sum8(const unsigned char* own, long slot, int world, size_t off) {
  return sum8_ranks<WN>(world, [&](int p) { return own + off + (size_t)p * slot; });
}

// sum of `world` bf16 vectors [i, i+8) at byte offset `off` of every rank's buffer
template <int WN>
__device__ __forceinline__ u16x8 ar_sum8(const ARPeers& P, int world, size_t off) {
  return sum8_ranks<WN>(world, [&](int p) { return P.base[p] + off; });
}

// n % 8 == 0 (host-checked); slice = elements per block (multiple of 8 * world)
template <bool TWO_SHOT, int WN>
__global__ void __launch_bounds__(AR_THREADS) ar_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                         long n, long slice, int world, int rank, ARPeers P,
                                                         long max_bytes, uint64_t timeout_ticks, int sim,
                                                         int fence_all) {
  const int b = blockIdx.x, t = threadIdx.x;
  unsigned char* own = P.base[rank];
  uint32_t* ep = reinterpret_cast<uint32_t*>(own + AR_EPOCH);
  uint32_t* arrivals = ep + 1;
  __shared__ uint32_t s_e;
  if (t == 0) s_e = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t e = s_e;
  const size_t data = AR_DATA + (size_t)(e & 1u) * max_bytes;
  const size_t res = AR_DATA + 2 * (size_t)max_bytes + (size_t)(e & 1u) * max_bytes;
  const long i0 = (long)b * slice, i1 = min(n, i0 + slice);

  // 1) stage this rank's slice
  for (long i = i0 + 8L * t; i < i1; i += 8L * AR_THREADS)
    *reinterpret_cast<u16x8*>(own + data + 2 * i) = *reinterpret_cast<const u16x8*>(in + i);
  ar_publish(P, AR_FLAGS_A, world, rank, b, e, fence_all);
  ar_wait(own, AR_FLAGS_A, world, b, e, timeout_ticks, sim);

  if (!TWO_SHOT) {
    for (long i = i0 + 8L * t; i < i1; i += 8L * AR_THREADS)
      *reinterpret_cast<u16x8*>(out + i) = ar_sum8<WN>(P, world, data + 2 * i);
  } else {
    const long part = slice / world;
    const long p0 = i0 + (long)rank * part, p1 = min(i1, p0 + part);
    for (long i = p0 + 8L * t; i < p1; i += 8L * AR_THREADS)
      *reinterpret_cast<u16x8*>(own + res + 2 * i) = ar_sum8<WN>(P, world, data + 2 * i);
    ar_publish(P, AR_FLAGS_B, world, rank, b, e, fence_all);
    ar_wait(own, AR_FLAGS_B, world, b, e, timeout_ticks, sim);
    for (long i = i0 + 8L * t; i < i1; i += 8L * AR_THREADS) {
      const int owner = (int)((i - i0) / part);
      *reinterpret_cast<u16x8*>(out + i) = *reinterpret_cast<const u16x8*>(P.base[owner] + res + 2 * i);
    }
  }
  __syncthreads();
  if (t == 0) {  // the last block of this call publishes the epoch for the next one
    const uint32_t d = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1) {
      __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ep, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// TP row-parallel output + residual add + RMSNorm in ONE launch (the o_proj /
// down_proj epilogue of a TP layer): out_row = sum over ranks of `in` (the
// rank's partial, fixed rank order, rounded to bf16 as the all-reduce does),
// res <- bf16(out + res), y = bf16(res * rsqrt(mean(res^2) + eps) * w).
// Replaces all-reduce + rmsnorm (two launches and a [T][H] round trip per
// call, 160 calls per 70B decode step).  Rows are the unit (a norm needs its
// whole row): block b owns rows b, b + nb, ...; its flags are the all-reduce's
// per-(rank, block) flags, on the same epoch sequence.
//   one-shot : every rank sums every peer's row itself (the arithmetic and
//              thread layout of rmsnorm_kernel: bit-identical to AR + norm);
//   two-shot : rank r sums, adds and squares only its 1/N column slice and
//              publishes the bf16 sums + the slice's sum of squares (RES);
//              then every rank takes the N partial sums of squares in rank
//              order (identical inverse norm on every rank) and gathers the
//              slices: 2 (N-1)/N of the row bytes move instead of N-1.
constexpr int AN_THREADS = 256;
constexpr int AN_NC = 4;  // 16-B chunks per thread per row: H <= 8192

__device__ __forceinline__ float an_block_sum(float v, float* scratch) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < AN_THREADS / 64; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

//   PUSH     : the row-parallel GEMM already stored its partial in the slots
//              (push epilogue, common.h K8sPush): no staging, no flag A; wait
//              for the `S` strip flags (one-shot: every strip of every rank;
//              two-shot: this rank's column slice), then the same arithmetic
//              with the local slots as the sum's source (bit-identical).
template <bool TWO_SHOT, bool PUSH, int WN>
__global__ void __launch_bounds__(AN_THREADS) ar_addnorm_kernel(const uint16_t* __restrict__ in,
                                                                 uint16_t* __restrict__ res,
                                                                 const uint16_t* __restrict__ w,
                                                                 uint16_t* __restrict__ y, int T, int H, float eps,
                                                                 int world, int rank, ARPeers P, long max_bytes,
                                                                 uint64_t timeout_ticks, int sim, int fence_all,
                                                                 int S = 0, long pslot = 0) {
  __shared__ float scratch[AN_THREADS / 64];
  __shared__ uint32_t s_e;
  const int b = blockIdx.x, t = threadIdx.x, nb = gridDim.x;
  unsigned char* own = P.base[rank];
  uint32_t* ep = reinterpret_cast<uint32_t*>(own + AR_EPOCH);
  uint32_t* arrivals = ep + 1;
  if (t == 0) s_e = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t e = s_e;
  const size_t data = AR_DATA + (size_t)(e & 1u) * max_bytes;
  const size_t rbuf = AR_DATA + 2 * (size_t)max_bytes + (size_t)(e & 1u) * max_bytes;
  const size_t ssbuf = rbuf + (size_t)T * H * 2;  // [T] fp32 slice sums of squares (two-shot)
  const int nv = H >> 3;
  // PUSH: this parity's slot 0 (slot p = source rank p's partial)
  const size_t pbase = push_region(max_bytes) + (size_t)(e & 1u) * world * pslot;
  const int pw = TWO_SHOT ? H / world : H;  // row length of a push slot

  if constexpr (PUSH) {
    if (TWO_SHOT)
      push_wait(own, world, rank * (S / world), S / world, e, timeout_ticks, sim);
    else
      push_wait(own, world, 0, S, e, timeout_ticks, sim);
  } else {
    // 1) stage this rank's rows
    for (int row = b; row < T; row += nb)
      for (int i = t; i < nv; i += AN_THREADS)
        *reinterpret_cast<u16x8*>(own + data + 2 * ((size_t)row * H + 8 * i)) =
            *reinterpret_cast<const u16x8*>(in + (size_t)row * H + 8 * i);
    ar_publish(P, AR_FLAGS_A, world, rank, b, e, fence_all);
    ar_wait(own, AR_FLAGS_A, world, b, e, timeout_ticks, sim);
  }

  if (!TWO_SHOT) {
    for (int row = b; row < T; row += nb) {
      u16x8 wv[AN_NC];
      float v[AN_NC][8];
      float ss = 0.f;
      // every load of the row first (no store in between for them to wait behind)
      // (unconditional: a chunk past the row re-reads the row's last one, never stored)
      u16x8 a[AN_NC], r0[AN_NC];
#pragma unroll
      for (int c = 0; c < AN_NC; ++c) {
        const int i = min(t + c * AN_THREADS, nv - 1);
        wv[c] = *reinterpret_cast<const u16x8*>(w + 8 * i);
        r0[c] = *reinterpret_cast<const u16x8*>(res + (size_t)row * H + 8 * i);
        a[c] = PUSH ? push_sum8<WN>(own, pslot, world, pbase + 2 * ((size_t)row * pw + 8 * i))
                    : ar_sum8<WN>(P, world, data + 2 * ((size_t)row * H + 8 * i));
      }
#pragma unroll
      for (int c = 0; c < AN_NC; ++c) {
        const int i = t + c * AN_THREADS;
        if (i < nv) {
          u16x8 sv;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            sv[j] = f2bf(bf2f(a[c][j]) + bf2f(r0[c][j]));
            v[c][j] = bf2f(sv[j]);
            ss += v[c][j] * v[c][j];
          }
          *reinterpret_cast<u16x8*>(res + (size_t)row * H + 8 * i) = sv;
        }
      }
      const float inv = rsqrtf(an_block_sum(ss, scratch) / (float)H + eps);
#pragma unroll
      for (int c = 0; c < AN_NC; ++c) {
        const int i = t + c * AN_THREADS;
        if (i < nv) {
          u16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[c][j] * inv * bf2f(wv[c][j]));
          *reinterpret_cast<u16x8*>(y + (size_t)row * H + 8 * i) = o;
        }
      }
    }
  } else {
    const int sl = nv / world;  // 16-B chunks per rank slice (host-checked: nv % world == 0)
    const int c0 = rank * sl;
    for (int row = b; row < T; row += nb) {
      float ss = 0.f;
      for (int i = c0 + t; i < c0 + sl; i += AN_THREADS) {
        const u16x8 a = PUSH ? push_sum8<WN>(own, pslot, world, pbase + 2 * ((size_t)row * pw + 8 * (i - c0)))
                             : ar_sum8<WN>(P, world, data + 2 * ((size_t)row * H + 8 * i));
        const u16x8 r0 = *reinterpret_cast<const u16x8*>(res + (size_t)row * H + 8 * i);
        u16x8 sv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sv[j] = f2bf(bf2f(a[j]) + bf2f(r0[j]));
          const float vj = bf2f(sv[j]);
          ss += vj * vj;
        }
        *reinterpret_cast<u16x8*>(own + rbuf + 2 * ((size_t)row * H + 8 * i)) = sv;
      }
      const float tot = an_block_sum(ss, scratch);
      if (t == 0) *reinterpret_cast<float*>(own + ssbuf + 4 * (size_t)row) = tot;
    }
    ar_publish(P, AR_FLAGS_B, world, rank, b, e, fence_all);
    ar_wait(own, AR_FLAGS_B, world, b, e, timeout_ticks, sim);
    for (int row = b; row < T; row += nb) {
      float tot = 0.f;  // the slices' sums of squares in rank order (loads first when WN > 0)
      if constexpr (WN > 0) {
        float sq[WN];
#pragma unroll
        for (int p = 0; p < WN; ++p) sq[p] = *reinterpret_cast<const float*>(P.base[p] + ssbuf + 4 * (size_t)row);
#pragma unroll
        for (int p = 0; p < WN; ++p) tot += sq[p];
      } else {
        for (int p = 0; p < world; ++p) tot += *reinterpret_cast<const float*>(P.base[p] + ssbuf + 4 * (size_t)row);
      }
      const float inv = rsqrtf(tot / (float)H + eps);
      u16x8 sv[AN_NC], wv[AN_NC];  // the row's peer reads all in flight at once (unconditional, clamped)
#pragma unroll
      for (int c = 0; c < AN_NC; ++c) {
        const int i = min(t + c * AN_THREADS, nv - 1);
        sv[c] = *reinterpret_cast<const u16x8*>(P.base[i / sl] + rbuf + 2 * ((size_t)row * H + 8 * i));
        wv[c] = *reinterpret_cast<const u16x8*>(w + 8 * i);
      }
#pragma unroll
      for (int c = 0; c < AN_NC; ++c) {
        const int i = t + c * AN_THREADS;
        if (i < nv) {
          *reinterpret_cast<u16x8*>(res + (size_t)row * H + 8 * i) = sv[c];
          u16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(sv[c][j]) * inv * bf2f(wv[c][j]));
          *reinterpret_cast<u16x8*>(y + (size_t)row * H + 8 * i) = o;
        }
      }
    }
  }
  __syncthreads();
  if (t == 0) {  // the last block of this call publishes the epoch for the next one
    const uint32_t d = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1) {
      __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ep, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Fixed-size all-to-all (EP token dispatch / combine, B15) over the same IPC
// buffers and the same per-call epoch as the all-reduce (calls of both kinds
// share one epoch sequence, issued in the same order on every rank).  Send
// buffer [world][chunk] bf16 (chunk elements per destination); push model:
// rank r writes its chunk for d straight into d's buffer, region [r], over
// xGMI, signals d, and d copies its regions out once every peer signalled.
// Block b owns the same element range of every chunk on every rank, so a
// block waits only for the peers' block b.  A region of the parity-(e & 1)
// half is rewritten only after every peer signalled epoch e - 1, i.e. after
// its call e - 2 -- the region's last reader -- completed.
__global__ void __launch_bounds__(AR_THREADS) a2a_kernel(const uint16_t* __restrict__ send, uint16_t* __restrict__ recv,
                                                        long chunk, long slice, int world, int rank, ARPeers P,
                                                        long max_bytes, uint64_t timeout_ticks, int sim,
                                                        int fence_all) {
  const int b = blockIdx.x, t = threadIdx.x;
  unsigned char* own = P.base[rank];
  uint32_t* ep = reinterpret_cast<uint32_t*>(own + AR_EPOCH);
  uint32_t* arrivals = ep + 1;
  __shared__ uint32_t s_e;
  if (t == 0) s_e = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  const uint32_t e = s_e;
  // its own region after the all-reduce's DATA / RES: no byte shared between the kinds
  const size_t half = AR_DATA + 4 * (size_t)max_bytes + (size_t)(e & 1u) * 2 * (size_t)max_bytes;
  const long i0 = (long)b * slice, i1 = min(chunk, i0 + slice);
  for (int d = 0; d < world; ++d) {
    unsigned char* dst = P.base[d] + half + 2 * ((size_t)rank * chunk);
    const uint16_t* src = send + (size_t)d * chunk;
    for (long i = i0 + 8L * t; i < i1; i += 8L * AR_THREADS)
      *reinterpret_cast<u16x8*>(dst + 2 * i) = *reinterpret_cast<const u16x8*>(src + i);
  }
  ar_publish(P, AR_FLAGS_A, world, rank, b, e, fence_all);
  ar_wait(own, AR_FLAGS_A, world, b, e, timeout_ticks, sim);
  for (int r = 0; r < world; ++r) {
    const unsigned char* srcb = own + half + 2 * ((size_t)r * chunk);
    uint16_t* dst = recv + (size_t)r * chunk;
    for (long i = i0 + 8L * t; i < i1; i += 8L * AR_THREADS)
      *reinterpret_cast<u16x8*>(dst + i) = *reinterpret_cast<const u16x8*>(srcb + 2 * i);
  }
  __syncthreads();
  if (t == 0) {
    const uint32_t d = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1) {
      __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ep, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ar_addnorm_kernel for (two-shot?, push?) x the communicator's world (2 / 4 / 8:
// unconditional peer loads; else the runtime-world loop)
template <bool TS, bool PU>
static void launch_addnorm_w(const ARCtx& c, int nb, const uint16_t* in, uint16_t* res, const uint16_t* w, uint16_t* y,
                             int T, int H, float eps, int S, long pslot, hipStream_t s) {
#define K8S_AN(WN)                                                                                              \
  hipLaunchKernelGGL((ar_addnorm_kernel<TS, PU, WN>), dim3(nb), dim3(AN_THREADS), 0, s, in, res, w, y, T, H, eps, \
                     c.world, c.rank, c.peers, c.max_bytes, c.timeout_ticks, c.sim, fence_all(), S, pslot)
  switch (c.world) {
    case 2: K8S_AN(2); break;
    case 4: K8S_AN(4); break;
    case 8: K8S_AN(8); break;
    default: K8S_AN(0); break;
  }
#undef K8S_AN
}

static int launch_addnorm(const ARCtx& c, bool two_shot, bool push, int nb, const uint16_t* in, uint16_t* res,
                          const uint16_t* w, uint16_t* y, int T, int H, float eps, int S, long pslot, hipStream_t s) {
  if (two_shot && push) launch_addnorm_w<true, true>(c, nb, in, res, w, y, T, H, eps, S, pslot, s);
  else if (two_shot) launch_addnorm_w<true, false>(c, nb, in, res, w, y, T, H, eps, S, pslot, s);
  else if (push) launch_addnorm_w<false, true>(c, nb, in, res, w, y, T, H, eps, S, pslot, s);
  else launch_addnorm_w<false, false>(c, nb, in, res, w, y, T, H, eps, S, pslot, s);
  return (int)hipGetLastError();
}

}  // namespace k8s

using namespace k8s;

// Equal-split all-to-all of bf16: send [world][chunk] -> recv [world][chunk]
// (recv[r] = rank r's send[this rank]); chunk % 8 == 0, world * chunk * 2 <= 2 * max_bytes.
K8S_API int k8s_ar_alltoall_bf16(int id, const void* send, void* recv, long chunk, hipStream_t s) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return (int)hipErrorInvalidValue;
  const ARCtx& c = g_ctx[id];
  if (chunk <= 0) return 0;
  if (chunk % 8 || 2 * chunk * c.world > 2 * c.max_bytes || send == recv) return (int)hipErrorInvalidValue;
  long nb = (chunk + 4095) / 4096;
  if (nb > c.max_blocks) nb = c.max_blocks;
  long slice = (chunk + nb - 1) / nb;
  slice = (slice + 7) / 8 * 8;
  nb = (chunk + slice - 1) / slice;
  hipLaunchKernelGGL(a2a_kernel, dim3((unsigned)nb), dim3(AR_THREADS), 0, s, (const uint16_t*)send, (uint16_t*)recv,
                     chunk, slice, c.world, c.rank, c.peers, c.max_bytes, c.timeout_ticks, c.sim, fence_all());
  return (int)hipGetLastError();
}

// header + DATA / RES (2 x 2 x max) + A2A (2 x 2 x max) + push slots (2 x max)
K8S_API long k8s_ar_buffer_bytes(long max_bytes) { return (long)AR_DATA + 10 * max_bytes; }

K8S_API int k8s_ar_alloc(long bytes, void** out) {
  hipError_t e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*out, 0, (size_t)bytes);
}

K8S_API int k8s_ar_free(void* p) { return (int)hipFree(p); }

K8S_API int k8s_ar_get_handle(void* p, void* handle64) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle64), p);
}

K8S_API int k8s_ar_open_handle(const void* handle64, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

K8S_API int k8s_ar_close_handle(void* p) { return (int)hipIpcCloseMemHandle(p); }

K8S_API int k8s_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// Register the mapped buffers of one communicator; returns an id >= 0.
K8S_API int k8s_ar_register(int world, int rank, void** bases, long max_bytes, double timeout_s) {
  if (world < 1 || world > AR_MAX_WORLD || rank < 0 || rank >= world || max_bytes % 16) return -1;
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  for (int id = 0; id < 16; ++id) {
    if (g_ctx[id].used) continue;
    ARCtx& c = g_ctx[id];
    for (int p = 0; p < AR_MAX_WORLD; ++p) c.peers.base[p] = p < world ? (unsigned char*)bases[p] : nullptr;
    c.world = world;
    c.rank = rank;
    c.max_bytes = max_bytes;
    c.timeout_ticks = (uint64_t)(timeout_s * khz * 1000.0);
    c.sim = 0;
    c.own_alloc = nullptr;
    c.max_blocks = AR_MAX_BLOCKS;
    c.used = true;
    return id;
  }
  return -1;
}

// tp-sim: a `world`-rank communicator whose every buffer lives on THIS GPU
// (one allocation, `world` slots), registered as rank 0 with the waits
// skipped.  The kernels then move exactly the bytes of the real collective
// -- stage, signal every "peer", read every "peer" slot -- but over local HBM
// instead of xGMI: a labelled stand-in for per-rank projections
// (bench --tp-sim), never a collective.
K8S_API int k8s_ar_register_loopback(int world, long max_bytes) {
  if (world < 1 || world > AR_MAX_WORLD || max_bytes % 16) return -1;
  const size_t per = (size_t)k8s_ar_buffer_bytes(max_bytes);
  void* base = nullptr;  // uncached, like the IPC buffers of a real communicator (k8s_ar_alloc)
  if (hipExtMallocWithFlags(&base, per * world, hipDeviceMallocUncached) != hipSuccess) return -1;
  if (hipMemset(base, 0, per * world) != hipSuccess) return -1;
  void* bases[AR_MAX_WORLD];
  for (int p = 0; p < world; ++p) bases[p] = (unsigned char*)base + per * p;
  const int id = k8s_ar_register(world, 0, bases, max_bytes, 1.0);
  if (id < 0) {
    (void)hipFree(base);
    return -1;
  }
  g_ctx[id].sim = 1;
  g_ctx[id].own_alloc = base;
  return id;
}

// Cap the grid of this communicator's collectives (1..AR_MAX_BLOCKS; every rank
// must set the same cap: block b of each rank pairs with block b of the others).
// Ranks that SHARE one GPU (the shared-GPU TP / EP tests) need it: a collective's
// blocks spin until the peer's arrive, and a full-size grid of spinning blocks on
// every CU can leave no room (registers, LDS) for the peer process's next kernel,
// so the peer never reaches the collective.  One rank per GPU never needs it.
K8S_API int k8s_ar_set_max_blocks(int id, int nb) {
  if (id < 0 || id >= 16 || !g_ctx[id].used || nb < 1 || nb > AR_MAX_BLOCKS) return (int)hipErrorInvalidValue;
  g_ctx[id].max_blocks = nb;
  return 0;
}

K8S_API int k8s_ar_unregister(int id) {
  if (id < 0 || id >= 16) return (int)hipErrorInvalidValue;
  if (g_ctx[id].own_alloc) (void)hipFree(g_ctx[id].own_alloc);
  g_ctx[id].own_alloc = nullptr;
  g_ctx[id].used = false;
  return 0;
}

// bf16 all-reduce (sum) of n elements; in == out is allowed.  mode: 1 one-shot, 2 two-shot.
K8S_API int k8s_ar_allreduce_bf16(int id, const void* in, void* out, long n, int mode, hipStream_t s) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return (int)hipErrorInvalidValue;
  const ARCtx& c = g_ctx[id];
  if (n <= 0) return 0;
  if (n % 8 || 2 * n > c.max_bytes) return (int)hipErrorInvalidValue;
  const long unit = 8L * (mode == 2 ? c.world : 1);
  long nb = (n + 4095) / 4096;  // >= 8 KB of bf16 per block
  if (nb > c.max_blocks) nb = c.max_blocks;
  long slice = (n + nb - 1) / nb;
  slice = (slice + unit - 1) / unit * unit;
  nb = (n + slice - 1) / slice;
#define K8S_AR(TS, WN)                                                                                        \
  hipLaunchKernelGGL((ar_kernel<TS, WN>), dim3((unsigned)nb), dim3(AR_THREADS), 0, s, (const uint16_t*)in,         \
                     (uint16_t*)out, n, slice, c.world, c.rank, c.peers, c.max_bytes, c.timeout_ticks, c.sim,       \
                     fence_all())
#define K8S_AR_W(TS)             \
  switch (c.world) {             \
    case 2: K8S_AR(TS, 2); break; \
    case 4: K8S_AR(TS, 4); break; \
    case 8: K8S_AR(TS, 8); break; \
    default: K8S_AR(TS, 0); break; \
  }
  if (mode == 2) {
    K8S_AR_W(true)
  } else {
    K8S_AR_W(false)
  }
#undef K8S_AR_W
#undef K8S_AR
  return (int)hipGetLastError();
}

// Fused TP epilogue (ar_addnorm_kernel): in [T][H] bf16 partial -> res (in/out)
// and y [T][H]; mode 1 one-shot, 2 two-shot.  Same epoch sequence as the
// all-reduce: issue it in the same order on every rank.
K8S_API int k8s_ar_addnorm_bf16(int id, const void* in, void* res, const void* w, void* y, int T, int H, float eps,
                                int mode, hipStream_t s) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return (int)hipErrorInvalidValue;
  const ARCtx& c = g_ctx[id];
  if (T <= 0) return 0;
  const long need = (long)T * H * 2 + 4L * T;  // staged rows / (two-shot) slice sums + sums of squares
  if (H % 8 || H / 8 > AN_THREADS * AN_NC || need > c.max_bytes || (mode == 2 && (H / 8) % c.world))
    return (int)hipErrorInvalidValue;
  const int nb = T < c.max_blocks ? T : c.max_blocks;
  return launch_addnorm(c, mode == 2, false, nb, (const uint16_t*)in, (uint16_t*)res, (const uint16_t*)w,
                        (uint16_t*)y, T, H, eps, 0, 0, s);
}

// ---------------------------------------------------------------- push epilogue
// The TP row-parallel outputs at decode sizes (o / down projections on the
// LDS-DMA stream GEMM, gemm_stream.hip k8s_gemm_stream_push) skip the staging
// copy: the GEMM's epilogue stores each output strip straight into the slots
// the fused all-reduce + add + RMSNorm reads, over xGMI, and raises one flag
// per strip; the consumer (ar_addnorm_kernel<., PUSH>) waits on those flags
// and sums its LOCAL slots.  Two-shot: each strip goes only to the rank that
// owns its columns ((H / world) % strip width == 0), i.e. the push IS the
// reduce-scatter's first leg; one-shot: the whole tile goes to every rank.
// Same epoch sequence as every other collective of the communicator (the GEMM
// reads the epoch, the consumer advances it): a push pair counts as one call.
// Slot parity safety is the all-reduce's argument: a rank pushes call E's
// tile only after its call E-1 waited for every peer's flags of E-1, i.e.
// after every peer finished call E-2, the last reader of parity E & 1.
static int push_check(const ARCtx& c, int N, int T, int mode) {
  const long slot = push_slot(c.max_bytes, c.world);
  if (N % 64 || N / 64 > kPushMaxStrips || T <= 0) return 0;
  if (mode == 1) return (long)T * N * 2 <= slot;
  if (mode != 2 || N % c.world) return 0;
  const int w = N / c.world;
  return w % 128 == 0 && (long)T * w * 2 <= slot;  // every 64- / 128-column strip inside one owner's slice
}

// 1 if a [T][N] row-parallel output of this communicator can take the push
// epilogue in `mode` (1 one-shot, 2 two-shot), else 0.
K8S_API int k8s_ar_push_ok(int id, int N, int T, int mode) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return 0;
  return push_check(g_ctx[id], N, T, mode);
}

// The producer's descriptor (common.h K8sPush) for a [T][N] output in `mode`.
K8S_API int k8s_ar_push_desc(int id, int N, int T, int mode, K8sPush* out) {
  if (id < 0 || id >= 16 || !g_ctx[id].used || !push_check(g_ctx[id], N, T, mode)) return (int)hipErrorInvalidValue;
  const ARCtx& c = g_ctx[id];
  for (int p = 0; p < AR_MAX_WORLD; ++p) out->base[p] = c.peers.base[p];
  out->world = c.world;
  out->rank = c.rank;
  out->two_shot = mode == 2;
  out->H = N;
  out->slot = push_slot(c.max_bytes, c.world);
  out->region = (long)push_region(c.max_bytes);
  out->flags = (long)AR_FLAGS_P;
  out->epoch = (long)AR_EPOCH;
  return 0;
}

// The consumer: residual += sum of the pushed partials, y = rmsnorm(residual) * w
// (res / y [T][H]); S = the producer's strip count (common.h k8s_push_strips).
K8S_API int k8s_ar_push_addnorm_bf16(int id, void* res, const void* w, void* y, int T, int H, float eps, int mode,
                                     int S, hipStream_t s) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return (int)hipErrorInvalidValue;
  const ARCtx& c = g_ctx[id];
  if (T <= 0) return 0;
  const long need = (long)T * H * 2 + 4L * T;  // two-shot: the reduced slices + sums of squares in RES
  if (!push_check(c, H, T, mode) || H / 8 > AN_THREADS * AN_NC || need > c.max_bytes || S < 1 || S > H / 64 ||
      H % S || (mode == 2 && S % c.world))
    return (int)hipErrorInvalidValue;
  const int nb = T < c.max_blocks ? T : c.max_blocks;
  return launch_addnorm(c, mode == 2, true, nb, nullptr, (uint16_t*)res, (const uint16_t*)w, (uint16_t*)y, T, H, eps,
                        S, push_slot(c.max_bytes, c.world), s);
}

// STATUS -> *host (pinned), stream-ordered after everything issued before it:
// read it once an event recorded behind this copy has completed.
K8S_API int k8s_ar_status_async(int id, int* host, hipStream_t s) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return (int)hipErrorInvalidValue;
  return (int)hipMemcpyAsync(host, g_ctx[id].peers.base[g_ctx[id].rank] + AR_STATUS, 4, hipMemcpyDeviceToHost, s);
}

// 0 = healthy, 1 = a wait timed out (a peer never arrived); synchronous read.
K8S_API int k8s_ar_status(int id, int* out) {
  if (id < 0 || id >= 16 || !g_ctx[id].used) return (int)hipErrorInvalidValue;
  uint32_t v = 0;
  hipError_t e = hipMemcpy(&v, g_ctx[id].peers.base[g_ctx[id].rank] + AR_STATUS, 4, hipMemcpyDeviceToHost);
  *out = (int)v;
  return (int)e;
}
