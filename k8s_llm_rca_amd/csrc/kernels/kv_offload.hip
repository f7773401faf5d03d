// Host (pinned DRAM) tier of the paged KV pool (engine/kv_offload.py).
//
// An idle conversation thread's pages leave HBM when the pool runs short and
// come back when the thread's next run is admitted, instead of being dropped
// and re-prefilled.  The PCIe transfer is done by the DMA engines (one
// hipMemcpyAsync per run of consecutive host slots, issued by the tier on its
// own copy stream); this file only gathers a swap's pages from the pool into a
// contiguous HBM staging buffer (PACK) and scatters them back (UNPACK), so the
// DMA never walks the pool's per-layer page layout:
//   pool   k[L][NB][slab], v[L][NB][slab]   slab = one layer's page of one block
//                                             (n_kv x BS x D bf16, V transposed)
//   stage  block i of the launch: [K layer 0..L-1][V layer 0..L-1], 2 L slabs
// A host slot holds exactly one staged block, so stage -> host is a plain
// contiguous copy.  Pure data movement: 16-byte vector loads and stores, no LDS.
#include "common.h"

namespace k8s {

constexpr int kKvMaxIds = 256;  // blocks per launch (the ids travel in the kernel arguments)
struct KvIds {
  int id[kKvMaxIds];
};

// grid (x: slab pieces, y: 2 L (K layers then V layers), z: block of the launch)
template <bool PACK>
__global__ void __launch_bounds__(256) kv_stage_kernel(uint4* __restrict__ pk, uint4* __restrict__ pv,
                                                      uint4* __restrict__ stage, long slab16, int L, long NB,
                                                      KvIds ids) {
  const int i = blockIdx.z, y = blockIdx.y;
  const int kv = y >= L, l = y - kv * L;
  uint4* pool = (kv ? pv : pk) + ((long)l * NB + ids.id[i]) * slab16;
  uint4* st = stage + ((long)i * 2 * L + y) * slab16;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < slab16; e += (long)gridDim.x * 256) {
    if constexpr (PACK)
      st[e] = pool[e];
    else
      pool[e] = st[e];
  }
}

}  // namespace k8s

using namespace k8s;

// pack != 0: stage[i] <- pool pages of block ids[i]; else pool pages <- stage[i].
// ids is a HOST array of n block ids (1 <= n <= 256), each in [0, NB).
K8S_API int k8s_kv_stage(void* k, void* v, void* stage, long slab_bytes, int L, int NB, const int* ids, int n,
                         int pack, hipStream_t s) {
  if (!k || !v || !stage || !ids || n < 1 || n > kKvMaxIds || L < 1 || NB < 1 || slab_bytes <= 0 ||
      slab_bytes % 16 || ((uintptr_t)k | (uintptr_t)v | (uintptr_t)stage) % 16)
    return (int)hipErrorInvalidValue;
  KvIds a;
  for (int i = 0; i < n; ++i) {
    if (ids[i] < 0 || ids[i] >= NB) return (int)hipErrorInvalidValue;
    a.id[i] = ids[i];
  }
  const long slab16 = slab_bytes / 16;
  long gx = slab16 / 1024;  // ~4 pieces per thread
  gx = gx < 1 ? 1 : (gx > 64 ? 64 : gx);
  const dim3 grid((unsigned)gx, 2 * L, n);
  if (pack)
    hipLaunchKernelGGL(kv_stage_kernel<true>, grid, dim3(256), 0, s, (uint4*)k, (uint4*)v, (uint4*)stage, slab16, L,
                       (long)NB, a);
  else
    hipLaunchKernelGGL(kv_stage_kernel<false>, grid, dim3(256), 0, s, (uint4*)k, (uint4*)v, (uint4*)stage, slab16, L,
                       (long)NB, a);
  return (int)hipGetLastError();
}

// The tier's host buffer is an ordinary allocation page-locked here (torch's
// pinned allocator rounds every request up to a power of two: 96 GB would pin 128).
K8S_API int k8s_host_register(void* p, long bytes) {
  return (int)hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault);
}
K8S_API int k8s_host_unregister(void* p) { return (int)hipHostUnregister(p); }

// stage <-> host slots by the DMA engines (registered host memory, so the copy
// is asynchronous on `s`)
K8S_API int k8s_memcpy_async(void* dst, const void* src, long bytes, hipStream_t s) {
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, s);
}
