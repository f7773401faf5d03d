// Graph traversal kernels over the HBM-resident CSR k8s graph (G3-G6).
//
//   substr_search   wave per (needle, row): lanes test 64 start offsets at once
//                   (first/last-byte prefilter, then byte compare) -> CONTAINS
//                   for many incidents' messages against every EVENT in one launch
//   graph_expand    one filtered hop (edge-type set, interned key) of a frontier:
//                   count pass + device scan + fill pass
//   state_lookup    per entity: HasState out-edges valid at ts (tmin <= ts < tmax,
//                   or interval overlap), STATE label filter, first `limit`
//   walks           relationship-unique walks of 1..3 hops from every start
//                   (Cypher -[*1..3]- semantics of find_metapath's queries), with
//                   an end-label filter pushed down; count pass + fill pass
// Node / edge ids are int64 in the host store and int32 on the device.
#include "common.h"

namespace k8s {

__global__ void __launch_bounds__(256) substr_kernel(const long long* __restrict__ offs,
                                                     const uint8_t* __restrict__ heap,
                                                     const long long* __restrict__ ids, int n_rows,
                                                     const uint8_t* __restrict__ needles,
                                                     const int* __restrict__ needle_off, int n_needles,
                                                     uint8_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long pair = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= (long long)n_rows * n_needles) return;
  const int q = (int)(pair / n_rows), row = (int)(pair % n_rows);
  const long long nid = ids[row];
  const uint8_t* s = heap + offs[nid];
  const int len = (int)(offs[nid + 1] - offs[nid]);
  const uint8_t* nd = needles + needle_off[q];
  const int L = needle_off[q + 1] - needle_off[q];
  bool hit = false;
  if (L == 0) {
    hit = true;
  } else if (L <= len) {
    const uint8_t f = nd[0], b = nd[L - 1];
    for (int p0 = 0; p0 <= len - L && !hit; p0 += 64) {
      const int p = p0 + lane;
      bool m = false;
      if (p <= len - L && s[p] == f && s[p + L - 1] == b) {
        m = true;
        for (int i = 1; i < L - 1; ++i)
          if (s[p + i] != nd[i]) {
            m = false;
            break;
          }
      }
      hit = __any(m);
    }
  }
  if (lane == 0) out[(size_t)q * n_rows + row] = hit ? 1 : 0;
}

__device__ __forceinline__ bool type_ok(int t, unsigned type_mask) { return type_mask == 0xFFFFFFFFu || ((type_mask >> t) & 1u); }

// pass 0: counts[i] = matching degree; pass 1: write at offsets[i]
__global__ void __launch_bounds__(256) expand_kernel(const int* __restrict__ indptr, const int* __restrict__ nbr,
                                                     const int* __restrict__ eid, const int* __restrict__ etype,
                                                     const int* __restrict__ ekey, const int* __restrict__ esrc,
                                                     const int* __restrict__ edst, const long long* __restrict__ frontier,
                                                     int n, unsigned type_mask, int key, int skip_self_loops,
                                                     int* __restrict__ counts, const long long* __restrict__ offsets,
                                                     long long* __restrict__ o_row, long long* __restrict__ o_eid,
                                                     long long* __restrict__ o_nbr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int v = (int)frontier[i];
  int c = 0;
  long long w = offsets ? offsets[i] : 0;
  for (int p = indptr[v]; p < indptr[v + 1]; ++p) {
    const int e = eid[p];
    if (!type_ok(etype[e], type_mask)) continue;
    if (key != -2 && ekey[e] != key) continue;
    if (skip_self_loops && esrc[e] == edst[e]) continue;
    if (offsets) {
      o_row[w] = i;
      o_eid[w] = e;
      o_nbr[w] = nbr[p];
      ++w;
    } else {
      ++c;
    }
  }
  if (!offsets) counts[i] = c;
}

// strict: tmin <= ts < tmax ; loose: tmin <= tq_max && tmax > ts
__global__ void __launch_bounds__(256) state_kernel(const int* __restrict__ indptr, const int* __restrict__ nbr,
                                                    const int* __restrict__ eid, const int* __restrict__ etype,
                                                    const int* __restrict__ nlabel, const long long* __restrict__ tmin,
                                                    const long long* __restrict__ tmax, int has_state_type,
                                                    int state_label, int loose, int limit,
                                                    const long long* __restrict__ ents,
                                                    const long long* __restrict__ ts,
                                                    const long long* __restrict__ tqmax, int n,
                                                    long long* __restrict__ out, int* __restrict__ counts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int v = (int)ents[i];
  const long long t = ts[i];
  const long long t2 = loose ? tqmax[i] : t;
  int c = 0;
  for (int p = indptr[v]; p < indptr[v + 1] && c < limit; ++p) {
    const int e = eid[p];
    if (etype[e] != has_state_type) continue;
    if (state_label >= 0 && nlabel[nbr[p]] != state_label) continue;
    if (!(tmin[e] <= t2 && tmax[e] > t)) continue;
    out[(size_t)i * limit + c] = e;
    ++c;
  }
  counts[i] = c;
}

// Walk enumeration (thread per start).  dir: 0 out, 1 in, 2 both.
// Each record: [row, hops, n0, n1, n2, n3, e0, e1, e2] (int32, -1 padded).
struct WalkArgs {
  const int *oip, *onb, *oei, *iip, *inb, *iei, *esrc, *edst, *etype, *nlabel;
  const long long* starts;
  int n, min_h, max_h, dir;
  unsigned type_mask;
  int end_label;
  int* counts;
  const long long* offsets;
  int* out;
};

__device__ __forceinline__ int deg_begin(const WalkArgs& a, int v, int side) { return side == 0 ? a.oip[v] : a.iip[v]; }
__device__ __forceinline__ int deg_end(const WalkArgs& a, int v, int side) { return side == 0 ? a.oip[v + 1] : a.iip[v + 1]; }

__global__ void __launch_bounds__(256) walks_kernel(WalkArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int s0 = (int)a.starts[i];
  const int s_lo = (a.dir == 1) ? 1 : 0, s_hi = (a.dir == 0) ? 0 : 1;
  long long w = a.offsets ? a.offsets[i] : 0;
  int cnt = 0;
  int nodes[4], edges[3];
  nodes[0] = s0;
  auto emit = [&](int hops) {
    if (hops < a.min_h) return;
    if (a.end_label >= 0 && a.nlabel[nodes[hops]] != a.end_label) return;
    if (a.offsets) {
      int* rec = a.out + w * 9;
      rec[0] = i;
      rec[1] = hops;
      for (int k = 0; k < 4; ++k) rec[2 + k] = k <= hops ? nodes[k] : -1;
      for (int k = 0; k < 3; ++k) rec[6 + k] = k < hops ? edges[k] : -1;
      ++w;
    } else {
      ++cnt;
    }
  };
  for (int sd1 = s_lo; sd1 <= s_hi; ++sd1)
    for (int p1 = deg_begin(a, s0, sd1); p1 < deg_end(a, s0, sd1); ++p1) {
      const int e1 = sd1 ? a.iei[p1] : a.oei[p1];
      if (!type_ok(a.etype[e1], a.type_mask)) continue;
      if (sd1 && a.dir == 2 && a.esrc[e1] == a.edst[e1]) continue;
      const int n1 = sd1 ? a.inb[p1] : a.onb[p1];
      edges[0] = e1;
      nodes[1] = n1;
      emit(1);
      if (a.max_h < 2) continue;
      for (int sd2 = s_lo; sd2 <= s_hi; ++sd2)
        for (int p2 = deg_begin(a, n1, sd2); p2 < deg_end(a, n1, sd2); ++p2) {
          const int e2 = sd2 ? a.iei[p2] : a.oei[p2];
          if (e2 == e1 || !type_ok(a.etype[e2], a.type_mask)) continue;
          if (sd2 && a.dir == 2 && a.esrc[e2] == a.edst[e2]) continue;
          const int n2 = sd2 ? a.inb[p2] : a.onb[p2];
          edges[1] = e2;
          nodes[2] = n2;
          emit(2);
          if (a.max_h < 3) continue;
          for (int sd3 = s_lo; sd3 <= s_hi; ++sd3)
            for (int p3 = deg_begin(a, n2, sd3); p3 < deg_end(a, n2, sd3); ++p3) {
              const int e3 = sd3 ? a.iei[p3] : a.oei[p3];
              if (e3 == e1 || e3 == e2 || !type_ok(a.etype[e3], a.type_mask)) continue;
              if (sd3 && a.dir == 2 && a.esrc[e3] == a.edst[e3]) continue;
              edges[2] = e3;
              nodes[3] = sd3 ? a.inb[p3] : a.onb[p3];
              emit(3);
            }
        }
    }
  if (!a.offsets) a.counts[i] = cnt;
}

}  // namespace k8s

using namespace k8s;

K8S_API int k8s_substr_search(const void* offs, const void* heap, const void* ids, int n_rows, const void* needles,
                              int n_needles, const int* needle_off, void* out, hipStream_t s) {
  const long long pairs = (long long)n_rows * n_needles;
  if (pairs <= 0) return 0;
  const long long blocks = (pairs + 3) / 4;
  if (blocks > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(substr_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const long long*)offs,
                     (const uint8_t*)heap, (const long long*)ids, n_rows, (const uint8_t*)needles, needle_off,
                     n_needles, (uint8_t*)out);
  return (int)hipGetLastError();
}

K8S_API int k8s_graph_expand2(const int* indptr, const int* nbr, const int* eid, const int* etype, const int* ekey,
                              const int* esrc, const int* edst, const long long* frontier, int n, int type_mask_i,
                              int key, int skip_self_loops, int* counts, const long long* offsets, long long* o_row,
                              long long* o_eid, long long* o_nbr, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(expand_kernel, dim3((n + 255) / 256), dim3(256), 0, s, indptr, nbr, eid, etype, ekey, esrc, edst,
                     frontier, n, (unsigned)type_mask_i, key, skip_self_loops, counts, offsets, o_row, o_eid, o_nbr);
  return (int)hipGetLastError();
}

K8S_API int k8s_state_lookup(const int* indptr, const int* nbr, const int* eid, const int* etype, const int* nlabel,
                             const long long* tmin, const long long* tmax, int has_state_type, int state_label,
                             int loose, int limit, const long long* ents, const long long* ts, const long long* tqmax,
                             int n, long long* out, int* counts, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(state_kernel, dim3((n + 255) / 256), dim3(256), 0, s, indptr, nbr, eid, etype, nlabel, tmin, tmax,
                     has_state_type, state_label, loose, limit, ents, ts, tqmax, n, out, counts);
  return (int)hipGetLastError();
}

K8S_API int k8s_walks(const int* oip, const int* onb, const int* oei, const int* iip, const int* inb, const int* iei,
                      const int* esrc, const int* edst, const int* etype, const int* nlabel, const long long* starts,
                      int n, int min_h, int max_h, int dir, int type_mask_i, int end_label, int* counts,
                      const long long* offsets, int* out, hipStream_t s) {
  if (n <= 0) return 0;
  if (max_h > 3 || min_h < 1) return (int)hipErrorInvalidValue;
  WalkArgs a{oip, onb, oei, iip, inb, iei, esrc, edst, etype, nlabel, starts, n, min_h, max_h, dir,
             (unsigned)type_mask_i, end_label, counts, offsets, out};
  hipLaunchKernelGGL(walks_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
