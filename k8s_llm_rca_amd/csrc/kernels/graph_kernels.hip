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
//                   an end-label filter pushed down; wave per start, LDS
//                   frontier, count pass + fill pass
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

// Walk enumeration, one wave per start with the frontier in LDS.
// dir: 0 out, 1 in, 2 both.  Level h (h = 1, 2, 3) flattens every (walk of
// h-1 hops) x (its adjacency entries) pair into one index space: the wave's 64
// lanes take 64 consecutive pairs at a time (a prefix sum of the parents'
// degrees in LDS + a binary search per lane), so a hub node's thousand edges
// are spread over the lanes instead of serialising one thread, and divergence
// is limited to the per-pair predicate.  Valid hop-h walks are compacted
// (ballot + popcount: lane order preserved) into the LDS frontier of level h.
// Every walk is emitted as a record
//   [row, hops, n0, n1, n2, n3, e0, e1, e2, k1, k2, k3]   (int32, -1 padded)
// where k_h is the walk's h-th step in the thread-per-start DFS enumeration
// order (side-major adjacency position); the host sorts records by (row, k1,
// k2, k3) to reproduce that order exactly.  Count pass (offsets == nullptr)
// and fill pass enumerate identically.  A frontier larger than WK_CAP sets
// counts[i] = -1: the host recomputes that start on its own path.
constexpr int WK_CAP = 384;  // 4 waves x 2 levels x 7.7 KB of LDS per block: 2 blocks per CU
constexpr int WK_WAVES = 4;
constexpr int WK_REC = 12;

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

struct WkLevel {
  int node[WK_CAP];
  int edge[WK_CAP];
  int parent[WK_CAP];
  int k[WK_CAP];
  int pre[WK_CAP + 1];  // exclusive prefix of the entries' adjacency sizes
};

// lanes of one wave exchange frontier data through LDS: order the writes
// before the other lanes' reads (compiler and lgkm counter)
__device__ __forceinline__ void wk_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int adj_size(const WalkArgs& a, int v) {
  int d = 0;
  if (a.dir != 1) d += a.oip[v + 1] - a.oip[v];
  if (a.dir != 0) d += a.iip[v + 1] - a.iip[v];
  return d;
}

// the j-th adjacency entry of v (out side first): edge id, neighbour, side
__device__ __forceinline__ void adj_at(const WalkArgs& a, int v, int j, int* e, int* nb, int* side) {
  const int dout = a.dir != 1 ? a.oip[v + 1] - a.oip[v] : 0;
  if (j < dout) {
    const int p = a.oip[v] + j;
    *e = a.oei[p];
    *nb = a.onb[p];
    *side = 0;
  } else {
    const int p = a.iip[v] + (j - dout);
    *e = a.iei[p];
    *nb = a.inb[p];
    *side = 1;
  }
}

// wave-wide exclusive scan of the levels' adjacency sizes into L.pre
__device__ __forceinline__ int wk_prefix(const WalkArgs& a, WkLevel& L, int n, int lane) {
  int carry = 0;
  for (int b = 0; b < n; b += 64) {
    const int i = b + lane;
    int v = i < n ? adj_size(a, L.node[i]) : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (i < n) L.pre[i] = carry + x - v;
    carry += __shfl(x, 63, 64);
  }
  if (lane == 0) L.pre[n] = carry;
  wk_sync();
  return carry;
}

__device__ __forceinline__ int wk_find(const WkLevel& L, int n, int k) {  // last i with pre[i] <= k
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.pre[mid] <= k) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void __launch_bounds__(64 * WK_WAVES) walks_kernel(WalkArgs a) {
  __shared__ WkLevel lv[WK_WAVES][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * WK_WAVES + wv;
  if (i >= a.n) return;  // wave-uniform: no block barrier below
  if (a.offsets && a.counts[i] < 0) return;  // overflowed in the count pass: the host enumerates this start
  WkLevel& L1 = lv[wv][0];
  WkLevel& L2 = lv[wv][1];
  const int s0 = (int)a.starts[i];
  long long w = a.offsets ? a.offsets[i] : 0;
  int cnt = 0;
  bool overflow = false;
  // emit the compacted valid lanes' walks of `hops` hops (lane order)
  auto emit = [&](bool valid, int hops, int n1v, int n2v, int n3v, int e1, int e2, int e3, int k1, int k2, int k3) {
    const int last = hops == 1 ? n1v : hops == 2 ? n2v : n3v;
    const bool ok = valid && hops >= a.min_h && (a.end_label < 0 || a.nlabel[last] == a.end_label);
    const unsigned long long m = __ballot(ok);
    if (ok && a.offsets) {
      const int pos = __popcll(m & ((1ull << lane) - 1ull));
      int* rec = a.out + (w + pos) * WK_REC;
      rec[0] = i;
      rec[1] = hops;
      rec[2] = s0;
      rec[3] = n1v;
      rec[4] = hops >= 2 ? n2v : -1;
      rec[5] = hops >= 3 ? n3v : -1;
      rec[6] = e1;
      rec[7] = hops >= 2 ? e2 : -1;
      rec[8] = hops >= 3 ? e3 : -1;
      rec[9] = k1;
      rec[10] = hops >= 2 ? k2 : -1;
      rec[11] = hops >= 3 ? k3 : -1;
    }
    w += __popcll(m);
    cnt += __popcll(m);
  };
  // ---- hop 1: the start's adjacency
  const int d0 = adj_size(a, s0);
  int n1 = 0;
  for (int b = 0; b < d0; b += 64) {
    const int j = b + lane;
    bool valid = false;
    int e = -1, nb = -1, side = 0;
    if (j < d0) {
      adj_at(a, s0, j, &e, &nb, &side);
      valid = type_ok(a.etype[e], a.type_mask) && !(side && a.dir == 2 && a.esrc[e] == a.edst[e]);
    }
    emit(valid, 1, nb, -1, -1, e, -1, -1, j, -1, -1);
    const unsigned long long m = __ballot(valid && a.max_h >= 2);
    if (valid && a.max_h >= 2) {
      const int pos = n1 + __popcll(m & ((1ull << lane) - 1ull));
      if (pos < WK_CAP) {
        L1.node[pos] = nb;
        L1.edge[pos] = e;
        L1.parent[pos] = -1;
        L1.k[pos] = j;
      }
    }
    n1 += __popcll(m);
  }
  if (n1 > WK_CAP) overflow = true;
  // ---- hop 2
  int n2 = 0;
  if (!overflow && a.max_h >= 2 && n1 > 0) {
    wk_sync();
    const int t2 = wk_prefix(a, L1, n1, lane);
    for (int b = 0; b < t2; b += 64) {
      const int q = b + lane;
      bool valid = false;
      int e = -1, nb = -1, side = 0, pi = 0, jj = 0;
      if (q < t2) {
        pi = wk_find(L1, n1, q);
        jj = q - L1.pre[pi];
        adj_at(a, L1.node[pi], jj, &e, &nb, &side);
        valid = e != L1.edge[pi] && type_ok(a.etype[e], a.type_mask) &&
                !(side && a.dir == 2 && a.esrc[e] == a.edst[e]);
      }
      emit(valid, 2, q < t2 ? L1.node[pi] : -1, nb, -1, q < t2 ? L1.edge[pi] : -1, e, -1, q < t2 ? L1.k[pi] : -1,
           jj, -1);
      const unsigned long long m = __ballot(valid && a.max_h >= 3);
      if (valid && a.max_h >= 3) {
        const int pos = n2 + __popcll(m & ((1ull << lane) - 1ull));
        if (pos < WK_CAP) {
          L2.node[pos] = nb;
          L2.edge[pos] = e;
          L2.parent[pos] = pi;
          L2.k[pos] = jj;
        }
      }
      n2 += __popcll(m);
    }
    if (n2 > WK_CAP) overflow = true;
  }
  // ---- hop 3 (emitted, not stored)
  if (!overflow && a.max_h >= 3 && n2 > 0) {
    wk_sync();
    const int t3 = wk_prefix(a, L2, n2, lane);
    for (int b = 0; b < t3; b += 64) {
      const int q = b + lane;
      bool valid = false;
      int e = -1, nb = -1, side = 0, pi = 0, jj = 0, gp = 0;
      if (q < t3) {
        pi = wk_find(L2, n2, q);
        jj = q - L2.pre[pi];
        gp = L2.parent[pi];
        adj_at(a, L2.node[pi], jj, &e, &nb, &side);
        valid = e != L2.edge[pi] && e != L1.edge[gp] && type_ok(a.etype[e], a.type_mask) &&
                !(side && a.dir == 2 && a.esrc[e] == a.edst[e]);
      }
      emit(valid, 3, q < t3 ? L1.node[gp] : -1, q < t3 ? L2.node[pi] : -1, nb, q < t3 ? L1.edge[gp] : -1,
           q < t3 ? L2.edge[pi] : -1, e, q < t3 ? L1.k[gp] : -1, q < t3 ? L2.k[pi] : -1, jj);
    }
  }
  if (!a.offsets && lane == 0) a.counts[i] = overflow ? -1 : cnt;
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
  hipLaunchKernelGGL(walks_kernel, dim3((n + WK_WAVES - 1) / WK_WAVES), dim3(64 * WK_WAVES), 0, s, a);
  return (int)hipGetLastError();
}
