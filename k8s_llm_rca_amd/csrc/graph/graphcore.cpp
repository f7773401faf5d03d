// Host-side graph operators for the in-process k8s property graph.
//
// Replaces the server-side work Neo4j does for the reference's queries
// (common/neo4j_query_executor.py:15-24 forwards every query over Bolt):
//   build_csr    - CSR adjacency from an edge list (counting sort, O(N+E))
//   expand       - one filtered hop (edge type set / interned key) from a frontier
//   substr_mask  - `prop CONTAINS needle` over a packed UTF-8 heap (memchr prefilter
//                  on the needle's rarest byte, then memcmp)
//   var_length   - relationship-unique walks of min..max hops (Cypher `-[*a..b]-`
//                  semantics used by find_metapath, find_srckind_metapath_neo4j.py:95-116)
// The batched device versions of these operators are HIP kernels in
// csrc/kernels/graph_kernels.hip; this file is the CPU path and the planner's
// default for small frontiers.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace py = pybind11;
using i64 = int64_t;
using i32 = int32_t;

template <typename T>
using arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <typename T>
static arr<T> make(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return arr<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}

static py::tuple build_csr(i64 n, arr<i64> src, arr<i64> dst) {
  const i64 e = src.size();
  const i64* s = src.data();
  const i64* d = dst.data();
  std::vector<i64> indptr(n + 1, 0), nbr(e), eid(e);
  for (i64 i = 0; i < e; ++i) {
    if (s[i] < 0 || s[i] >= n) throw std::out_of_range("edge endpoint out of range");
    indptr[s[i] + 1]++;
  }
  for (i64 i = 0; i < n; ++i) indptr[i + 1] += indptr[i];
  std::vector<i64> cur(indptr.begin(), indptr.end() - 1);
  for (i64 i = 0; i < e; ++i) {  // stable: edge order preserved within a row
    const i64 p = cur[s[i]]++;
    nbr[p] = d[i];
    eid[p] = i;
  }
  return py::make_tuple(make(std::move(indptr)), make(std::move(nbr)), make(std::move(eid)));
}

static py::tuple expand(arr<i64> indptr, arr<i64> nbr, arr<i64> eid, arr<i64> ids, arr<i32> e_type,
                        arr<i32> e_key, arr<i32> tids, bool filter_type, i32 kid) {
  const i64* ip = indptr.data();
  const i64* nb = nbr.data();
  const i64* ei = eid.data();
  const i64* id = ids.data();
  const i32* et = e_type.data();
  const i32* ek = e_key.data();
  const i32* tt = tids.data();
  const i64 nt = tids.size();
  const i64 nn = indptr.size() - 1;
  std::vector<i64> row, oe, on;
  i64 reserve = 0;
  for (i64 j = 0; j < ids.size(); ++j) {
    if (id[j] < 0 || id[j] >= nn) throw std::out_of_range("node id out of range");
    reserve += ip[id[j] + 1] - ip[id[j]];
  }
  row.reserve(reserve);
  oe.reserve(reserve);
  on.reserve(reserve);
  {
    py::gil_scoped_release nogil;
    for (i64 j = 0; j < ids.size(); ++j) {
      for (i64 p = ip[id[j]]; p < ip[id[j] + 1]; ++p) {
        const i64 e = ei[p];
        if (filter_type) {
          bool ok = false;
          for (i64 t = 0; t < nt; ++t) ok |= (et[e] == tt[t]);
          if (!ok) continue;
        }
        if (kid != -2 && ek[e] != kid) continue;
        row.push_back(j);
        oe.push_back(e);
        on.push_back(nb[p]);
      }
    }
  }
  return py::make_tuple(make(std::move(row)), make(std::move(oe)), make(std::move(on)));
}

static arr<bool> substr_mask(arr<i64> offs, arr<uint8_t> buf, arr<i64> ids, py::bytes needle_b) {
  std::string needle = needle_b;
  const i64* o = offs.data();
  const uint8_t* b = buf.data();
  const i64* id = ids.data();
  const i64 m = ids.size();
  const i64 nn = offs.size() - 1;
  arr<bool> out(m);
  bool* r = out.mutable_data();
  const size_t L = needle.size();
  for (i64 j = 0; j < m; ++j)
    if (id[j] < 0 || id[j] >= nn) throw std::out_of_range("node id out of range");
  py::gil_scoped_release nogil;
  if (L == 0) {
    for (i64 j = 0; j < m; ++j) r[j] = true;
    return out;
  }
  const uint8_t first = (uint8_t)needle[0];
  for (i64 j = 0; j < m; ++j) {
    const uint8_t* s = b + o[id[j]];
    const i64 len = o[id[j] + 1] - o[id[j]];
    bool hit = false;
    i64 pos = 0;
    while (pos + (i64)L <= len) {
      const void* f = memchr(s + pos, first, (size_t)(len - pos - (i64)L + 1));
      if (!f) break;
      const i64 at = (const uint8_t*)f - s;
      if (memcmp(s + at, needle.data(), L) == 0) {
        hit = true;
        break;
      }
      pos = at + 1;
    }
    r[j] = hit;
  }
  return out;
}

// Relationship-unique DFS.  dir: 0 out, 1 in, 2 both (undirected).
static py::tuple var_length(arr<i64> oip, arr<i64> onb, arr<i64> oei, arr<i64> iip, arr<i64> inb,
                            arr<i64> iei, arr<i64> esrc, arr<i64> edst, arr<i32> etype, arr<i64> starts,
                            int min_h, int max_h, int dir, arr<i32> tids, bool filter_type) {
  const i64 *op = oip.data(), *on = onb.data(), *oe = oei.data();
  const i64 *ip = iip.data(), *in = inb.data(), *ie = iei.data();
  const i64 *es = esrc.data(), *ed = edst.data();
  const i32* et = etype.data();
  const i32* tt = tids.data();
  const i64 nt = tids.size();
  const i64* st = starts.data();
  const i64 ns = starts.size();
  if (max_h > 16) throw std::invalid_argument("var-length upper bound > 16 not supported");
  std::vector<i64> rows, nodes_flat, edges_flat, hops;
  {
    py::gil_scoped_release nogil;
    struct Frame {
      i64 node;
      int depth;
      // iteration state over the two adjacency lists
      i64 p, pend;
      int phase;  // 0: out list, 1: in list, 2: done
    };
    std::vector<i64> path_nodes(max_h + 1), path_edges(max_h + 1);
    std::vector<Frame> stack;
    auto type_ok = [&](i64 e) {
      if (!filter_type) return true;
      for (i64 t = 0; t < nt; ++t)
        if (et[e] == tt[t]) return true;
      return false;
    };
    auto emit = [&](i64 row, int depth) {
      rows.push_back(row);
      hops.push_back(depth);
      for (int k = 0; k <= depth; ++k) nodes_flat.push_back(path_nodes[k]);
      for (int k = 0; k < depth; ++k) edges_flat.push_back(path_edges[k]);
    };
    auto init_frame = [&](i64 node, int depth) {
      Frame f{node, depth, 0, 0, 0};
      if (dir == 0 || dir == 2) {
        f.p = op[node];
        f.pend = op[node + 1];
        f.phase = 0;
      } else {
        f.p = ip[node];
        f.pend = ip[node + 1];
        f.phase = 1;
      }
      return f;
    };
    for (i64 r = 0; r < ns; ++r) {
      path_nodes[0] = st[r];
      if (min_h == 0) emit(r, 0);
      if (max_h == 0) continue;
      stack.clear();
      stack.push_back(init_frame(st[r], 0));
      while (!stack.empty()) {
        Frame& f = stack.back();
        if (f.p >= f.pend) {
          if (f.phase == 0 && dir == 2) {
            f.phase = 1;
            f.p = ip[f.node];
            f.pend = ip[f.node + 1];
            continue;
          }
          stack.pop_back();
          continue;
        }
        const bool outgoing = (f.phase == 0);
        const i64 e = outgoing ? oe[f.p] : ie[f.p];
        const i64 m = outgoing ? on[f.p] : in[f.p];
        f.p++;
        if (!outgoing && dir == 2 && es[e] == ed[e]) continue;  // self-loop seen once
        if (!type_ok(e)) continue;
        const int d = f.depth;
        bool used = false;
        for (int k = 0; k < d; ++k) used |= (path_edges[k] == e);
        if (used) continue;
        path_edges[d] = e;
        path_nodes[d + 1] = m;
        if (d + 1 >= min_h) emit(r, d + 1);
        if (d + 1 < max_h) stack.push_back(init_frame(m, d + 1));
      }
    }
  }
  return py::make_tuple(make(std::move(rows)), make(std::move(nodes_flat)), make(std::move(edges_flat)),
                        make(std::move(hops)));
}

PYBIND11_MODULE(_graphcore, m) {
  m.doc() = "k8s_llm_rca_amd native graph operators (CSR build, expand, substring scan, walks)";
  m.def("build_csr", &build_csr);
  m.def("expand", &expand);
  m.def("substr_mask", &substr_mask);
  m.def("var_length", &var_length);
}
