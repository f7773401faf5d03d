// Pure C++ core of the host graph operators (no Python): shared by the pybind11
// module (graphcore.cpp) and the sanitizer test driver (graphcore_test.cpp),
// so the exact code the extension runs is what ASan/UBSan exercise
// (SURVEY.md §5.2).  See graphcore.cpp for what each operator replaces.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace gcore {

using i64 = int64_t;
using i32 = int32_t;

// CSR from an edge list (counting sort, stable within a row).
inline void build_csr(i64 n, const i64* s, const i64* d, i64 e, std::vector<i64>& indptr, std::vector<i64>& nbr,
                      std::vector<i64>& eid) {
  indptr.assign(n + 1, 0);
  nbr.resize(e);
  eid.resize(e);
  for (i64 i = 0; i < e; ++i) {
    if (s[i] < 0 || s[i] >= n) throw std::out_of_range("edge endpoint out of range");
    indptr[s[i] + 1]++;
  }
  for (i64 i = 0; i < n; ++i) indptr[i + 1] += indptr[i];
  std::vector<i64> cur(indptr.begin(), indptr.end() - 1);
  for (i64 i = 0; i < e; ++i) {
    const i64 p = cur[s[i]]++;
    nbr[p] = d[i];
    eid[p] = i;
  }
}

// One filtered hop from `ids` (edge type in `tids` if filter_type, key == kid unless kid == -2).
inline void check_ids(const i64* id, i64 m, i64 nn) {
  for (i64 j = 0; j < m; ++j)
    if (id[j] < 0 || id[j] >= nn) throw std::out_of_range("node id out of range");
}

inline void expand(const i64* ip, i64 nn, const i64* nb, const i64* ei, const i64* id, i64 m, const i32* et,
                   const i32* ek, const i32* tt, i64 nt, bool filter_type, i32 kid, std::vector<i64>& row,
                   std::vector<i64>& oe, std::vector<i64>& on) {
  (void)nn;
  for (i64 j = 0; j < m; ++j) {
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

// `prop CONTAINS needle` over a packed heap: memchr prefilter then memcmp.
inline void substr_mask(const i64* o, const uint8_t* b, const i64* id, i64 m, const std::string& needle, bool* r) {
  const size_t L = needle.size();
  if (L == 0) {
    for (i64 j = 0; j < m; ++j) r[j] = true;
    return;
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
}

struct Adj {
  const i64 *op, *on, *oe;  // out CSR: indptr, neighbour, edge id
  const i64 *ip, *in, *ie;  // in CSR
  const i64 *es, *ed;       // edge endpoints
  const i32* et;            // edge types
};

// Relationship-unique walks of min_h..max_h hops; dir 0 out, 1 in, 2 both.
inline void var_length(const Adj& g, const i64* st, i64 ns, int min_h, int max_h, int dir, const i32* tt, i64 nt,
                       bool filter_type, std::vector<i64>& rows, std::vector<i64>& nodes_flat,
                       std::vector<i64>& edges_flat, std::vector<i64>& hops) {
  if (max_h > 16) throw std::invalid_argument("var-length upper bound > 16 not supported");
  struct Frame {
    i64 node;
    int depth;
    i64 p, pend;
    int phase;  // 0: out list, 1: in list
  };
  std::vector<i64> path_nodes(max_h + 1), path_edges(max_h + 1);
  std::vector<Frame> stack;
  auto type_ok = [&](i64 e) {
    if (!filter_type) return true;
    for (i64 t = 0; t < nt; ++t)
      if (g.et[e] == tt[t]) return true;
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
      f.p = g.op[node];
      f.pend = g.op[node + 1];
      f.phase = 0;
    } else {
      f.p = g.ip[node];
      f.pend = g.ip[node + 1];
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
      Frame& f = stack.back();  // not used after the push_back below (which may reallocate)
      if (f.p >= f.pend) {
        if (f.phase == 0 && dir == 2) {
          f.phase = 1;
          f.p = g.ip[f.node];
          f.pend = g.ip[f.node + 1];
          continue;
        }
        stack.pop_back();
        continue;
      }
      const bool outgoing = (f.phase == 0);
      const i64 e = outgoing ? g.oe[f.p] : g.ie[f.p];
      const i64 m = outgoing ? g.on[f.p] : g.in[f.p];
      f.p++;
      if (!outgoing && dir == 2 && g.es[e] == g.ed[e]) continue;  // self-loop seen once
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

}  // namespace gcore
