// Sanitizer driver for the host graph core (graphcore_core.h): random graphs,
// every operator checked against a brute-force reference.  Built with
// -fsanitize=address,undefined by _build.build_graphcore_sanitized and run by
// tests/test_sanitizers.py.  Exit code 0 = all checks passed, no sanitizer report.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "graphcore_core.h"

using gcore::i32;
using gcore::i64;

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                 \
    }                                                             \
  } while (0)

// brute-force walks: relationship-unique paths of min..max hops
static void brute(const std::vector<i64>& es, const std::vector<i64>& ed, const std::vector<i32>& et, i64 start,
                  int min_h, int max_h, int dir, const std::set<i32>* types, std::vector<i64>& path_e, i64 node,
                  std::set<std::vector<i64>>& out) {
  const int d = (int)path_e.size();
  if (d >= min_h) {
    std::vector<i64> key = path_e;
    key.insert(key.begin(), start);
    out.insert(key);
  }
  if (d == max_h) return;
  for (i64 e = 0; e < (i64)es.size(); ++e) {
    if (types && !types->count(et[e])) continue;
    bool used = false;
    for (i64 x : path_e) used |= (x == e);
    if (used) continue;
    if ((dir == 0 || dir == 2) && es[e] == node) {
      path_e.push_back(e);
      brute(es, ed, et, start, min_h, max_h, dir, types, path_e, ed[e], out);
      path_e.pop_back();
    }
    if ((dir == 1 || dir == 2) && ed[e] == node && !(dir == 2 && es[e] == ed[e])) {
      path_e.push_back(e);
      brute(es, ed, et, start, min_h, max_h, dir, types, path_e, es[e], out);
      path_e.pop_back();
    }
  }
}

int main() {
  std::mt19937_64 rng(12345);
  for (int trial = 0; trial < 40; ++trial) {
    const i64 n = 1 + rng() % 12, e = rng() % 30;
    std::vector<i64> es(e), ed(e);
    std::vector<i32> et(e), ek(e);
    for (i64 i = 0; i < e; ++i) {
      es[i] = rng() % n;
      ed[i] = rng() % n;
      et[i] = (i32)(rng() % 3);
      ek[i] = (i32)(rng() % 4);
    }
    std::vector<i64> oip, onb, oei, iip, inb, iei;
    gcore::build_csr(n, es.data(), ed.data(), e, oip, onb, oei);
    gcore::build_csr(n, ed.data(), es.data(), e, iip, inb, iei);
    // CSR: every edge once in its source row, stable order
    for (i64 v = 0; v < n; ++v)
      for (i64 p = oip[v]; p < oip[v + 1]; ++p) {
        CHECK(es[oei[p]] == v && ed[oei[p]] == onb[p]);
        if (p > oip[v]) CHECK(oei[p] > oei[p - 1]);
      }
    CHECK(oip[n] == e);
    // expand with type + key filters
    std::vector<i64> ids;
    for (i64 v = 0; v < n; ++v)
      if (rng() % 2) ids.push_back(v);
    const i32 types[2] = {0, 2};
    for (int kid : {-2, 1}) {
      std::vector<i64> row, oe, on;
      gcore::check_ids(ids.data(), (i64)ids.size(), n);
      gcore::expand(oip.data(), n, onb.data(), oei.data(), ids.data(), (i64)ids.size(), et.data(), ek.data(), types,
                    2, true, kid, row, oe, on);
      std::multiset<std::pair<i64, i64>> got, want;
      for (size_t i = 0; i < row.size(); ++i) got.insert({ids[row[i]], oe[i]});
      for (size_t j = 0; j < ids.size(); ++j)
        for (i64 x = 0; x < e; ++x)
          if (es[x] == ids[j] && (et[x] == 0 || et[x] == 2) && (kid == -2 || ek[x] == kid)) want.insert({ids[j], x});
      CHECK(got == want);
    }
    // walks in all three directions, with and without a type filter
    gcore::Adj g{oip.data(), onb.data(), oei.data(), iip.data(), inb.data(), iei.data(), es.data(), ed.data(),
                 et.data()};
    for (int dir = 0; dir < 3; ++dir)
      for (int filt = 0; filt < 2; ++filt) {
        const int min_h = (int)(rng() % 2), max_h = 1 + (int)(rng() % 3);
        std::vector<i64> starts;
        for (i64 v = 0; v < n; ++v) starts.push_back(v);
        std::vector<i64> rows, nodes, edges, hops;
        gcore::var_length(g, starts.data(), (i64)starts.size(), min_h, max_h, dir, types, 2, filt == 1, rows, nodes,
                          edges, hops);
        std::set<std::vector<i64>> got, want;
        size_t eo = 0;
        for (size_t i = 0; i < rows.size(); ++i) {
          std::vector<i64> key{starts[rows[i]]};
          for (i64 k = 0; k < hops[i]; ++k) key.push_back(edges[eo + k]);
          eo += hops[i];
          got.insert(key);
        }
        std::set<i32> ts{0, 2};
        for (i64 v = 0; v < n; ++v) {
          std::vector<i64> pe;
          brute(es, ed, et, v, min_h, max_h, dir, filt ? &ts : nullptr, pe, v, want);
        }
        CHECK(got == want);
      }
  }
  // substring scan incl. needles at the boundaries and empty strings
  const std::vector<std::string> props = {"secret \"db\" not found", "", "nfs mount failed", "x", "aaab"};
  std::vector<i64> offs{0};
  std::string heap;
  for (auto& p : props) {
    heap += p;
    offs.push_back((i64)heap.size());
  }
  std::vector<i64> ids{0, 1, 2, 3, 4};
  const std::vector<std::pair<std::string, std::vector<bool>>> cases = {
      {"not found", {1, 0, 0, 0, 0}}, {"", {1, 1, 1, 1, 1}}, {"x", {0, 0, 0, 1, 0}},
      {"aab", {0, 0, 0, 0, 1}},       {"b\" n", {1, 0, 0, 0, 0}}, {"nfs mount failed!", {0, 0, 0, 0, 0}}};
  for (auto& c : cases) {
    bool r[5];
    gcore::substr_mask(offs.data(), (const uint8_t*)heap.data(), ids.data(), 5, c.first, r);
    for (int j = 0; j < 5; ++j) CHECK(r[j] == c.second[j]);
  }
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("graphcore sanitizer driver: all checks passed\n");
  return 0;
}
