"""Property-based graph-engine tests (hypothesis): random small multigraphs,
the stage-1 metapath queries (find_metapath Q_DIRECTED / Q_UNDIRECTED, i.e.
``/root/reference/find_metapath/find_srckind_metapath_neo4j.py:60-96``)
against a brute-force enumeration of Cypher's path semantics, and the native
CSR / expansion helpers against their NumPy twins."""
import itertools

import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from k8s_llm_rca_amd.graph import native  # noqa: E402
from k8s_llm_rca_amd.graph.cypher import Executor  # noqa: E402
from k8s_llm_rca_amd.graph.store import PropertyGraph  # noqa: E402
from k8s_llm_rca_amd.pipeline import find_metapath as FM  # noqa: E402

KINDS = ["A", "B", "C", "Namespace", "Event"]
EXCLUDED = {"Event", "Namespace"}


@st.composite
def multigraphs(draw):
    n = draw(st.integers(2, 7))
    kinds = draw(st.lists(st.sampled_from(KINDS), min_size=n, max_size=n))
    edges = draw(st.lists(st.tuples(st.integers(0, n - 1), st.integers(0, n - 1)), max_size=14))
    return kinds, edges


def _build(kinds, edges):
    g = PropertyGraph()
    ids = [g.add_node("K", {"kind": k}) for k in kinds]
    for i, (s, d) in enumerate(edges):
        g.add_edge(ids[s], ids[d], "R", {"key": str(i)})
    return g.finalize(), ids


def _oracle(kinds, edges, src, dst, inter, directed):
    """Every path (n1)-[*1..3]-(n2) as Cypher enumerates it: distinct
    relationships, then the query's filters (no repeated node, no Event /
    Namespace node, an interior node of an intermediate kind if any given)."""
    steps = [(i, s, d) for i, (s, d) in enumerate(edges)]
    if not directed:
        steps += [(i, d, s) for i, (s, d) in enumerate(edges)]
    out = []
    for k in range(1, 4):
        for seq in itertools.product(steps, repeat=k):
            if len({e for e, _, _ in seq}) < k:
                continue  # a relationship appears once per path
            if any(seq[j][2] != seq[j + 1][1] for j in range(k - 1)):
                continue
            nodes = [seq[0][1]] + [d for _, _, d in seq]
            if kinds[nodes[0]] != src or kinds[nodes[-1]] != dst:
                continue
            if len(set(nodes)) < len(nodes) or any(kinds[x] in EXCLUDED for x in nodes):
                continue
            if inter and not any(kinds[x] in inter for x in nodes[1:-1]):
                continue
            out.append((tuple(nodes), tuple(e for e, _, _ in seq)))
    return sorted(out)


@settings(max_examples=80, deadline=None)
@given(multigraphs(), st.sampled_from(["A", "B", "C"]), st.sampled_from(["A", "B", "C"]),
       st.lists(st.sampled_from(["A", "B", "C"]), max_size=2, unique=True), st.booleans())
def test_metapath_queries_match_bruteforce(g, src, dst, inter, directed):
    kinds, edges = g
    graph, ids = _build(kinds, edges)
    q = FM.Q_DIRECTED if directed else FM.Q_UNDIRECTED
    rows = Executor(graph).run(q, {"srcKind": src, "destKind": dst, "intermediateKinds": inter})
    pos = {nid: i for i, nid in enumerate(ids)}
    got = sorted((tuple(pos[n.id] for n in r["path"].nodes), tuple(int(x.id) for x in r["path"].relationships))
                 for r in rows)
    eid = {}  # store edge id -> insertion index (the store may renumber edges)
    for r in rows:
        for rel in r["path"].relationships:
            eid[int(rel.id)] = int(rel["key"])
    got = sorted((nodes, tuple(eid[e] for e in rels)) for nodes, rels in got)
    assert got == _oracle(kinds, edges, src, dst, set(inter), directed)


@settings(max_examples=60, deadline=None)
@given(st.integers(1, 40), st.lists(st.tuples(st.integers(0, 39), st.integers(0, 39)), max_size=120),
       st.integers(0, 2**31 - 1))
def test_native_csr_expand_match_numpy(n, pairs, seed):
    if not native.have_native():
        pytest.skip("native _graphcore not built")
    pairs = [(s % n, d % n) for s, d in pairs]
    src = np.array([s for s, _ in pairs], dtype=np.int64)
    dst = np.array([d for _, d in pairs], dtype=np.int64)
    a = native.build_csr(n, src, dst)
    b = native.build_csr_np(n, src, dst)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    rng = np.random.default_rng(seed)
    e = len(pairs)
    et = rng.integers(0, 3, e).astype(np.int32)
    ek = rng.integers(-1, 4, e).astype(np.int32)
    ids = rng.integers(0, n, 8)
    for tids, kid in [(None, -2), (np.array([1], np.int32), -2), (np.array([0, 2], np.int32), 3)]:
        r1 = native.expand(a[0], a[1], a[2], ids, et, ek, tids, kid)
        r2 = native.expand_np(a[0], a[1], a[2], ids, et, ek, tids, kid)
        for x, y in zip(r1, r2):
            assert np.array_equal(x, y)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.binary(max_size=12), min_size=1, max_size=10), st.binary(max_size=5),
       st.lists(st.integers(0, 9), max_size=12))
def test_native_substring_mask_matches_numpy(strings, needle, picks):
    if not native.have_native():
        pytest.skip("native _graphcore not built")
    offs = np.zeros(len(strings) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for s in strings])
    buf = np.frombuffer(b"".join(strings) or b"\0", dtype=np.uint8).copy()
    ids = np.array([p % len(strings) for p in picks], dtype=np.int64)
    got = native.substr_mask(offs, buf, ids, needle)
    assert np.array_equal(got, native.substr_mask_np(offs, buf, ids, needle))
    assert [bool(x) for x in got] == [needle in strings[i] for i in ids]
