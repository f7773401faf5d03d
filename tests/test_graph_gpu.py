"""HIP graph kernels vs the host operators on a synthetic k8s graph."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.graph.device import DeviceGraph
    from k8s_llm_rca_amd.graph.synth import generate_cluster
    c = generate_cluster(20000, 40, seed=5)
    return c, DeviceGraph(c.stategraph, "cuda", min_gpu_rows=1)


def test_contains_many(gg):
    c, dg = gg
    g = c.stategraph
    ids = g.label_scan("EVENT")
    needles = c.messages[:8] + ["MountVolume", "", "zzz-not-there"]
    got = dg.contains_many(ids, "message", needles)
    offs, buf = g.string_heap("message")
    from k8s_llm_rca_amd.graph import native
    for q, nd in enumerate(needles):
        exp = native.substr_mask_np(offs, buf, ids, nd.encode())
        assert np.array_equal(got[q], exp), nd[:30]


@pytest.mark.parametrize("direction", ["out", "in", "both"])
@pytest.mark.parametrize("types,key", [(None, None), (["ReferInternal"], None),
                                       (["ReferInternal"], "involvedObject_uid"), (["HasState"], None)])
def test_expand(gg, direction, types, key):
    c, dg = gg
    g = c.stategraph
    ids = np.concatenate([g.label_scan("Pod"), g.label_scan("Event")[:300]])
    dev = g.device
    g.device = None
    try:
        ref = g.expand(ids, direction, types, key)
    finally:
        g.device = dev
    got = dg.expand(ids, direction, types, key)
    a = sorted(zip(*[x.tolist() for x in ref]))
    b = sorted(zip(*[x.tolist() for x in got]))
    assert a == b


@pytest.mark.parametrize("mode", ["strict", "loose"])
def test_state_lookup(gg, mode):
    c, dg = gg
    g = c.stategraph
    from k8s_llm_rca_amd.graph.store import ts_to_ms
    ents = np.concatenate([g.label_scan("Pod"), g.label_scan("nfs"), g.label_scan("ResourceQuota")])
    ts = np.full(len(ents), ts_to_ms("2020-12-12 12:00:00.000"), dtype=np.int64)
    tq = ts + 3_600_000
    dev = g.device
    g.device = None
    try:
        ref = g.state_lookup(ents, ts, None, mode, tq, 10)
    finally:
        g.device = dev
    got = dg.state_lookup(ents, ts, None, mode, tq, 10)
    for a, b in zip(ref, got):
        assert sorted(a.tolist()) == sorted(b.tolist())


@pytest.mark.parametrize("direction", ["out", "both"])
@pytest.mark.parametrize("end_label", [None, "nfs", "Secret"])
def test_walks(gg, direction, end_label):
    c, dg = gg
    g = c.stategraph
    starts = g.label_scan("Pod")[:400]
    dev = g.device
    g.device = None
    try:
        ref = g.var_length(starts, 1, 3 if direction == "out" else 2, direction, ["ReferInternal", "UseExternal"],
                           end_label)
    finally:
        g.device = dev
    rec = dg.walks(starts, 1, 3 if direction == "out" else 2, direction, ["ReferInternal", "UseExternal"], end_label)
    got = [(r[0], tuple(r[2:3 + r[1]]), tuple(r[6:6 + r[1]])) for r in rec.tolist()]
    assert sorted(got) == sorted((r, tuple(n), tuple(e)) for r, n, e in ref)


def test_executor_on_device_matches_host(gg):
    from k8s_llm_rca_amd.graph.cypher import Executor
    c, dg = gg
    g = c.stategraph
    q = ("MATCH (n1:Event)-[s1:HasEvent]->(N1:EVENT) WHERE N1.message contains $message WITH n1, N1, s1 "
         "MATCH (n1:Event)-[r1:ReferInternal]->(n2) WHERE r1.key = 'involvedObject_uid' RETURN distinct n2.kind2")
    for inc in c.incidents[:10]:
        r = Executor(g).run(q, {"message": inc.message})
        assert r and r[0][0] == inc.src_kind


def test_walks_hub_overflow_falls_back_exactly(gg):
    """Starts whose frontier exceeds the kernel's LDS capacity (hub nodes such
    as the StorageClass or a Namespace) are enumerated on the host; the merged
    records keep the host enumeration order."""
    c, dg = gg
    g = c.stategraph
    starts = np.concatenate([g.label_scan("StorageClass"), g.label_scan("Namespace")[:20], g.label_scan("Pod")[:50]])
    dev = g.device
    g.device = None
    try:
        ref = g.var_length(starts, 1, 2, "both", None, None)
    finally:
        g.device = dev
    rec = dg.walks(starts, 1, 2, "both", None, None)
    got = [(r[0], list(r[2:3 + r[1]]), list(r[6:6 + r[1]])) for r in rec.tolist()]
    assert got == [(int(r), list(n), list(e)) for r, n, e in ref]  # same order, not just the same set


def test_batched_pipeline_queries_match_host():
    """16 pipeline threads issue the RCA queries concurrently through the
    batcher (CONTAINS over every EVENT, temporal STATE lookups, the metagraph
    var-length cascade): identical results to the host executor, and the
    calls were coalesced into fewer kernel batches than requests."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import threading
    from k8s_llm_rca_amd.graph.batcher import enable_batching
    from k8s_llm_rca_amd.graph.cypher import Executor
    from k8s_llm_rca_amd.graph.device import to_device
    from k8s_llm_rca_amd.graph.synth import generate_cluster
    from k8s_llm_rca_amd.pipeline import find_metapath as FM
    from k8s_llm_rca_amd.pipeline.check_state import find_strict_states
    c = generate_cluster(10000, 64, seed=9)
    qs = []
    for inc in c.incidents:
        qs.append(("state", FM.Q_SRCKIND, {"message": inc.message}))
        qs.append(("state", find_strict_states(inc.src_kind, inc.involved_id, inc.timestamp), None))
        qs.append(("state", find_strict_states(inc.dest_kind, inc.root_id, inc.timestamp), None))
        qs.append(("meta", FM.Q_DIRECTED, {"srcKind": inc.src_kind, "destKind": inc.dest_kind,
                                           "intermediateKinds": inc.path_kinds[1:-1]}))
        qs.append(("meta", FM.Q_UNDIRECTED, {"srcKind": inc.src_kind, "destKind": inc.dest_kind,
                                             "intermediateKinds": []}))

    def run_all(items):
        out = []
        for which, q, p in items:
            g = c.stategraph if which == "state" else c.metagraph
            out.append([repr(r.values()) for r in Executor(g).run(q, p)])
        return out

    host = run_all(qs)
    bs = []
    for g in (c.stategraph, c.metagraph):
        to_device(g, "cuda")  # no device index: the batcher thread uses the current device
        bs.append(enable_batching(g))
    got = [None] * len(qs)

    def worker(t):
        for i in range(t, len(qs), 16):
            got[i] = run_all([qs[i]])[0]

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for b in bs:
        b.close()
    assert got == host
    req = sum(b.stats["requests"] for b in bs)
    assert req > 0 and sum(b.stats["batches"] for b in bs) < req
    assert sum(g.device.launches for g in (c.stategraph, c.metagraph)) > 0
