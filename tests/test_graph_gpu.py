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
