"""End-to-end pipeline control flow with a scripted (oracle) backend."""
import json

import pytest

from k8s_llm_rca_amd.api.graph import GraphQueryExecutor
from k8s_llm_rca_amd.api.service import AssistantService, ScriptedBackend
from k8s_llm_rca_amd.engine.grammar import hinted_render
from k8s_llm_rca_amd.pipeline import prompts
from k8s_llm_rca_amd.pipeline.rca import Compat, RCAConfig, RCAPipeline, append_result, read_results, run_batch

KEYS = ["error_message", "locator_attempts", "analysis", "time_cost", "token_usage"]


def oracle(rs):
    g = rs.response_format
    return hinted_render(g, fill="state inspected") if g is not None else "ok"


def make(cluster, responder, **cfg):
    svc = AssistantService(ScriptedBackend(responder))
    return RCAPipeline(svc, GraphQueryExecutor(cluster.metagraph), GraphQueryExecutor(cluster.stategraph),
                       RCAConfig(hints=True, **cfg))


def test_batch_all_faults(small_cluster, tmp_path):
    out = tmp_path / "res.json"
    st = run_batch(lambda: make(small_cluster, oracle), small_cluster.messages, concurrency=3,
                   truths=small_cluster.incidents, output_path=str(out))
    assert not st.errors
    assert len(st.results) == len(small_cluster.incidents)
    for inc, r in zip(small_cluster.incidents, st.results):
        assert list(r.keys()) == KEYS
        assert r["locator_attempts"] == 1
        assert r["analysis"], inc.fault
        if inc.fault != "cni_failure":  # CNI messages never name the Node: the reference filters everything
            assert any(a["statepath"] for a in r["analysis"]), inc.fault
        for a in r["analysis"]:
            assert list(a.keys())[:3] == ["extend_metapath", "cypher_query", "cypher_attempts"]
        assert r["token_usage"]["total_tokens"] > 0
    back = read_results(str(out))
    assert len(back) == len(st.results)


def test_root_cause_clue_for_missing_secret(small_cluster):
    p = make(small_cluster, oracle)
    inc = next(i for i in small_cluster.incidents if i.fault == "secret_missing")
    r = p.analyze(inc.message, inc)
    sp = r["analysis"][0]["statepath"][0]
    assert any(f"Secret({inc.root_id})" == k for k in sp["clue"])
    assert "there is not a STATE (SECRET) node" in sp["clue"][f"Secret({inc.root_id})"][0]


def test_locator_repair_loop(small_cluster):
    calls = {"n": 0}

    def bad_then_good(rs):
        if rs.assistant.name == prompts.LOCATOR_NAME:
            calls["n"] += 1
            if calls["n"] == 1:
                return "no fence here"
        return oracle(rs)

    p = make(small_cluster, bad_then_good)
    inc = small_cluster.incidents[2]
    r = p.analyze(inc.message, inc)
    assert r["locator_attempts"] == 2
    msgs = [m.text for m in p.locator.get_all_message().data]
    assert any("An unexpected error occurred" in m for m in msgs)


def test_cypher_repair_and_fallback(small_cluster):
    def bad_cypher(rs):
        if rs.assistant.name == prompts.GENERATOR_NAME:
            return "```cypher\nMATCH (n RETURN n\n```"
        return oracle(rs)

    p = make(small_cluster, bad_cypher)
    inc = next(i for i in small_cluster.incidents if i.fault == "secret_missing")
    r = p.analyze(inc.message, inc)
    a = r["analysis"][0]
    assert a["cypher_attempts"] == 3 and "human_cypher_query" in a and a["statepath"]
    msgs = [m.text for m in p.generator.get_all_message().data]
    assert sum("Cypher Syntax Error occurred" in m for m in msgs) == 3 * len(r["analysis"])


def test_compat_shared_statepath_dict(small_cluster):
    p = make(small_cluster, oracle, compat=Compat(shared_statepath_dict=True))
    inc = next(i for i in small_cluster.incidents if i.fault == "quota_pods")
    r = p.analyze(inc.message, inc)
    sps = [sp for a in r["analysis"] for sp in a["statepath"]]
    assert sps and all(sp is sps[0] for sp in sps)


def test_failed_run_counts_as_attempt(small_cluster):
    def fail_locator(rs):
        if rs.assistant.name == prompts.LOCATOR_NAME:
            raise RuntimeError("engine fault")
        return oracle(rs)

    p = make(small_cluster, fail_locator)
    inc = small_cluster.incidents[0]
    r = p.analyze(inc.message, inc)
    assert r["locator_attempts"] == 3 and r["analysis"] == []


def test_batch_failed_incidents_are_not_throughput(small_cluster):
    """An incident whose analysis raises keeps its ``{"error": ...}`` record in
    the batch output but is not counted as a completed analysis (ADVICE r1:
    failures that end fast must not inflate analyses/s)."""
    msgs = list(small_cluster.messages[:4])

    class Boom(RCAPipeline):
        def analyze(self, message, truth=None):
            if message == msgs[1]:
                raise RuntimeError("injected")
            return super().analyze(message, truth)

    def mk():
        base = make(small_cluster, oracle)
        base.__class__ = Boom
        return base

    st = run_batch(mk, msgs, concurrency=2, truths=small_cluster.incidents[:4])
    assert len(st.results) == 4 and len(st.errors) == 1
    assert st.n_ok == 3
    assert st.analyses_per_s == pytest.approx(3 / st.wall_s)
