"""Reference import paths (``k8s_llm_rca_amd.compat``): a driver written like
the reference's ``test_all.py:54-131`` runs unchanged against this framework
(scripted replies in place of GPT-4, a synthetic graph file in place of Neo4j)."""
import json

import pytest

from k8s_llm_rca_amd.api.service import AssistantService, ScriptedBackend, set_default_service
from k8s_llm_rca_amd.compat import install


@pytest.fixture()
def ref_env(tmp_path):
    from k8s_llm_rca_amd.graph import io as GIO
    from k8s_llm_rca_amd.graph.synth import generate_cluster
    c = generate_cluster(300, 12, seed=5)
    GIO.save_graph(c.metagraph, str(tmp_path / "metagraph.jsonl"))
    GIO.save_graph(c.stategraph, str(tmp_path / "stategraph.jsonl"))
    inc = next(i for i in c.incidents if i.fault == "secret_missing")
    install()
    yield tmp_path, inc
    set_default_service(None)


def test_reference_driver_runs_on_compat_paths(ref_env):
    tmp, inc = ref_env
    # the reference's module paths
    from check_state.analyze_root_cause import check_statepath, setup_state_semantic_analyzer
    from common.neo4j_query_executor import Neo4jQueryExecutor
    from common.openai_generic_assistant import OpenAIGenericAssistant
    from find_metapath.find_srckind_metapath_neo4j import (build_prompt_template, find_destKind_relevantResources,
                                                          find_metapath, find_native_external_kinds, find_srcKind,
                                                          setup_root_cause_locator)
    from generate_query.generate_query import (extend_metapath_construct_string, generate_cypher_query,
                                               human_generate_cypher_query, run_and_filter_query,
                                               setup_cypher_generator)

    current = {}

    def responder(rs):  # GPT-4 stand-in keyed on the prompt text
        last = rs.thread.messages[-1].text
        if "DestinationKind" in last:
            return "```json\n" + json.dumps({"SourceKind": inc.src_kind, "DestinationKind": inc.dest_kind,
                                             "RelevantResources": inc.path_kinds, "PrimaryPath": []}) + "\n```"
        if "generation-template-1" in last:
            return "```cypher\n" + human_generate_cypher_query(current["mp"], msg) + "\n```"
        if "relevance_score" in last:
            return '{"summary": [], "conclusion": "missing secret", "resolution": "kubectl create secret"}'
        return "the STATE is consistent with the error"

    set_default_service(AssistantService(ScriptedBackend(responder)))
    metagraph = Neo4jQueryExecutor(f"file://{tmp}/metagraph.jsonl", "neo4j", "pw")
    stategraph = Neo4jQueryExecutor(str(tmp / "stategraph.jsonl"), "neo4j", "pw")
    assert isinstance(OpenAIGenericAssistant(), object)
    locator = setup_root_cause_locator()
    generator = setup_cypher_generator()
    analyzer = setup_state_semantic_analyzer()
    native, external = find_native_external_kinds(metagraph)
    template = build_prompt_template(native, external)

    msg = inc.message
    src = find_srcKind(stategraph, msg)
    assert src == inc.src_kind
    dest_relevant = find_destKind_relevantResources(msg, src, template, locator)
    dest = dest_relevant["DestinationKind"]
    inter = [k for k in dest_relevant["RelevantResources"] if k not in (src, dest) and k in native + external]
    paths = find_metapath(metagraph, src, dest, inter)
    assert paths
    n_records = 0
    for p in paths:
        mp = extend_metapath_construct_string(p)
        current["mp"] = mp
        q = generate_cypher_query(mp, msg, generator)
        records = run_and_filter_query(stategraph, q)
        if not records:  # the reference's deterministic fallback (test_all.py:127-131)
            records = run_and_filter_query(stategraph, human_generate_cypher_query(mp, msg))
        for r in records:
            report, clues = check_statepath(stategraph, analyzer, r)
            assert "missing secret" in report
            assert any("does not exist" in c for cs in clues.values() for c in cs)
            n_records += 1
    assert n_records >= 1
    metagraph.close()
    stategraph.close()
