"""OpenAI-Assistants-shaped HTTP API (api/http.py) and its client."""
import pytest

from k8s_llm_rca_amd.api.assistant import GenericAssistant
from k8s_llm_rca_amd.api.graph import GraphQueryExecutor
from k8s_llm_rca_amd.api.http import RemoteAssistantService, create_app
from k8s_llm_rca_amd.api.service import AssistantService, ScriptedBackend
from k8s_llm_rca_amd.engine.grammar import (Choice, Free, Grammar, Lit, Ref, Repeat, grammar_from_json,
                                            grammar_to_json, hinted_render)
from k8s_llm_rca_amd.pipeline.rca import RCAConfig, RCAPipeline, run_batch

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402


def oracle(rs):
    g = rs.response_format
    return hinted_render(g, fill="state inspected") if g is not None else "ok"


def _client():
    svc = AssistantService(ScriptedBackend(oracle))
    return svc, TestClient(create_app(svc))


def test_grammar_json_roundtrip():
    g = Grammar([Lit("{"), Choice(["a", "b"], "k"), Free(7, name="f"),
                 Repeat([Lit("x"), Choice(["1", "2"], "n")], ",", "]", 1, 3, "r"), Ref("k")],
                hints={"k": "b", "r": 2}, name="demo")
    assert grammar_from_json(grammar_to_json(g)) == g


def test_rest_roundtrip_and_errors():
    svc, c = _client()
    a = c.post("/v1/assistants", json={"instructions": "be terse", "name": "t", "model": "llama3-8b"}).json()
    t = c.post("/v1/threads", json={}).json()
    assert c.get(f"/v1/threads/{t['id']}").json()["id"] == t["id"]
    c.post(f"/v1/threads/{t['id']}/messages", json={"role": "user", "content": "hello"})
    g = Grammar([Lit('{"x": '), Choice(['"p"', '"q"'], "c"), Lit("}")], hints={"c": '"q"'})
    r = c.post(f"/v1/threads/{t['id']}/runs", json={"assistant_id": a["id"], "response_format":
               {"type": "k8s_grammar", "grammar": grammar_to_json(g)}, "max_completion_tokens": 20}).json()
    r = c.get(f"/v1/threads/{t['id']}/runs/{r['id']}", params={"wait": 10}).json()
    assert r["status"] == "completed" and r["usage"]["total_tokens"] > 0
    msgs = c.get(f"/v1/threads/{t['id']}/messages", params={"limit": 1}).json()["data"]
    assert msgs[0]["role"] == "assistant" and msgs[0]["content"][0]["text"]["value"] == '{"x": "q"}'
    assert len(c.get(f"/v1/threads/{t['id']}/runs").json()["data"]) == 1
    assert c.get("/v1/threads/nope").status_code == 404
    assert c.post(f"/v1/threads/{t['id']}/runs", json={"assistant_id": "nope"}).status_code == 404
    assert c.post(f"/v1/threads/{t['id']}/runs", json={"assistant_id": a["id"],
                                                       "response_format": {"type": "xml"}}).status_code == 400
    m = c.get("/metrics").text
    assert 'k8srca_runs{status="completed"} 1.0' in m
    assert c.delete(f"/v1/threads/{t['id']}").json()["deleted"]


def test_generic_assistant_over_http():
    svc, c = _client()
    ga = GenericAssistant(RemoteAssistantService(c))
    ga.create_assistant("inst", "name", "llama3-8b")
    ga.create_thread()
    ga.add_message("message one")
    ga.run_assistant(max_tokens=8)
    m = ga.wait_get_last_k_message(1, timeout=30)
    assert m is not None and m.data[0].text == "ok"
    usage = ga.get_token_usage(0, 1e12, 10)
    assert usage["completion_tokens"] > 0


def test_rca_pipeline_over_http_matches_in_process(small_cluster):
    """The whole three-stage pipeline against the REST server gives the same
    results as against the in-process service."""
    svc, c = _client()
    remote = RemoteAssistantService(c)
    meta, state = GraphQueryExecutor(small_cluster.metagraph), GraphQueryExecutor(small_cluster.stategraph)
    incs = small_cluster.incidents[:4]
    st_http = run_batch(lambda: RCAPipeline(remote, meta, state, RCAConfig(hints=True)),
                        [i.message for i in incs], concurrency=2, truths=incs)
    local = AssistantService(ScriptedBackend(oracle))
    st_local = run_batch(lambda: RCAPipeline(local, meta, state, RCAConfig(hints=True)),
                         [i.message for i in incs], concurrency=2, truths=incs)
    assert not st_http.errors

    def strip(r):
        return {k: v for k, v in r.items() if k not in ("time_cost", "token_usage")}
    assert [strip(r) for r in st_http.results] == [strip(r) for r in st_local.results]


def test_cli_serve_and_remote_run(tmp_path):
    """`serve` (oracle backend) in one process, `run --server` in another, over TCP."""
    import json
    import os
    import socket
    import subprocess
    import sys
    import time

    import httpx
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    srv = subprocess.Popen([sys.executable, "-m", "k8s_llm_rca_amd", "serve", "--backend", "oracle", "--port",
                            str(port), "--graph-nodes", "300", "--incidents", "4"], env=env,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        url = f"http://127.0.0.1:{port}"
        for _ in range(200):
            try:
                if httpx.get(url + "/health", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.1)
        out = tmp_path / "res.json"
        r = subprocess.run([sys.executable, "-m", "k8s_llm_rca_amd", "run", "--server", url, "--graph-nodes",
                            "300", "--incidents", "4", "--limit", "3", "--concurrency", "2", "--output", str(out)],
                           env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        summary = json.loads(r.stdout.strip().splitlines()[-1])
        assert summary["analyses"] == 3 and summary["errors"] == 0
    finally:
        srv.terminate()
        srv.wait(30)


def test_cypher_tx_commit_endpoint(small_cluster):
    """Neo4j HTTP transactional endpoint over the in-process graphs: rows match
    the executor, nodes come back as property maps with node meta, syntax
    errors carry Neo4j's SyntaxError code."""
    svc = AssistantService(ScriptedBackend(lambda rs: "ok"))
    client = TestClient(create_app(svc, graphs={"stategraph": small_cluster.stategraph,
                                                 "metagraph": small_cluster.metagraph}))
    q = "MATCH (n:Pod) RETURN n.id AS name, n LIMIT 3"
    body = client.post("/db/stategraph/tx/commit", json={"statements": [{"statement": q}]}).json()
    assert body["errors"] == []
    res = body["results"][0]
    want = GraphQueryExecutor(small_cluster.stategraph).run_query(q)
    assert res["columns"] == ["name", "n"]
    assert [d["row"][0] for d in res["data"]] == [r["name"] for r in want]
    assert all(d["row"][1]["id"] == d["row"][0] and d["meta"][1]["type"] == "node" for d in res["data"])
    body = client.post("/db/metagraph/tx/commit",
                       json={"statements": [{"statement": "MATCH (n) RETURN count(n) AS c"},
                                            {"statement": "MATCH (n RETURN n"}]}).json()
    assert len(body["results"]) == 1 and body["results"][0]["data"][0]["row"][0] > 0
    assert body["errors"][0]["code"] == "Neo.ClientError.Statement.SyntaxError"
    assert client.post("/db/nope/tx/commit", json={"statements": []}).json()["errors"][0]["code"].endswith(
        "DatabaseNotFound")
