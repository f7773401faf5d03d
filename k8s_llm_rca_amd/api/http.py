"""HTTP serving: an OpenAI-Assistants-shaped REST API over :class:`AssistantService`.

The reference reaches GPT-4 through the OpenAI Assistants REST API
(``common/openai_generic_assistant.py:14-133``: assistants, threads, messages,
runs, run polling, run usage).  ``create_app`` serves the same resources from
the in-process engine, so a client written against that API can point its base
URL at this server:

    POST /v1/assistants                      {instructions, name, model}
    GET  /v1/assistants/{id}
    POST /v1/threads                         {}
    GET  /v1/threads/{id}      DELETE /v1/threads/{id}
    POST /v1/threads/{id}/messages           {role, content}
    GET  /v1/threads/{id}/messages?limit=&order=
    POST /v1/threads/{id}/runs               {assistant_id, instructions?, response_format?,
                                              max_completion_tokens?, temperature?}
    GET  /v1/threads/{id}/runs?limit=&order=
    GET  /v1/threads/{id}/runs/{run_id}?wait=S   (``wait``: long-poll up to S seconds
                                              instead of the reference's 5 s sleep loop)
    POST /v1/threads/{id}/runs/{run_id}/cancel
    GET  /health      GET /metrics (Prometheus: run counts, engine counters)
    POST /db/{name}/tx/commit                {statements: [{statement, parameters}]}
                                              (Neo4j's HTTP transactional endpoint shape,
                                              over the in-process graphs passed as ``graphs``)

``response_format`` is ``{"type": "text"}`` or ``{"type": "k8s_grammar",
"grammar": ...}`` (:func:`..engine.grammar.grammar_to_json`) for constrained
decoding.  :class:`RemoteAssistantService` is the matching client: it has the
``AssistantService`` methods :class:`..api.assistant.GenericAssistant` uses, so
the RCA pipeline runs unchanged against a remote engine server.
"""
from __future__ import annotations

import dataclasses
import threading
import time
from typing import Any, Dict, List, Optional

from .service import Assistant, AssistantService, Message, MessageList, Run, Text, TextContent, Thread


def _dump(obj) -> dict:
    return dataclasses.asdict(obj)


def _response_format_in(rf: Any):
    if rf is None or rf == "auto" or (isinstance(rf, dict) and rf.get("type") in (None, "text")):
        return None
    if isinstance(rf, dict) and rf.get("type") == "k8s_grammar":
        from ..engine.grammar import grammar_from_json
        return grammar_from_json(rf["grammar"])
    raise ValueError(f"unsupported response_format {rf!r}")


def _response_format_out(rf: Any):
    if rf is None:
        return None
    from ..engine.grammar import Grammar, grammar_to_json
    if isinstance(rf, Grammar):
        return {"type": "k8s_grammar", "grammar": grammar_to_json(rf)}
    return rf


def _cypher_value(v):
    """Neo4j HTTP "row" encoding: nodes and relationships as their property
    maps, paths as the alternating node/relationship list."""
    from ..graph.model import Entity, Path
    if isinstance(v, Path):
        out = []
        for i, n in enumerate(v.nodes):
            if i:
                out.append(dict(v.relationships[i - 1].items()))
            out.append(dict(n.items()))
        return out
    if isinstance(v, Entity):
        return dict(v.items())
    if isinstance(v, (list, tuple)):
        return [_cypher_value(x) for x in v]
    if isinstance(v, dict):
        return {k: _cypher_value(x) for k, x in v.items()}
    return v


def _cypher_meta(v):
    from ..graph.model import Node, Path, Relationship
    if isinstance(v, Node):
        return {"id": v.id, "elementId": v.element_id, "type": "node", "deleted": False}
    if isinstance(v, Relationship):
        return {"id": v.id, "elementId": v.element_id, "type": "relationship", "deleted": False}
    if isinstance(v, Path):
        return [_cypher_meta(x) for i, n in enumerate(v.nodes)
                for x in ((v.relationships[i - 1], n) if i else (n,))]
    return None


def cypher_commit(executors: Dict[str, Any], db: str, body: Dict[str, Any]) -> Dict[str, Any]:
    """One ``/db/{db}/tx/commit`` request: run each statement in order; the
    first failing statement ends the request with a Neo4j-coded error (the
    reference's retry loop keys on ``CypherSyntaxError``, ``test_all.py:109``)."""
    from ..graph.model import CypherSyntaxError
    ex = executors.get(db)
    if ex is None:
        return {"results": [], "errors": [{"code": "Neo.ClientError.Database.DatabaseNotFound",
                                            "message": f"database {db!r} not found"}]}
    results, errors = [], []
    for st in body.get("statements", []):
        try:
            recs = ex.run_query(st["statement"], st.get("parameters") or None)
        except CypherSyntaxError as e:
            errors.append({"code": "Neo.ClientError.Statement.SyntaxError", "message": str(e)})
            break
        except Exception as e:  # noqa: BLE001 - surfaced to the client, as Neo4j does
            errors.append({"code": "Neo.DatabaseError.Statement.ExecutionFailed", "message": str(e)})
            break
        cols = recs[0].keys() if recs else []
        results.append({"columns": cols,
                        "data": [{"row": [_cypher_value(v) for v in r.values()],
                                  "meta": [_cypher_meta(v) for v in r.values()]} for r in recs]})
    return {"results": results, "errors": errors}


def create_app(service: AssistantService, engine=None, graphs: Optional[Dict[str, Any]] = None):
    """FastAPI app serving ``service`` (``engine``: optional LLMEngine for /metrics;
    ``graphs``: database name -> PropertyGraph / graph URI for the Cypher endpoint)."""
    from fastapi import Body, FastAPI, HTTPException, Query
    from fastapi.responses import PlainTextResponse

    app = FastAPI(title="k8s-llm-rca-amd assistants API")

    def nf(e: Exception):
        raise HTTPException(status_code=404, detail=str(e))

    @app.get("/health")
    def health():
        return {"status": "ok", "engine_error": repr(engine.error) if engine is not None and engine.error else None}

    @app.post("/v1/assistants")
    def create_assistant(body: Dict[str, Any] = Body(...)):
        a = service.create_assistant(body.get("instructions", ""), body.get("name", ""), body.get("model", ""))
        return _dump(a)

    @app.get("/v1/assistants/{aid}")
    def get_assistant(aid: str):
        try:
            return _dump(service.retrieve_assistant(aid))
        except KeyError as e:
            nf(e)

    @app.post("/v1/threads")
    def create_thread(body: Optional[Dict[str, Any]] = Body(None)):
        return _dump(service.create_thread())

    @app.get("/v1/threads/{tid}")
    def get_thread(tid: str):
        try:
            return _dump(service.retrieve_thread(tid))
        except KeyError as e:
            nf(e)

    @app.delete("/v1/threads/{tid}")
    def delete_thread(tid: str):
        try:
            service.delete_thread(tid)
        except KeyError as e:
            nf(e)
        return {"id": tid, "object": "thread.deleted", "deleted": True}

    @app.post("/v1/threads/{tid}/messages")
    def add_message(tid: str, body: Dict[str, Any] = Body(...)):
        try:
            m = service.add_message(tid, body["content"], role=body.get("role", "user"))
        except KeyError as e:
            nf(e)
        except RuntimeError as e:
            raise HTTPException(status_code=409, detail=str(e))
        return _dump(m)

    @app.get("/v1/threads/{tid}/messages")
    def list_messages(tid: str, limit: int = Query(20), order: str = Query("desc")):
        try:
            ml = service.list_messages(tid, limit=limit, order=order)
        except KeyError as e:
            nf(e)
        return {"object": "list", "data": [_dump(m) for m in ml.data], "has_more": ml.has_more}

    @app.post("/v1/threads/{tid}/runs")
    def create_run(tid: str, body: Dict[str, Any] = Body(...)):
        try:
            rf = _response_format_in(body.get("response_format"))
        except (ValueError, KeyError, TypeError) as e:
            raise HTTPException(status_code=400, detail=str(e))
        sampling = {k: body[k] for k in ("temperature", "seed") if body.get(k) is not None}
        try:
            r = service.create_run(tid, body["assistant_id"], instructions=body.get("instructions"),
                                   response_format=rf, max_tokens=body.get("max_completion_tokens"),
                                   sampling=sampling or None)
        except KeyError as e:
            nf(e)
        except RuntimeError as e:
            raise HTTPException(status_code=409, detail=str(e))
        return _dump(r)

    @app.get("/v1/threads/{tid}/runs")
    def list_runs(tid: str, limit: int = Query(20), order: str = Query("desc")):
        return {"object": "list", "data": [_dump(r) for r in service.list_runs(tid, limit=limit, order=order)]}

    @app.get("/v1/threads/{tid}/runs/{rid}")
    def get_run(tid: str, rid: str, wait: float = Query(0.0)):
        try:
            r = service.retrieve_run(tid, rid)
            if wait > 0 and r.status in ("queued", "in_progress"):
                rs = service.runs[rid]
                rs.done.wait(min(wait, 600.0))
                r = rs.run
        except KeyError as e:
            nf(e)
        return _dump(r)

    @app.post("/v1/threads/{tid}/runs/{rid}/cancel")
    def cancel_run(tid: str, rid: str):
        try:
            service.retrieve_run(tid, rid)
            service.cancel_run(rid)
            return _dump(service.retrieve_run(tid, rid))
        except KeyError as e:
            nf(e)

    executors: Dict[str, Any] = {}
    if graphs:
        from .graph import GraphQueryExecutor
        executors = {name: GraphQueryExecutor(g) for name, g in graphs.items()}

    @app.post("/db/{db}/tx/commit")
    def tx_commit(db: str, body: Dict[str, Any] = Body(...)):
        return cypher_commit(executors, db, body)

    @app.get("/metrics")
    def metrics():
        return PlainTextResponse(prometheus_text(service, engine), media_type="text/plain; version=0.0.4")

    return app


def prometheus_text(service: AssistantService, engine=None) -> str:
    """Prometheus exposition of run states and engine counters."""
    from prometheus_client import CollectorRegistry, generate_latest
    from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

    class _Collector:
        def collect(self):
            runs = GaugeMetricFamily("k8srca_runs", "runs by status", labels=["status"])
            counts: Dict[str, int] = {}
            for rs in list(service.runs.values()):
                counts[rs.run.status] = counts.get(rs.run.status, 0) + 1
            for k, v in sorted(counts.items()):
                runs.add_metric([k], v)
            yield runs
            yield GaugeMetricFamily("k8srca_threads", "live threads", value=len(service.threads))
            if engine is not None:
                for k, v in sorted(engine.stats.items()):
                    if isinstance(v, (int, float)):
                        yield CounterMetricFamily(f"k8srca_engine_{k}", f"engine counter {k}", value=float(v))
                yield GaugeMetricFamily("k8srca_kv_free_blocks", "free KV blocks", value=engine.kv.free_blocks)
                host = getattr(engine, "kv_host", None)
                if host is not None:  # the KV host tier (engine/kv_offload.py)
                    yield GaugeMetricFamily("k8srca_kv_host_free_blocks", "free KV host-tier blocks",
                                            value=host.free_slots)
                    yield GaugeMetricFamily("k8srca_kv_host_pending_blocks",
                                            "HBM pages whose swap-out copy is still in flight",
                                            value=host.pending_blocks)

    reg = CollectorRegistry()
    reg.register(_Collector())
    return generate_latest(reg).decode()


# ---------------------------------------------------------------- client
class RemoteAssistantService:
    """``AssistantService``-compatible client of :func:`create_app` (what
    GenericAssistant needs), over any httpx-compatible client or a base URL."""

    def __init__(self, base_url_or_client: Any, timeout: float = 600.0):
        if isinstance(base_url_or_client, str):
            import httpx
            self.http = httpx.Client(base_url=base_url_or_client.rstrip("/"), timeout=timeout)
        else:
            self.http = base_url_or_client
        self._run_thread: Dict[str, str] = {}
        self._lock = threading.Lock()

    def _ok(self, r):
        if r.status_code == 404:
            raise KeyError(r.json().get("detail"))
        if r.status_code == 409:
            raise RuntimeError(r.json().get("detail"))
        r.raise_for_status()
        return r.json()

    @staticmethod
    def _run(d: dict) -> Run:
        return Run(**{k: d.get(k) for k in (f.name for f in dataclasses.fields(Run))})

    @staticmethod
    def _msg(d: dict) -> Message:
        content = [TextContent(Text(c["text"]["value"], c["text"].get("annotations", [])), c.get("type", "text"))
                   for c in d["content"]]
        return Message(d["id"], d["thread_id"], d["role"], content, d["created_at"], d.get("assistant_id"),
                       d.get("run_id"))

    def create_assistant(self, instructions: str, name: str, model: str) -> Assistant:
        d = self._ok(self.http.post("/v1/assistants", json={"instructions": instructions, "name": name,
                                                             "model": model}))
        return Assistant(**{k: d[k] for k in ("id", "name", "instructions", "model", "created_at")})

    def retrieve_assistant(self, assistant_id: str) -> Assistant:
        d = self._ok(self.http.get(f"/v1/assistants/{assistant_id}"))
        return Assistant(**{k: d[k] for k in ("id", "name", "instructions", "model", "created_at")})

    def create_thread(self) -> Thread:
        d = self._ok(self.http.post("/v1/threads", json={}))
        return Thread(d["id"], d["created_at"])

    def retrieve_thread(self, thread_id: str) -> Thread:
        d = self._ok(self.http.get(f"/v1/threads/{thread_id}"))
        return Thread(d["id"], d["created_at"])

    def delete_thread(self, thread_id: str) -> None:
        self._ok(self.http.delete(f"/v1/threads/{thread_id}"))

    def add_message(self, thread_id: str, content: str, role: str = "user") -> Message:
        return self._msg(self._ok(self.http.post(f"/v1/threads/{thread_id}/messages",
                                                 json={"role": role, "content": content})))

    def list_messages(self, thread_id: str, limit: int = 20, order: str = "desc") -> MessageList:
        d = self._ok(self.http.get(f"/v1/threads/{thread_id}/messages", params={"limit": limit, "order": order}))
        return MessageList([self._msg(m) for m in d["data"]], d.get("has_more", False))

    def create_run(self, thread_id: str, assistant_id: str, instructions: Optional[str] = None,
                   response_format: Any = None, max_tokens: Optional[int] = None,
                   sampling: Optional[dict] = None) -> Run:
        body = {"assistant_id": assistant_id, "instructions": instructions,
                "response_format": _response_format_out(response_format), "max_completion_tokens": max_tokens}
        body.update(sampling or {})
        r = self._run(self._ok(self.http.post(f"/v1/threads/{thread_id}/runs", json=body)))
        with self._lock:
            self._run_thread[r.id] = thread_id
        return r

    def retrieve_run(self, thread_id: str, run_id: str) -> Run:
        return self._run(self._ok(self.http.get(f"/v1/threads/{thread_id}/runs/{run_id}")))

    def list_runs(self, thread_id: str, limit: int = 20, order: str = "desc") -> List[Run]:
        d = self._ok(self.http.get(f"/v1/threads/{thread_id}/runs", params={"limit": limit, "order": order}))
        return [self._run(x) for x in d["data"]]

    def wait_run(self, run_id: str, timeout: Optional[float] = None) -> Run:
        tid = self._run_thread[run_id]
        deadline = time.time() + (timeout if timeout is not None else 3600.0)
        while True:
            left = max(0.0, deadline - time.time())
            r = self._run(self._ok(self.http.get(f"/v1/threads/{tid}/runs/{run_id}",
                                                 params={"wait": min(left, 60.0)})))
            if r.status not in ("queued", "in_progress"):
                return r
            if left <= 0:
                self.cancel_run(run_id, status="expired")
                return self.retrieve_run(tid, run_id)

    def cancel_run(self, run_id: str, status: str = "cancelled") -> None:
        tid = self._run_thread[run_id]
        self._ok(self.http.post(f"/v1/threads/{tid}/runs/{run_id}/cancel"))
