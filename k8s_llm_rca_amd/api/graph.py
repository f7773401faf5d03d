"""``GraphQueryExecutor``: the in-process replacement for ``Neo4jQueryExecutor``.

Same surface as ``common/neo4j_query_executor.py:6-24`` -- ``__init__(uri,
user, password)``, ``run_query(query, parameters=None) -> list[Record]`` and
``close()`` -- but the graph lives in this process (host CSR + optional HBM
mirror) instead of behind a Bolt connection.

``uri`` may be a :class:`PropertyGraph`, a ``mem://<name>`` URI registered
with :func:`register_graph` (so driver code keeps the reference's
"two executors, two URIs" shape: metagraph + stategraph), or a graph file
written by ``gen-graph`` / :func:`..graph.io.save_graph` (``file:///x.jsonl``
or a plain path; loaded once per process and cached under its path).
"""
from __future__ import annotations

import os
import threading
import time
from typing import Any, Dict, List, Optional, Union

from ..graph.cypher import Executor
from ..graph.model import CypherError, CypherSyntaxError, Record
from ..graph.store import PropertyGraph
from ..utils import tracing

_REGISTRY: Dict[str, PropertyGraph] = {}
_LOCK = threading.Lock()


def register_graph(name: str, graph: PropertyGraph) -> str:
    with _LOCK:
        _REGISTRY[name] = graph
    return f"mem://{name}"


def resolve_graph(uri: Union[str, PropertyGraph]) -> PropertyGraph:
    if isinstance(uri, PropertyGraph):
        return uri
    scheme, _, rest = uri.rpartition("://")
    name = rest if scheme else uri
    with _LOCK:
        g = _REGISTRY.get(name)
    if g is None and scheme in ("", "file") and os.path.isfile(name):
        from ..graph.io import load_graph
        g = load_graph(name, os.path.splitext(os.path.basename(name))[0])
        with _LOCK:
            g = _REGISTRY.setdefault(name, g)
    if g is None:
        raise ConnectionError(f"no in-process graph registered as {uri!r}")
    return g


class GraphQueryExecutor:
    def __init__(self, uri: Union[str, PropertyGraph], user: Optional[str] = None,
                 password: Optional[str] = None):
        self.graph = resolve_graph(uri)
        self._exec = Executor(self.graph)
        self.queries_run = 0
        self.query_seconds = 0.0
        self._closed = False

    def verify_connectivity(self) -> None:
        if self._closed:
            raise ConnectionError("executor closed")

    def close(self) -> None:
        self._closed = True

    def run_query(self, query: str, parameters: Optional[Dict[str, Any]] = None) -> List[Record]:
        if self._closed:
            raise ConnectionError("executor closed")
        t0 = time.perf_counter()
        with tracing.span("graph.query"):
            try:
                return self._exec.run(query, parameters)
            finally:
                dt = time.perf_counter() - t0
                self.queries_run += 1
                self.query_seconds += dt


# name used by the reference (common/neo4j_query_executor.py:6)
Neo4jQueryExecutor = GraphQueryExecutor

__all__ = ["GraphQueryExecutor", "Neo4jQueryExecutor", "register_graph", "resolve_graph",
           "CypherSyntaxError", "CypherError"]
