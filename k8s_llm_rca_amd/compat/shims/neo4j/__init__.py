"""``neo4j`` driver surface over the in-process graph engine.

Only what the reference touches (``common/neo4j_query_executor.py:3-24``,
``check_state/analyze_root_cause.py:85,97``, ``test_all.py:109``):
``GraphDatabase.driver(uri, auth) -> Driver`` with ``verify_connectivity`` /
``session()`` / ``close``; ``Session.run(query, parameters)`` iterating
``Record`` objects; ``neo4j.graph.Node/Relationship/Path`` and
``neo4j.exceptions.CypherSyntaxError`` as the very classes the engine returns
and raises, so ``isinstance`` checks and ``except`` clauses in unchanged
reference code match.

URIs resolve through :func:`k8s_llm_rca_amd.api.graph.resolve_graph`
(``mem://name`` registrations, graph files) plus :func:`map_uri`, which binds
a ``bolt://host:port`` the reference hard-codes (``test_all.py:21-22``) to a
registered graph or a graph file; ``K8SRCA_NEO4J_URIS="bolt://a=path,..."``
does the same from the environment.  Credentials are ignored.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

from k8s_llm_rca_amd.api.graph import GraphQueryExecutor

import sys
import types

from k8s_llm_rca_amd.graph import model as _model


def _submodule(name: str, doc: str, **attrs) -> types.ModuleType:
    """``neo4j.<name>`` holding the engine's own classes (registered in
    ``sys.modules`` so ``import neo4j.graph`` / ``from neo4j.exceptions import
    ...`` resolve to it)."""
    m = types.ModuleType(f"{__name__}.{name}", doc)
    for k, v in attrs.items():
        setattr(m, k, v)
    m.__all__ = list(attrs)
    sys.modules[m.__name__] = m
    return m


graph = _submodule("graph", "the engine's Node / Relationship / Path result types",
                   Node=_model.Node, Relationship=_model.Relationship, Path=_model.Path)
exceptions = _submodule("exceptions", "the engine's own Cypher error classes",
                        CypherSyntaxError=_model.CypherSyntaxError, CypherTypeError=_model.CypherTypeError,
                        CypherError=_model.CypherError, Neo4jError=_model.CypherError,
                        ClientError=_model.CypherError, ServiceUnavailable=ConnectionError)

__all__ = ["GraphDatabase", "Driver", "Session", "Result", "map_uri", "exceptions", "graph", "basic_auth"]

_URI_MAP: Dict[str, Any] = {}


def map_uri(uri: str, target: Any) -> None:
    """Serve ``uri`` (e.g. ``bolt://10.1.0.174:7687``) from ``target``: a
    PropertyGraph, a ``mem://`` name or a graph file path."""
    _URI_MAP[uri] = target


def _resolve(uri: str) -> Any:
    if uri in _URI_MAP:
        return _URI_MAP[uri]
    for item in filter(None, os.environ.get("K8SRCA_NEO4J_URIS", "").split(",")):
        k, _, v = item.partition("=")
        if k.strip() == uri:
            return v.strip()
    return uri


def basic_auth(user: str, password: str, realm: Optional[str] = None) -> tuple:
    return (user, password)


class Result:
    def __init__(self, records):
        self._records = list(records)

    def __iter__(self):
        return iter(self._records)

    def data(self):
        return [r.data() if hasattr(r, "data") else dict(r) for r in self._records]

    def single(self):
        return self._records[0] if self._records else None

    def consume(self):
        return None


class Session:
    def __init__(self, executor: GraphQueryExecutor):
        self._ex = executor

    def run(self, query: str, parameters: Optional[Dict[str, Any]] = None, **kw) -> Result:
        params = dict(parameters or {})
        params.update(kw)
        return Result(self._ex.run_query(query, params or None))

    def close(self) -> None:
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


class Driver:
    def __init__(self, uri: str, auth=None, **kw):
        self.uri = uri
        self._ex = GraphQueryExecutor(_resolve(uri))

    def verify_connectivity(self, **kw) -> None:
        self._ex.verify_connectivity()

    def session(self, **kw) -> Session:
        return Session(self._ex)

    def execute_query(self, query: str, parameters: Optional[Dict[str, Any]] = None, **kw):
        return self._ex.run_query(query, parameters), None, list()

    def close(self) -> None:
        self._ex.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


class GraphDatabase:
    @staticmethod
    def driver(uri: str, auth=None, **kw) -> Driver:
        return Driver(uri, auth, **kw)
