"""``common/neo4j_query_executor.py`` path: :class:`Neo4jQueryExecutor`."""
from k8s_llm_rca_amd.api.graph import GraphQueryExecutor, register_graph


class Neo4jQueryExecutor(GraphQueryExecutor):
    """``Neo4jQueryExecutor(uri, user, password)`` over an in-process graph
    (``neo4j_query_executor.py:6-24``); ``uri`` is ``mem://name`` or a graph file."""


__all__ = ["Neo4jQueryExecutor", "register_graph"]
