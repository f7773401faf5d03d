"""``neo4j.exceptions``: the engine's own Cypher error classes."""
from k8s_llm_rca_amd.graph.model import CypherError, CypherSyntaxError, CypherTypeError

Neo4jError = CypherError
ClientError = CypherError
ServiceUnavailable = ConnectionError

__all__ = ["CypherSyntaxError", "CypherTypeError", "CypherError", "Neo4jError", "ClientError", "ServiceUnavailable"]
