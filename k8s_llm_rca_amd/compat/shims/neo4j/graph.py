"""``neo4j.graph``: the engine's Node / Relationship / Path result types."""
from k8s_llm_rca_amd.graph.model import Node, Path, Relationship

__all__ = ["Node", "Relationship", "Path"]
