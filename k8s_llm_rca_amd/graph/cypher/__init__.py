"""Cypher-subset engine: parser, evaluator and columnar executor (G8)."""
from .executor import Executor
from .parser import parse

__all__ = ["Executor", "parse"]
