"""Result objects returned by the in-process graph engine.

They honour the record contract the reference pipeline relies on when it talks
to Neo4j:

* ``record['n2.kind2']`` / ``record[0]`` / iteration / ``len(record)``
  (``find_metapath/find_srckind_metapath_neo4j.py:88``, ``generate_query/generate_query.py:106,110``)
* ``path.nodes`` / ``path.relationships`` / ``len(path)`` == number of hops
  (``find_srckind_metapath_neo4j.py:153,163-164``)
* ``rel.type`` and ``entity['prop']`` returning ``None`` for a missing key
  (``generate_query.py:55,107``)
* ``node.keys()`` (``check_state/analyze_root_cause.py:227``)

Entities are light views onto the columnar store: properties are materialised
lazily from the store on first access so a query that returns 10^5 rows does
not build 10^5 dicts up front.
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple


class CypherError(Exception):
    """Base class of query-engine errors (runtime, not syntax)."""


class CypherSyntaxError(CypherError):
    """Raised for queries outside the supported Cypher subset.

    Plays the role of ``neo4j.exceptions.CypherSyntaxError`` that the reference
    driver catches to feed the error text back to the query generator
    (``test_all.py:109-115``).
    """


class CypherTypeError(CypherError):
    pass


class Entity:
    __slots__ = ("_graph", "_id", "_props")

    def __init__(self, graph, eid: int, props: Optional[Dict[str, Any]] = None):
        self._graph = graph
        self._id = int(eid)
        self._props = props

    # -- property access (None when missing, like the neo4j driver's Entity) --
    def _p(self) -> Dict[str, Any]:
        if self._props is None:
            self._props = self._load_props()
        return self._props

    def _load_props(self) -> Dict[str, Any]:  # pragma: no cover - overridden
        return {}

    def __getitem__(self, key: str) -> Any:
        return self._p().get(key)

    def get(self, key: str, default: Any = None) -> Any:
        return self._p().get(key, default)

    def __contains__(self, key: str) -> bool:
        return key in self._p()

    def keys(self):
        return self._p().keys()

    def values(self):
        return self._p().values()

    def items(self):
        return self._p().items()

    def __iter__(self):
        return iter(self._p().items())

    def __len__(self) -> int:
        return len(self._p())

    @property
    def id(self) -> int:
        return self._id

    @property
    def element_id(self) -> str:
        return f"{type(self).__name__[0]}:{self._id}"

    def __eq__(self, other) -> bool:
        return type(self) is type(other) and self._id == other._id and self._graph is other._graph

    def __hash__(self) -> int:
        return hash((type(self).__name__, self._id))


class Node(Entity):
    __slots__ = ()

    def _load_props(self) -> Dict[str, Any]:
        return self._graph.node_props(self._id)

    @property
    def labels(self) -> frozenset:
        return frozenset(self._graph.node_labels(self._id))

    def __repr__(self) -> str:
        lab = ":".join(sorted(self.labels))
        return f"<Node element_id='{self.element_id}' labels={{{lab!r}}} properties={self._p()!r}>"


class Relationship(Entity):
    __slots__ = ()

    def _load_props(self) -> Dict[str, Any]:
        return self._graph.edge_props(self._id)

    @property
    def type(self) -> str:
        return self._graph.edge_type_name(self._id)

    @property
    def start_node(self) -> Node:
        return Node(self._graph, self._graph.edge_src(self._id))

    @property
    def end_node(self) -> Node:
        return Node(self._graph, self._graph.edge_dst(self._id))

    @property
    def nodes(self) -> Tuple[Node, Node]:
        return (self.start_node, self.end_node)

    def __repr__(self) -> str:
        return (f"<Relationship element_id='{self.element_id}' type={self.type!r} "
                f"properties={self._p()!r}>")


class Path:
    """A walk through the graph: ``len(path)`` counts relationships."""

    __slots__ = ("_nodes", "_rels")

    def __init__(self, nodes: Sequence[Node], rels: Sequence[Relationship]):
        if len(nodes) != len(rels) + 1:
            raise ValueError("a path has exactly one more node than relationships")
        self._nodes = tuple(nodes)
        self._rels = tuple(rels)

    @property
    def nodes(self) -> Tuple[Node, ...]:
        return self._nodes

    @property
    def relationships(self) -> Tuple[Relationship, ...]:
        return self._rels

    @property
    def start_node(self) -> Node:
        return self._nodes[0]

    @property
    def end_node(self) -> Node:
        return self._nodes[-1]

    def __len__(self) -> int:
        return len(self._rels)

    def __iter__(self) -> Iterator[Relationship]:
        return iter(self._rels)

    def __eq__(self, other) -> bool:
        return isinstance(other, Path) and self._nodes == other._nodes and self._rels == other._rels

    def __hash__(self) -> int:
        return hash((self._nodes, self._rels))

    def __repr__(self) -> str:
        return f"<Path start={self.start_node!r} end={self.end_node!r} size={len(self)}>"


class Record:
    """Ordered key/value row, indexable by key or by position."""

    __slots__ = ("_keys", "_values", "_index")

    def __init__(self, keys: Sequence[str], values: Sequence[Any]):
        self._keys = tuple(keys)
        self._values = tuple(values)
        self._index = None

    def __getitem__(self, key):
        if isinstance(key, (int, slice)):
            return self._values[key]
        if self._index is None:
            self._index = {k: i for i, k in enumerate(self._keys)}
        try:
            return self._values[self._index[key]]
        except KeyError:
            raise KeyError(key) from None

    def get(self, key: str, default: Any = None) -> Any:
        try:
            return self[key]
        except (KeyError, IndexError):
            return default

    def keys(self) -> List[str]:
        return list(self._keys)

    def values(self) -> List[Any]:
        return list(self._values)

    def items(self) -> List[Tuple[str, Any]]:
        return list(zip(self._keys, self._values))

    def data(self) -> Dict[str, Any]:
        return dict(zip(self._keys, self._values))

    def __iter__(self):
        return iter(self._values)

    def __len__(self) -> int:
        return len(self._values)

    def __eq__(self, other) -> bool:
        return isinstance(other, Record) and self._keys == other._keys and self._values == other._values

    def __repr__(self) -> str:
        inner = " ".join(f"{k}={v!r}" for k, v in zip(self._keys, self._values))
        return f"<Record {inner}>"
