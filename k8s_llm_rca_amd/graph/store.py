"""Columnar property-graph store (G1 in SURVEY.md §2 Part B).

Replaces the two Neo4j servers the reference talks to over Bolt
(``common/neo4j_query_executor.py:6-24``).  Layout:

* nodes: one primary label id per node (``int32``) + a property dict per node;
* edges: ``src/dst`` (``int64``), type id (``int32``), interned ``key`` id
  (``int32``, -1 when absent) and ``tmin/tmax`` as int64 milliseconds for
  ``HasState`` edges (lexicographic order of the reference's fixed-width
  timestamps == numeric order, ``check_state/analyze_root_cause.py:56,75``);
* CSR out- and in-adjacency (``indptr``/``nbr``/``eid``) built once by
  :meth:`PropertyGraph.finalize` (native C++ when ``_graphcore`` is built);
* a packed UTF-8 heap (``offsets``/``bytes``) for string columns that are
  scanned with ``CONTAINS`` (the EVENT ``message``), mirrored to HBM by
  :mod:`k8s_llm_rca_amd.graph.device` for the HIP substring kernel.

The Cypher executor (:mod:`k8s_llm_rca_amd.graph.cypher`) only uses the
operator API at the bottom of this file, so the storage can move between host
and device without touching the planner.
"""
from __future__ import annotations

import datetime as _dt
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import native as _native

TS_FORMAT = "%Y-%m-%d %H:%M:%S.%f"


def ts_to_ms(ts: Optional[str]) -> int:
    """'2020-12-13 15:30:02.013' -> int64 ms since epoch (UTC); None -> INT64 max."""
    if ts is None:
        return np.iinfo(np.int64).max
    d = _dt.datetime.strptime(ts, TS_FORMAT).replace(tzinfo=_dt.timezone.utc)
    return int(d.timestamp() * 1000.0 + 0.5)


def ms_to_ts(ms: int) -> str:
    d = _dt.datetime.fromtimestamp(ms / 1000.0, tz=_dt.timezone.utc)
    return d.strftime(TS_FORMAT)[:-3]


class _Interner:
    __slots__ = ("ids", "names")

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.names: List[str] = []

    def get(self, name: str) -> int:
        i = self.ids.get(name)
        if i is None:
            i = len(self.names)
            self.ids[name] = i
            self.names.append(name)
        return i

    def lookup(self, name: str) -> int:
        return self.ids.get(name, -1)


class PropertyGraph:
    """Append-then-finalize property graph with CSR adjacency."""

    def __init__(self, name: str = "graph"):
        self.name = name
        self.labels = _Interner()
        self.rel_types = _Interner()
        self.keys = _Interner()  # interned values of the edge 'key' property
        self._node_label: List[int] = []
        self._node_props: List[Dict[str, Any]] = []
        self._extra_labels: Dict[int, List[int]] = {}
        self._e_src: List[int] = []
        self._e_dst: List[int] = []
        self._e_type: List[int] = []
        self._e_props: List[Dict[str, Any]] = []
        self.finalized = False
        self._prop_index: Dict[Tuple[int, str], Dict[Any, np.ndarray]] = {}
        self._col_cache: Dict[Tuple[str, str], np.ndarray] = {}
        self._heaps: Dict[str, Tuple[np.ndarray, np.ndarray]] = {}
        self.device = None  # set by graph.device.to_device()

    # ------------------------------------------------------------------ build
    def add_node(self, label: str, props: Optional[Dict[str, Any]] = None,
                 extra_labels: Sequence[str] = ()) -> int:
        assert not self.finalized, "graph already finalized"
        nid = len(self._node_label)
        self._node_label.append(self.labels.get(label))
        self._node_props.append(dict(props or {}))
        if extra_labels:
            self._extra_labels[nid] = [self.labels.get(x) for x in extra_labels]
        return nid

    def add_edge(self, src: int, dst: int, rel_type: str,
                 props: Optional[Dict[str, Any]] = None) -> int:
        assert not self.finalized, "graph already finalized"
        eid = len(self._e_src)
        self._e_src.append(int(src))
        self._e_dst.append(int(dst))
        self._e_type.append(self.rel_types.get(rel_type))
        self._e_props.append(dict(props or {}))
        return eid

    def finalize(self) -> "PropertyGraph":
        n = len(self._node_label)
        self.node_label = np.asarray(self._node_label, dtype=np.int32)
        self.e_src = np.asarray(self._e_src, dtype=np.int64)
        self.e_dst = np.asarray(self._e_dst, dtype=np.int64)
        self.e_type = np.asarray(self._e_type, dtype=np.int32)
        ek = np.full(len(self._e_props), -1, dtype=np.int32)
        tmin = np.full(len(self._e_props), np.iinfo(np.int64).min, dtype=np.int64)
        tmax = np.full(len(self._e_props), np.iinfo(np.int64).max, dtype=np.int64)
        for i, p in enumerate(self._e_props):
            k = p.get("key")
            if isinstance(k, str):
                ek[i] = self.keys.get(k)
            if "tmin" in p:
                tmin[i] = ts_to_ms(p["tmin"])
            if "tmax" in p:
                tmax[i] = ts_to_ms(p["tmax"])
        self.e_key = ek
        self.e_tmin = tmin
        self.e_tmax = tmax
        # CSR (out: grouped by src; in: grouped by dst)
        self.out_indptr, self.out_nbr, self.out_eid = _native.build_csr(n, self.e_src, self.e_dst)
        self.in_indptr, self.in_nbr, self.in_eid = _native.build_csr(n, self.e_dst, self.e_src)
        # label -> sorted node ids
        order = np.argsort(self.node_label, kind="stable")
        counts = np.bincount(self.node_label, minlength=len(self.labels.names))
        self.label_indptr = np.zeros(len(self.labels.names) + 1, dtype=np.int64)
        np.cumsum(counts, out=self.label_indptr[1:])
        self.label_nodes = order.astype(np.int64)
        self.finalized = True
        return self

    # ---------------------------------------------------------------- access
    @property
    def num_nodes(self) -> int:
        return len(self._node_label)

    @property
    def num_edges(self) -> int:
        return len(self._e_src)

    def node_props(self, nid: int) -> Dict[str, Any]:
        return self._node_props[nid]

    def node_labels(self, nid: int) -> List[str]:
        out = [self.labels.names[self._node_label[nid]]]
        for x in self._extra_labels.get(nid, ()):
            out.append(self.labels.names[x])
        return out

    def edge_props(self, eid: int) -> Dict[str, Any]:
        return self._e_props[eid]

    def edge_type_name(self, eid: int) -> str:
        return self.rel_types.names[self._e_type[eid]]

    def edge_src(self, eid: int) -> int:
        return self._e_src[eid]

    def edge_dst(self, eid: int) -> int:
        return self._e_dst[eid]

    # ------------------------------------------------------------- operators
    def all_nodes(self) -> np.ndarray:
        return np.arange(self.num_nodes, dtype=np.int64)

    def label_scan(self, label: str) -> np.ndarray:
        lid = self.labels.lookup(label)
        if lid < 0:
            return np.zeros(0, dtype=np.int64)
        ids =self.label_nodes[self.label_indptr[lid]:self.label_indptr[lid + 1]]
        if self._extra_labels:
            more = [n for n, ls in self._extra_labels.items() if lid in ls]
            if more:
                ids = np.union1d(ids, np.asarray(more, dtype=np.int64))
        return ids

    def has_label(self, ids: np.ndarray, label: str) -> np.ndarray:
        lid = self.labels.lookup(label)
        if lid < 0:
            return np.zeros(len(ids), dtype=bool)
        m = self.node_label[ids] == lid
        if self._extra_labels:
            for j, n in enumerate(ids.tolist()):
                if not m[j] and lid in self._extra_labels.get(n, ()):
                    m[j] = True
        return m

    def node_column(self, key: str) -> np.ndarray:
        """Object array of a node property over all nodes (None when missing)."""
        c = self._col_cache.get(("n", key))
        if c is None:
            c = np.empty(self.num_nodes, dtype=object)
            c[:] = [p.get(key) for p in self._node_props]
            self._col_cache[("n", key)] = c
        return c

    def edge_column(self, key: str) -> np.ndarray:
        c = self._col_cache.get(("e", key))
        if c is None:
            c = np.empty(self.num_edges, dtype=object)
            c[:] = [p.get(key) for p in self._e_props]
            self._col_cache[("e", key)] = c
        return c

    def index_lookup(self, label: Optional[str], key: str, value: Any) -> np.ndarray:
        """Hash-index equality lookup (G7): nodes with ``label`` and ``key == value``."""
        lid = -1 if label is None else self.labels.lookup(label)
        if label is not None and lid < 0:
            return np.zeros(0, dtype=np.int64)
        idx = self._prop_index.get((lid, key))
        if idx is None:
            ids = self.label_scan(label) if label is not None else self.all_nodes()
            col = self.node_column(key)[ids]
            tmp: Dict[Any, List[int]] = {}
            for n, v in zip(ids.tolist(), col.tolist()):
                if v is not None:
                    try:
                        tmp.setdefault(v, []).append(n)
                    except TypeError:  # unhashable property value
                        pass
            idx = {k: np.asarray(v, dtype=np.int64) for k, v in tmp.items()}
            self._prop_index[(lid, key)] = idx
        try:
            return idx.get(value, np.zeros(0, dtype=np.int64))
        except TypeError:
            return np.zeros(0, dtype=np.int64)

    def string_heap(self, key: str) -> Tuple[np.ndarray, np.ndarray]:
        """Packed UTF-8 heap of a node string property: (offsets[N+1] int64, bytes uint8).

        Missing / non-string values are empty strings (they never match CONTAINS).
        """
        h = self._heaps.get(key)
        if h is None:
            parts = []
            offs = np.zeros(self.num_nodes + 1, dtype=np.int64)
            pos = 0
            for i, p in enumerate(self._node_props):
                v = p.get(key)
                b = v.encode("utf-8") if isinstance(v, str) else b""
                parts.append(b)
                pos += len(b)
                offs[i + 1] = pos
            buf = np.frombuffer(b"".join(parts), dtype=np.uint8).copy() if pos else np.zeros(0, np.uint8)
            h = (offs, buf)
            self._heaps[key] = h
        return h

    def contains_scan(self, ids: np.ndarray, key: str, needle: str) -> np.ndarray:
        """Boolean mask: ``node[key] CONTAINS needle`` for each id (G3).

        Dispatches to the HIP kernel when the graph is mirrored to a GPU, to the
        native C++ scanner otherwise.
        """
        if len(ids) == 0:
            return np.zeros(0, dtype=bool)
        if self.device is not None and self.device.batcher is not None:  # coalesced with the other pipelines'
            return self.device.batcher.contains(np.asarray(ids), key, needle)
        if self.device is not None and len(ids) >= self.device.min_gpu_rows:
            return self.device.contains(ids, key, needle)
        offs, buf = self.string_heap(key)
        return _native.substr_mask(offs, buf, ids, needle.encode("utf-8"))

    def expand(self, ids: np.ndarray, direction: str, rel_types: Optional[Sequence[str]] = None,
               key: Optional[str] = None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """One hop from each id.  Returns (row, edge_id, neighbour) arrays (G5).

        ``direction`` is 'out', 'in' or 'both'.  ``rel_types`` / ``key`` filter
        edges by type / interned key equality.
        """
        if self.device is not None and len(ids) >= self.device.min_gpu_rows:
            return self.device.expand(np.asarray(ids), direction, rel_types, key)
        tids = None
        if rel_types:
            tids = np.asarray([self.rel_types.lookup(t) for t in rel_types], dtype=np.int32)
            tids = tids[tids >= 0]
            if len(tids) == 0:
                z = np.zeros(0, dtype=np.int64)
                return z, z, z
        kid = -2
        if key is not None:
            kid = self.keys.lookup(key)
            if kid < 0:
                z = np.zeros(0, dtype=np.int64)
                return z, z, z
        outs = []
        if direction in ("out", "both"):
            outs.append(_native.expand(self.out_indptr, self.out_nbr, self.out_eid, ids,
                                       self.e_type, self.e_key, tids, kid))
        if direction in ("in", "both"):
            r = _native.expand(self.in_indptr, self.in_nbr, self.in_eid, ids,
                               self.e_type, self.e_key, tids, kid)
            if direction == "both":
                # an undirected self-loop would otherwise be reported twice
                keep = self.e_src[r[1]] != self.e_dst[r[1]]
                r = (r[0][keep], r[1][keep], r[2][keep])
            outs.append(r)
        if len(outs) == 1:
            return outs[0]
        row = np.concatenate([o[0] for o in outs])
        eid = np.concatenate([o[1] for o in outs])
        nbr = np.concatenate([o[2] for o in outs])
        order = np.argsort(row, kind="stable")
        return row[order], eid[order], nbr[order]

    def var_length(self, starts: np.ndarray, min_hops: int, max_hops: int, direction: str,
                   rel_types: Optional[Sequence[str]] = None,
                   end_label: Optional[str] = None) -> List[Tuple[int, List[int], List[int]]]:
        """Enumerate relationship-unique walks of ``min_hops..max_hops`` hops from each start.

        Returns a list of ``(start_row, node_ids, edge_ids)`` (Cypher
        var-length semantics: a relationship appears at most once per path).
        ``end_label`` keeps only walks ending on that label (planner pushdown).
        """
        dev = self.device
        if (dev is not None and (dev.batcher is not None or len(starts) >= dev.min_gpu_rows) and 1 <= min_hops
                and max_hops <= 3 and len(starts)):
            if dev.batcher is not None:
                rec = dev.batcher.walks(np.asarray(starts), min_hops, max_hops, direction, rel_types, end_label)
            else:
                rec = dev.walks(np.asarray(starts), min_hops, max_hops, direction, rel_types, end_label)
            out = []
            for r in rec.tolist():
                h = r[1]
                out.append((r[0], r[2:3 + h], r[6:6 + h]))
            return out
        tids = None
        if rel_types:
            tids = np.asarray([self.rel_types.lookup(t) for t in rel_types], dtype=np.int32)
        walks = _native.var_length(self, starts, min_hops, max_hops, direction, tids)
        if end_label is not None:
            lid = self.labels.lookup(end_label)
            walks = [w for w in walks if self.node_label[w[1][-1]] == lid]
        return walks

    def state_lookup(self, entity_ids: np.ndarray, ts_ms: np.ndarray, state_label: Optional[str] = None,
                     mode: str = "strict", tmax_ms: Optional[np.ndarray] = None,
                     limit: int = 10) -> List[np.ndarray]:
        """Temporal STATE lookup (G6): per entity, HasState edges valid at ``ts``.

        strict: ``tmin <= ts < tmax`` (``analyze_root_cause.py:70-79``);
        loose: ``tmin <= tmax_q and tmax > ts`` (interval overlap, ``:51-60``).
        Returns, per entity, the edge ids (first ``limit`` in CSR order).
        """
        if self.device is not None and self.device.batcher is not None and len(entity_ids):
            return self.device.batcher.state_lookup(entity_ids, ts_ms, state_label, mode, tmax_ms, limit)
        if self.device is not None and len(entity_ids) >= self.device.min_gpu_rows:
            return self.device.state_lookup(entity_ids, ts_ms, state_label, mode, tmax_ms, limit)
        tid = self.rel_types.lookup("HasState")
        lid = -1 if state_label is None else self.labels.lookup(state_label)
        out = []
        for j, n in enumerate(np.asarray(entity_ids).tolist()):
            a, b = self.out_indptr[n], self.out_indptr[n + 1]
            e = self.out_eid[a:b]
            m = self.e_type[e] == tid
            if lid >= 0:
                m &= self.node_label[self.e_dst[e]] == lid
            t = ts_ms[j]
            if mode == "strict":
                m &= (self.e_tmin[e] <= t) & (self.e_tmax[e] > t)
            else:
                m &= (self.e_tmin[e] <= tmax_ms[j]) & (self.e_tmax[e] > t)
            out.append(e[m][:limit])
        return out

    # ------------------------------------------------------------ statistics
    def stats(self) -> Dict[str, Any]:
        per_label = {self.labels.names[i]: int(self.label_indptr[i + 1] - self.label_indptr[i])
                     for i in range(len(self.labels.names))}
        per_type = {}
        if self.num_edges:
            cnt = np.bincount(self.e_type, minlength=len(self.rel_types.names))
            per_type = {self.rel_types.names[i]: int(c) for i, c in enumerate(cnt)}
        return {"nodes": self.num_nodes, "edges": self.num_edges, "labels": per_label, "rel_types": per_type}
