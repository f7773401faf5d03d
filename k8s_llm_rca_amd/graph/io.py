"""Graph persistence: JSON-lines import / export of a :class:`PropertyGraph`.

Format (one JSON object per line)::

    {"t": "node", "id": 17, "label": "Pod", "props": {...}}
    {"t": "edge", "src": 17, "dst": 42, "type": "ReferInternal", "props": {"key": ...}}

This is how a cluster snapshot exported from another system (e.g. the
reference's Neo4j metagraph / stategraph via APOC ``export.json``, mapped to
this shape) is brought in, and how synthetic clusters are checkpointed.
Incidents are written next to the graph as a CSV whose first column is the
error message (the reference's input format, ``test_with_file.py:42-53``).
"""
from __future__ import annotations

import csv
import gzip
import json
from typing import Iterable, List, Optional

from .store import PropertyGraph


def _open(path: str, mode: str):
    return gzip.open(path, mode + "t") if path.endswith(".gz") else open(path, mode)


def save_graph(g: PropertyGraph, path: str) -> None:
    with _open(path, "w") as f:
        f.write(json.dumps({"t": "graph", "name": g.name}) + "\n")
        for i in range(g.num_nodes):
            labels = g.node_labels(i)
            rec = {"t": "node", "id": i, "label": labels[0], "props": g.node_props(i)}
            if len(labels) > 1:
                rec["extra_labels"] = labels[1:]
            f.write(json.dumps(rec) + "\n")
        for e in range(g.num_edges):
            f.write(json.dumps({"t": "edge", "src": g.edge_src(e), "dst": g.edge_dst(e), "type": g.edge_type_name(e),
                                "props": g.edge_props(e)}) + "\n")


def load_graph(path: str, name: Optional[str] = None) -> PropertyGraph:
    g = PropertyGraph(name or "graph")
    remap = {}
    with _open(path, "r") as f:
        for line in f:
            if not line.strip():
                continue
            r = json.loads(line)
            t = r.get("t")
            if t == "graph":
                g.name = name or r.get("name", g.name)
            elif t == "node":
                remap[r["id"]] = g.add_node(r["label"], r.get("props") or {}, r.get("extra_labels", ()))
            elif t == "edge":
                g.add_edge(remap[r["src"]], remap[r["dst"]], r["type"], r.get("props") or {})
    return g.finalize()


def save_incidents_csv(incidents: Iterable, path: str) -> None:
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["message", "fault", "timestamp", "src_kind", "dest_kind", "path_kinds", "involved_id",
                    "root_id"])
        for i in incidents:
            w.writerow([i.message, i.fault, i.timestamp, i.src_kind, i.dest_kind, "|".join(i.path_kinds),
                        i.involved_id, i.root_id])


def load_incidents_csv(path: str) -> List:
    from .synth import Incident
    out = []
    with open(path, newline="") as f:
        r = csv.reader(f)
        header = next(r, None)
        for row in r:
            if not row:
                continue
            if header and len(row) >= 8:
                out.append(Incident(row[1], row[0], row[2], row[3], row[4], row[5].split("|"), row[6], row[7]))
            else:
                out.append(Incident("unknown", row[0], "", "", "", [], "", ""))
    return out
