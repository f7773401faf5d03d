"""Stage 2 "generate query": metapath -> Cypher statepath query -> records.

Functional equivalent of ``generate_query/generate_query.py``:

* :func:`setup_cypher_generator` seeds the thread with the label message and
  generation-template-1 (``:18-43``)
* :func:`extend_metapath_construct_string` (``:46-57``) -- keeps the stored
  ``srcKind/destKind`` so the true edge direction survives undirected matches
* :func:`generate_cypher_query` / :func:`extract_cypher` (``:60-85``)
* :func:`run_and_filter_query` / :func:`message_compatible` (``:88-129``)
* :func:`human_generate_cypher_query` -- deterministic fallback (``:214-266``),
  same output text
"""
from __future__ import annotations

import logging
from typing import List

from ..api.assistant import GenericAssistant
from . import prompts

log = logging.getLogger(__name__)

build_generation_template = prompts.build_generation_template


def setup_cypher_generator(service=None, model: str = "llama3-8b") -> GenericAssistant:
    g = GenericAssistant(service)
    g.create_assistant(prompts.GENERATOR_INSTRUCTIONS, prompts.GENERATOR_NAME, model)
    g.create_thread()
    g.add_message(prompts.GENERATION_LABEL_MESSAGE)
    g.add_message(prompts.build_generation_template())
    return g


def extend_metapath_construct_string(partial_path) -> str:
    src_kind = partial_path.nodes[0]["kind"]
    out = ("\n    HasEvent, Event, EVENT, metadata_uid;\n"
           f"    ReferInternal, Event, {src_kind}, involvedObject_uid;\n    ")
    for rel in partial_path.relationships:
        out += ", ".join([rel.type, rel["srcKind"], rel["destKind"], rel["key"]]) + ";\n"
    return out


def generate_cypher_query(metapath_str: str, error_message: str, cypherQueryGenerator: GenericAssistant,
                          response_format=None) -> str:
    cypherQueryGenerator.add_message(prompts.cypher_prompt(metapath_str, error_message))
    cypherQueryGenerator.run_assistant(response_format=response_format)
    messages = cypherQueryGenerator.wait_get_last_k_message(1)
    if messages is None:
        raise RuntimeError(f"cypher run {cypherQueryGenerator.run.id} did not complete")
    q = extract_cypher(messages.data[0].content[0].text.value)
    log.info("generated cypher query:\n%s", q)
    return q


def extract_cypher(message_str: str) -> str:
    return message_str.split("```cypher")[1].split("```")[0].strip()


def run_and_filter_query(query_executor, cypher_query: str) -> list:
    records = query_executor.run_query(cypher_query)
    res = [r for r in records if message_compatible(r)]
    if not res:
        log.warning("ALL records are not message compatible")
    return res


def _name_key(dest):
    if dest["isNative"] == "true":
        return "name2"
    if dest["isAtomic"] == "true":
        return "val"
    if dest["tag"] in ("nfs", "hostPath"):
        return "path"
    if dest["tag"] == "container":
        return "containerName"
    if dest["tag"] == "image":
        return "imageName"
    return None


def message_compatible(record) -> bool:
    """Keep a statepath whose destination's name or kind appears in the EVENT message."""
    message = None
    for ele in record:
        if ele["kind"] == "Event":
            message = ele["message"]
    if message is None:
        raise ValueError("statepath has no EVENT node (kind == 'Event') to take the message from")
    dest = record[len(record) - 1]
    k1 = _name_key(dest)
    if k1 is None:
        raise ValueError("cannot determine the name property of the statepath's destination")
    k2 = "kind2" if dest["isNative"] == "true" else ("tag" if dest["isNative"] == "false" else None)
    if k2 is None:
        raise ValueError("cannot determine the kind property of the statepath's destination")
    name, kind = dest[k1], dest[k2]
    return (isinstance(name, str) and name in message) or (isinstance(kind, str) and kind in message)


def human_generate_cypher_query(metapath_str: str, error_message: str) -> str:
    """Template query: one ``MATCH (a:K)-[rI:T]->(b:K) WHERE rI.key = 'v'`` per segment."""
    segments: List[List[str]] = [seg.strip().split(", ") for seg in metapath_str.split(";")[:-1]]
    alias = {"EVENT": "evt"}
    for seg in segments:
        for k in (seg[1], seg[2]):
            if k not in alias:
                alias[k] = f"n{len(alias)}"
    parts = [f"\nMATCH (evt:EVENT)\nWHERE evt.message CONTAINS {error_message!r}\nWITH evt\nLIMIT 1"]
    for i, (rel_type, src, dst, value) in enumerate(segments, start=1):
        parts.append(f"\nMATCH ({alias[src]}:{src})-[r{i}:{rel_type}]->({alias[dst]}:{dst})\nWHERE r{i}.key = {value!r}")
    nodes = list(alias.values())
    rels = [f"r{i}" for i in range(1, len(segments) + 1)]
    assert len(nodes) == len(rels) + 1, "metapath revisits a kind: no chain alias assignment"
    interleaved = [x for pair in zip(nodes, rels + [None]) for x in pair if x is not None]
    parts.append("\nRETURN " + ", ".join(interleaved))
    q = "\n".join(parts).strip()
    log.info("human generated cypher query:\n%s", q)
    return q
