"""Stage 1 "locate": source kind, LLM-chosen destination kind, metapath search.

Functional equivalent of ``find_metapath/find_srckind_metapath_neo4j.py``
(same function names and signatures; extra keyword arguments are optional):

* :func:`setup_root_cause_locator` -- assistant + thread (``:20-60``)
* :func:`find_native_external_kinds` -- sorted kind catalogue (``:63-72``)
* :func:`find_srcKind` -- EVENT ``CONTAINS`` -> Event -> involved object kind (``:75-90``)
* :func:`find_metapath` -- directed / undirected / single-hop / via-Namespace
  cascade, keeping every minimum-length path (``:93-160``)
* :func:`find_destKind_relevantResources` + :func:`extract_json` (``:178-196``)
* :func:`build_prompt_template` (``:200-240``, byte-identical text)
"""
from __future__ import annotations

import json
import logging
from typing import List, Optional, Sequence

from ..api.assistant import GenericAssistant
from . import prompts

log = logging.getLogger(__name__)

build_prompt_template = prompts.build_prompt_template

Q_KINDS = """
        MATCH (n1)
        WHERE n1.category IN ['NativeEntity', 'ExternalEntity']
        RETURN n1.category AS category, n1.kind AS kind
        """

Q_SRCKIND = """
        MATCH (n1:Event)-[s1:HasEvent]->(N1:EVENT)
        WHERE N1.message contains $message
        WITH n1, N1, s1
        MATCH (n1:Event)-[r1:ReferInternal]->(n2)
        WHERE r1.key = 'involvedObject_uid'
        RETURN distinct n2.kind2
        LIMIT 5;
        """

_PATH_FILTERS = """
        AND all(node in nodes(path) WHERE single(x in nodes(path) WHERE x = node))
        AND all(node in nodes(path) WHERE not node.kind in ['Event', 'Namespace'])
        AND ($intermediateKinds IS NULL
            OR size($intermediateKinds) = 0
            OR any(node in nodes(path)[1..-1] WHERE node.kind in $intermediateKinds))
        RETURN path
        """
Q_DIRECTED = "\n        MATCH path = (n1)-[*1..3]->(n2)\n        WHERE n1.kind = $srcKind and n2.kind = $destKind" + _PATH_FILTERS
Q_UNDIRECTED = "\n        MATCH path = (n1)-[*1..3]-(n2)\n        WHERE n1.kind = $srcKind and n2.kind = $destKind" + _PATH_FILTERS
Q_SINGLE = """
        MATCH path = (n1)-[r1]-(n2)
        WHERE n1.kind = $srcKind and n2.kind = $destKind
        RETURN path
        """
Q_NAMESPACE = """
        MATCH path = (n1)-[r1]-(n2)-[r2]-(n3)
        WHERE n1.kind = $srcKind and n2.kind = 'Namespace' and n3.kind = $destKind
        RETURN path
        """


def setup_root_cause_locator(service=None, model: str = "llama3-8b") -> GenericAssistant:
    a = GenericAssistant(service)
    a.create_assistant(prompts.LOCATOR_INSTRUCTIONS, prompts.LOCATOR_NAME, model)
    a.create_thread()
    log.info("locator assistant=%s thread=%s", a.assistant.id, a.thread.id)
    return a


def find_native_external_kinds(query_executor):
    records = query_executor.run_query(Q_KINDS)
    native = sorted(r["kind"] for r in records if r["category"] == "NativeEntity")
    external = sorted(r["kind"] for r in records if r["category"] == "ExternalEntity")
    return native, external


def find_srcKind(query_executor, message: str) -> str:
    records = query_executor.run_query(Q_SRCKIND, {"message": message})
    src = records[0]["n2.kind2"]  # IndexError when the message is unknown, as in the reference
    log.info("srcKind = %s", src)
    return src


def find_metapath(query_executor, srcKind: str, destKind: str, intermediateKinds: Optional[Sequence[str]] = None):
    inter = [x for x in (intermediateKinds or []) if x != "Namespace"]
    params = {"srcKind": srcKind, "destKind": destKind, "intermediateKinds": inter}
    records = []
    for q, what in ((Q_DIRECTED, "directed"), (Q_UNDIRECTED, "undirected"), (Q_SINGLE, "one-step"),
                    (Q_NAMESPACE, "src-Namespace-dest")):
        records = query_executor.run_query(q, params)
        if records:
            break
        log.info("no %s path %s -> %s", what, srcKind, destKind)
    min_len = min(len(r["path"]) for r in records)  # ValueError when the cascade is empty (reference semantics)
    metapaths = [r["path"] for r in records if len(r["path"]) == min_len]
    for mp in metapaths:
        print_metapath(mp)
    return metapaths


def print_metapath(path) -> None:
    lines = ["Nodes:"] + [str(n["kind"]) for n in path.nodes] + ["Relationships:"]
    lines += [f"{r.type} {r['srcKind']} {r['destKind']} {r['key']}" for r in path.relationships]
    lines.append("-" * 34)
    log.info("\n".join(lines))


def find_destKind_relevantResources(errorMessage: str, srcKind: str, promptTemplate: str,
                                    rootCauseLocator: GenericAssistant, response_format=None):
    prompt = promptTemplate.format(error_message=errorMessage, involved_object=srcKind)
    rootCauseLocator.add_message(prompt)
    rootCauseLocator.run_assistant(response_format=response_format)
    messages = rootCauseLocator.wait_get_last_k_message(1)
    if messages is None:
        raise RuntimeError(f"locator run {rootCauseLocator.run.id} did not complete")
    return extract_json(messages.data[0].content[0].text.value)


def extract_json(message_str: str):
    part = message_str.split("```json")[1].split("```")[0].strip()
    return json.loads(part)


def intermediate_kinds(relevant: List[str], src: str, dest: str, native: List[str], external: List[str]) -> List[str]:
    """RelevantResources minus src/dest, restricted to known kinds (test_with_file.py:103-106)."""
    return [x for x in relevant if x not in (src, dest) and (x in native or x in external)]
