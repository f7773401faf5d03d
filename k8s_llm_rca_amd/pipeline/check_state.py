"""Stage 3 "analyze root cause": temporal STATE checks + LLM semantic analysis.

Functional equivalent of ``check_state/analyze_root_cause.py``:

* :func:`setup_state_semantic_analyzer` -- assistant seeded with the state rule
  and the task prompt (``:6-46``)
* :func:`find_loose_states` / :func:`find_strict_states` -- Cypher builders for
  interval overlap and half-open ``tmin <= ts < tmax`` validity (``:51-79``)
* :func:`check_statepath` -- per-entity checks, then one summary run
  (``:82-150``); returns ``(raw_report_text, {"Kind(id)": [clues]})``
* :func:`check_states_of_entity` -- missing STATE => clue added to the thread
  *without* a run; otherwise one semantic run per STATE node (``:173-197``)
* :func:`ad_hoc_find_entity_name`, :func:`check_semantic`,
  :func:`check_states_existence_and_semantic` (``:155-250``)
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional, Tuple

from ..api.assistant import GenericAssistant
from ..graph.model import Node
from . import prompts

log = logging.getLogger(__name__)


def setup_state_semantic_analyzer(service=None, model: str = "llama3-8b") -> GenericAssistant:
    a = GenericAssistant(service)
    a.create_assistant(prompts.ANALYZER_INSTRUCTIONS, prompts.ANALYZER_NAME, model)
    a.create_thread()
    a.add_message(prompts.STATE_RULE)
    a.add_message(prompts.TASK_PROMPT)
    return a


def find_loose_states(entityKind: str, entityId: str, tmin: str, tmax: str) -> str:
    stateKind = entityKind.upper()
    return f"""
    MATCH (n1:{entityKind})-[r1:HasState]->(n2:{stateKind})
    WHERE n1.id = '{entityId}'
    AND r1.tmin <= '{tmax}' AND r1.tmax > '{tmin}'
    RETURN n2
    LIMIT 10;
    """


def find_strict_states(entityKind: str, entityId: str, timestamp: str) -> str:
    stateKind = entityKind.upper()
    return f"""
    MATCH (n1:{entityKind})-[r1:HasState]->(n2:{stateKind})
    WHERE n1.id = '{entityId}'
    AND r1.tmin <= '{timestamp}' AND r1.tmax > '{timestamp}'
    RETURN n2
    LIMIT 10;
    """


def _entity_kind(ele) -> Optional[str]:
    if ele["isNative"] == "true":
        return ele["kind2"]
    if ele["isNative"] == "false":
        return ele["tag"]
    return None


def check_statepath(query_executor, semanticAnalyzer: GenericAssistant, statepath,
                    semantic_format=None, summary_format_fn=None) -> Tuple[Optional[str], Dict[str, List[str]]]:
    timestamp = error_message = None
    for ele in statepath:
        if isinstance(ele, Node) and ele["kind"] == "Event":
            timestamp = ele["timestamp"]
            error_message = ele["message"]
    path_clues: Dict[str, List[str]] = {}
    kinds: List[str] = []
    for ele in statepath:
        if isinstance(ele, Node) and not (ele["kind2"] == "Event" or ele["kind"] == "Event"):
            kind = _entity_kind(ele)
            eid = ele["id"]
            kinds.append(kind)
            path_clues[f"{kind}({eid})"] = check_states_of_entity(
                kind, eid, error_message, timestamp, query_executor, semanticAnalyzer,
                semantic_format=semantic_format)
    semanticAnalyzer.add_message(prompts.summary_prompt(kinds))
    fmt = summary_format_fn(kinds) if summary_format_fn is not None else None
    semanticAnalyzer.run_assistant(response_format=fmt)
    messages = semanticAnalyzer.wait_get_last_k_message(1)
    if messages is None:
        raise RuntimeError(f"summary run {semanticAnalyzer.run.id} did not complete")
    report = messages.data[0].content[0].text.value
    return report, path_clues


def check_states_existence_and_semantic(query_executor, cypher_query: str, semanticAnalyzer: GenericAssistant,
                                        error_message: str, semantic_format=None) -> List[str]:
    clues = []
    records = query_executor.run_query(cypher_query)
    if not records:
        clues.append("There is not a STATE node corresponds to the Entity node")
    else:
        for r in records:
            state = r["n2"]
            clues.append(state["kind"] + "(" + state["id"] + "): " +
                         check_semantic(state, error_message, semanticAnalyzer, semantic_format))
    return clues


def check_states_of_entity(entity_kind: str, entity_id: str, error_message: str, timestamp: str,
                           query_executor, semanticAnalyzer: GenericAssistant, semantic_format=None) -> List[str]:
    records = query_executor.run_query(find_strict_states(entity_kind, entity_id, timestamp))
    clues: List[str] = []
    if not records:
        name = ad_hoc_find_entity_name(entity_kind, entity_id, query_executor)
        clue = prompts.missing_state_clue(entity_kind, entity_id, name)
        clues.append(clue)
        semanticAnalyzer.add_message(clue)  # recorded in the thread, no run (analyze_root_cause.py:182-184)
    else:
        for r in records:
            state = r["n2"]
            clues.append(state["kind"].upper() + "(" + state["id"] + "): " +
                         check_semantic(state, error_message, semanticAnalyzer, semantic_format))
    for c in clues:
        log.info("clue: %s", c)
    return clues


def ad_hoc_find_entity_name(entity_kind: str, entity_id: str, query_executor):
    q = f"""
    match (n1:{entity_kind})
    where n1.id = '{entity_id}'
    return n1
    limit 1
    """
    entity = query_executor.run_query(q)[0]["n1"]
    if entity["isNative"] == "true":
        key = "name2"
    elif entity["isAtomic"] == "true":
        key = "val"
    elif entity["tag"] in ("nfs", "hostPath"):
        key = "path"
    elif entity["tag"] == "container":
        key = "containerName"
    elif entity["tag"] == "image":
        key = "imageName"
    else:
        raise ValueError(f"cannot name entity {entity_kind}({entity_id})")
    return entity[key]


def check_semantic(state_node, error_message: str, semanticAnalyzer: GenericAssistant, semantic_format=None) -> str:
    subset = prompts.state_subset(dict(state_node.items()))
    prompt = prompts.semantic_prompt(state_node["kind"], error_message, subset)
    semanticAnalyzer.add_message(prompt)
    semanticAnalyzer.run_assistant(response_format=semantic_format)
    messages = semanticAnalyzer.wait_get_last_k_message(1)
    if messages is None:
        raise RuntimeError(f"semantic run {semanticAnalyzer.run.id} did not complete")
    return messages.data[0].content[0].text.value
