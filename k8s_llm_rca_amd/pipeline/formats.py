"""Per-stage response grammars (what each assistant is allowed to emit).

Shapes follow what the reference asks its assistants for and then parses:

* locator -- fenced JSON ``{SourceKind, DestinationKind, RelevantResources,
  PrimaryPath}`` (``find_srckind_metapath_neo4j.py:222-235``), parsed by
  ``extract_json`` (``:193-196``);
* cypher generator -- fenced ``cypher`` block in the generation-template-1
  shape (``generate_query.py:62-71,141-208``), parsed by ``extract_cypher``;
* semantic analyzer -- free text (``analyze_root_cause.py:245-249``);
* summary -- the JSON-style report requested at ``analyze_root_cause.py:127-140``.

``budget`` controls the free-text lengths (tokens) so benchmark work per
incident is fixed and comparable.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from ..engine.grammar import Choice, Free, Grammar, Lit, Repeat


@dataclass
class GenerationBudget:
    semantic_tokens: int = 192     # one check_semantic reply
    explanation_tokens: int = 40   # per summary entry
    conclusion_tokens: int = 80
    resolution_tokens: int = 80
    max_relevant: int = 6
    max_path_edges: int = 5


def _q(s: str) -> str:
    return '"' + s + '"'


def locator_grammar(kinds: Sequence[str], src_kind: str, budget: GenerationBudget,
                    truth: Optional[Tuple[str, str, List[str]]] = None) -> Grammar:
    """truth = (src_kind, dest_kind, path_kinds) enables oracle hints."""
    kinds = list(kinds)
    ks = [_q(k) for k in kinds]
    segs = [
        Lit('```json\n{\n    "SourceKind": '), Choice(ks, "src"),
        Lit(',\n    "DestinationKind": '), Choice(ks, "dest"),
        Lit(',\n    "RelevantResources": ['),
        Repeat([Choice(ks, "rel")], sep=", ", close="]", min=1, max=budget.max_relevant, name="nrel"),
        Lit(',\n    "PrimaryPath": [\n'),
        Repeat([Lit('        {"Edge": '), Choice([str(i) for i in range(1, budget.max_path_edges + 1)], "edge"),
                Lit(', "start": '), Choice(ks, "start"), Lit(', "end": '), Choice(ks, "end"), Lit("}")],
               sep=",\n", close="\n    ]", min=1, max=budget.max_path_edges, name="npath"),
        Lit("\n}\n```"),
    ]
    hints: Dict[str, object] = {}
    if truth is not None:
        src, dest, path = truth
        hints["src"] = _q(src)
        hints["dest"] = _q(dest)
        rel = [k for k in path if k in kinds][: budget.max_relevant]
        hints["nrel"] = max(1, len(rel))
        for i, k in enumerate(rel):
            hints[f"rel.{i}"] = _q(k)
        edges = list(zip(path[:-1], path[1:]))[: budget.max_path_edges]
        hints["npath"] = max(1, len(edges))
        for i, (a, b) in enumerate(edges):
            hints[f"edge.{i}"] = str(i + 1)
            hints[f"start.{i}"] = _q(a)
            hints[f"end.{i}"] = _q(b)
    return Grammar(segs, hints, name="locator")


def parse_metapath_str(metapath_str: str) -> List[List[str]]:
    return [seg.strip().split(", ") for seg in metapath_str.split(";")[:-1]]


def cypher_grammar(metapath_str: str, error_message: str, hint: bool = True) -> Grammar:
    """generation-template-1 shaped query over the extended metapath's labels/types/keys."""
    segs_mp = parse_metapath_str(metapath_str)
    aliases: Dict[str, str] = {"EVENT": "evt"}
    idx = 1
    for seg in segs_mp:
        for k in (seg[1], seg[2]):
            if k not in aliases:
                aliases[k] = f"n{idx}"
                idx += 1
    node_opts = [f"{a}:{k}" for k, a in aliases.items()]
    rel_types = sorted({s[0] for s in segs_mp})
    keys = sorted({s[3] for s in segs_mp})
    segs: list = [Lit("```cypher\nMATCH (evt:EVENT)\nWHERE evt.message CONTAINS " + repr(error_message) +
                      "\nWITH evt\nLIMIT 1\n")]
    hints: Dict[str, object] = {}
    for i, (rt, sk, dk, key) in enumerate(segs_mp, start=1):
        segs += [Lit("MATCH ("), Choice(node_opts, f"src{i}"), Lit(f")-[r{i}:"), Choice(rel_types, f"type{i}"),
                 Lit("]->("), Choice(node_opts, f"dst{i}"), Lit(f")\nWHERE r{i}.key = '"), Choice(keys, f"key{i}"),
                 Lit("'\n")]
        if hint:
            hints[f"src{i}"] = f"{aliases[sk]}:{sk}"
            hints[f"type{i}"] = rt
            hints[f"dst{i}"] = f"{aliases[dk]}:{dk}"
            hints[f"key{i}"] = key
    ret = []
    vals = list(aliases.values())
    for j, a in enumerate(vals):
        ret.append(a)
        if j < len(segs_mp):
            ret.append(f"r{j + 1}")
    segs.append(Lit("RETURN " + ", ".join(ret) + "\n```"))
    return Grammar(segs, hints, name="cypher")


def semantic_grammar(budget: GenerationBudget) -> Grammar:
    return Grammar([Free(budget.semantic_tokens, forbid="", min_tokens=budget.semantic_tokens // 4)],
                   name="semantic")


def summary_grammar(kinds_on_path: Sequence[str], budget: GenerationBudget,
                    truth_dest: Optional[str] = None) -> Grammar:
    ks = [_q(k) for k in dict.fromkeys(kinds_on_path)] or ['"Pod"']
    scores = [_q(str(i)) for i in range(11)]
    segs = [
        Lit('{\n    "summary": [\n'),
        Repeat([Lit('        {"kind": '), Choice(ks, "kind"), Lit(', "explanation": "'),
                Free(budget.explanation_tokens), Lit('", "relevance_score": '), Choice(scores, "score"), Lit("}")],
               sep=",\n", close="\n    ],", min=1, max=max(1, len(ks)), name="nsum"),
        Lit('\n    "conclusion": "'), Free(budget.conclusion_tokens),
        Lit('",\n    "resolution": "'), Free(budget.resolution_tokens), Lit('"\n}'),
    ]
    hints: Dict[str, object] = {"nsum": len(ks)}
    for i, k in enumerate(ks):
        hints[f"kind.{i}"] = k
        hints[f"score.{i}"] = _q("10" if truth_dest and k == _q(truth_dest) else str(max(1, 6 - i)))
    return Grammar(segs, hints, name="summary")
