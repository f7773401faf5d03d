"""Response grammars for constrained decoding (SURVEY.md §7.4 hard part #1).

The reference pipeline only proceeds when GPT-4 returns a fenced JSON block
with a valid ``DestinationKind`` (``find_srckind_metapath_neo4j.py:193-196``)
and a fenced, executable Cypher query (``generate_query.py:83-85``).  With
random-init weights that only happens if decoding is constrained, so each
stage hands the engine a small grammar:

``Lit(text)``            forced text (jump-forward: prefilled, not sampled)
``Choice(options)``      one of a finite set of strings (token trie mask)
``Free(max_tokens)``     free text over a token subset that excludes the
                         ``forbid`` characters; ends by sampling a terminator
                         or by hitting ``max_tokens``
``Repeat(body, ...)``    ``min..max`` repetitions with a separator; the
                         model decides to continue or close
``Ref(name)``            re-emits the text a previous named ``Choice`` produced

A ``Grammar`` can carry ``hints`` ({choice name: option}) -- oracle guidance
used by benchmarks so random weights follow the incident's true metapath;
with hints off the model's own logits choose.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Union


@dataclass
class Lit:
    text: str


@dataclass
class Choice:
    options: List[str]
    name: Optional[str] = None


@dataclass
class Free:
    max_tokens: int
    forbid: str = '"\n`\\{}'
    min_tokens: int = 1
    name: Optional[str] = None


@dataclass
class Repeat:
    body: List["Seg"]
    sep: str
    close: str
    min: int = 1
    max: int = 4
    name: Optional[str] = None


@dataclass
class Ref:
    name: str


Seg = Union[Lit, Choice, Free, Repeat, Ref]


@dataclass
class Grammar:
    segments: List[Seg]
    hints: Dict[str, Union[str, int]] = field(default_factory=dict)
    name: str = ""


def slot_key(name: Optional[str], suffix: str) -> Optional[str]:
    """Hint key of a named slot; slots inside a Repeat get '.<iteration>' suffixes."""
    return None if name is None else name + suffix


def render(g: Grammar, choose: Callable[[Choice, Dict[str, str]], str],
           free_text: Callable[[Free], str], repeat_count: Callable[[Repeat], int]) -> str:
    """Produce a string in the grammar's language (used by scripted backends/tests)."""
    out: List[str] = []
    named: Dict[str, str] = {}

    def emit(segs: Sequence[Seg], suffix: str):
        for s in segs:
            if isinstance(s, Lit):
                out.append(s.text)
            elif isinstance(s, Choice):
                key = slot_key(s.name, suffix)
                v = choose(Choice(s.options, key), named)
                if v not in s.options:
                    raise ValueError(f"{v!r} not an option of {key}")
                if key:
                    named[key] = v
                out.append(v)
            elif isinstance(s, Free):
                out.append(free_text(s))
            elif isinstance(s, Ref):
                out.append(named.get(slot_key(s.name, suffix), named.get(s.name, "")))
            elif isinstance(s, Repeat):
                n = max(s.min, min(s.max, repeat_count(Repeat(s.body, s.sep, s.close, s.min, s.max,
                                                              slot_key(s.name, suffix)))))
                for i in range(n):
                    if i:
                        out.append(s.sep)
                    emit(s.body, f"{suffix}.{i}")
                out.append(s.close)

    emit(g.segments, "")
    return "".join(out)


def hinted_render(g: Grammar, fill: str = "ok") -> str:
    """Render following ``g.hints`` (first option when no hint)."""
    def choose(c: Choice, named):
        h = g.hints.get(c.name) if c.name else None
        return h if h in c.options else c.options[0]

    def rep(r: Repeat):
        h = g.hints.get(r.name) if r.name else None
        return int(h) if h is not None else r.min

    return render(g, choose, lambda f: fill, rep)


# ---------------------------------------------------------------- JSON form
# Grammars travel over the HTTP API as ``response_format = {"type":
# "k8s_grammar", "grammar": grammar_to_json(g)}`` (api/http.py).

def _seg_to_json(s: Seg) -> dict:
    if isinstance(s, Lit):
        return {"lit": s.text}
    if isinstance(s, Choice):
        return {"choice": list(s.options), "name": s.name}
    if isinstance(s, Free):
        return {"free": s.max_tokens, "forbid": s.forbid, "min": s.min_tokens, "name": s.name}
    if isinstance(s, Repeat):
        return {"repeat": [_seg_to_json(b) for b in s.body], "sep": s.sep, "close": s.close, "min": s.min,
                "max": s.max, "name": s.name}
    if isinstance(s, Ref):
        return {"ref": s.name}
    raise TypeError(f"not a grammar segment: {s!r}")


def _seg_from_json(d: dict) -> Seg:
    if "lit" in d:
        return Lit(str(d["lit"]))
    if "choice" in d:
        return Choice([str(o) for o in d["choice"]], d.get("name"))
    if "free" in d:
        return Free(int(d["free"]), d.get("forbid", '"\n`\\{}'), int(d.get("min", 1)), d.get("name"))
    if "repeat" in d:
        return Repeat([_seg_from_json(b) for b in d["repeat"]], str(d["sep"]), str(d["close"]),
                      int(d.get("min", 1)), int(d.get("max", 4)), d.get("name"))
    if "ref" in d:
        return Ref(str(d["ref"]))
    raise ValueError(f"unknown grammar segment {d!r}")


def grammar_to_json(g: Grammar) -> dict:
    return {"segments": [_seg_to_json(s) for s in g.segments], "hints": dict(g.hints), "name": g.name}


def grammar_from_json(d: dict) -> Grammar:
    return Grammar([_seg_from_json(s) for s in d["segments"]], dict(d.get("hints") or {}), d.get("name", ""))
