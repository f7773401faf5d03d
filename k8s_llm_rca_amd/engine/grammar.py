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
