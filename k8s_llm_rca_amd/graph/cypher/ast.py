"""AST of the supported Cypher subset (SURVEY.md §2 'Cypher constructs G8 must accept')."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple


class Expr:
    text: str = ""


@dataclass
class Literal(Expr):
    value: Any
    text: str = ""


@dataclass
class Param(Expr):
    name: str
    text: str = ""


@dataclass
class Var(Expr):
    name: str
    text: str = ""


@dataclass
class Prop(Expr):
    target: Expr
    key: str
    text: str = ""


@dataclass
class Index(Expr):
    target: Expr
    index: Expr
    text: str = ""


@dataclass
class Slice(Expr):
    target: Expr
    lo: Optional[Expr]
    hi: Optional[Expr]
    text: str = ""


@dataclass
class BinOp(Expr):
    op: str  # and or xor + - * / % ^ = <> < <= > >= in contains starts ends =~
    left: Expr
    right: Expr
    text: str = ""


@dataclass
class UnaryOp(Expr):
    op: str  # not, neg, pos
    operand: Expr
    text: str = ""


@dataclass
class IsNull(Expr):
    operand: Expr
    negate: bool
    text: str = ""


@dataclass
class FuncCall(Expr):
    name: str  # lower-cased
    args: List[Expr]
    distinct: bool = False
    star: bool = False
    text: str = ""


@dataclass
class ListLit(Expr):
    items: List[Expr]
    text: str = ""


@dataclass
class MapLit(Expr):
    items: Dict[str, Expr]
    text: str = ""


@dataclass
class ListPredicate(Expr):
    kind: str  # all any none single
    var: str
    source: Expr
    where: Expr
    text: str = ""


@dataclass
class ListComprehension(Expr):
    var: str
    source: Expr
    where: Optional[Expr]
    mapping: Optional[Expr]
    text: str = ""


@dataclass
class CaseExpr(Expr):
    subject: Optional[Expr]
    whens: List[Tuple[Expr, Expr]]
    default: Optional[Expr]
    text: str = ""


# ------------------------------------------------------------------ patterns
@dataclass
class NodePat:
    var: Optional[str]
    labels: List[str] = field(default_factory=list)
    props: Dict[str, Expr] = field(default_factory=dict)


@dataclass
class RelPat:
    var: Optional[str]
    types: List[str] = field(default_factory=list)
    direction: str = "out"  # out: -[]->  in: <-[]-  both: -[]-
    var_length: bool = False
    min_hops: int = 1
    max_hops: int = 1
    props: Dict[str, Expr] = field(default_factory=dict)


@dataclass
class PatternPath:
    var: Optional[str]
    nodes: List[NodePat]
    rels: List[RelPat]


# ------------------------------------------------------------------- clauses
@dataclass
class ReturnItem:
    expr: Expr
    alias: Optional[str]
    name: str  # column name: alias or source text


@dataclass
class OrderItem:
    expr: Expr
    descending: bool


@dataclass
class Match:
    patterns: List[PatternPath]
    where: Optional[Expr]
    optional: bool = False


@dataclass
class Projection:
    """WITH or RETURN."""
    kind: str  # 'with' | 'return'
    items: List[ReturnItem]
    star: bool = False
    distinct: bool = False
    order: List[OrderItem] = field(default_factory=list)
    skip: Optional[Expr] = None
    limit: Optional[Expr] = None
    where: Optional[Expr] = None  # WITH ... WHERE


@dataclass
class Unwind:
    expr: Expr
    alias: str


@dataclass
class Query:
    clauses: list
