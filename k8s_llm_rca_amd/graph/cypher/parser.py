"""Lexer + recursive-descent parser for the Cypher subset.

Accepts every construct in the reference's own queries and generation
template (SURVEY.md §2 'Cypher constructs G8 must accept'): node/relationship
patterns incl. ``-[*1..3]-``, named paths, WHERE with boolean / comparison /
``CONTAINS`` / ``IN`` / ``IS NULL`` / list predicates / slicing / ``$params``,
``WITH``, ``RETURN [DISTINCT] ... AS``, ``ORDER BY``, ``SKIP``, ``LIMIT``,
``UNWIND``, trailing ``;`` and case-insensitive keywords.  Anything else raises
:class:`CypherSyntaxError` with a Neo4j-style message so the LLM repair loop of
the pipeline gets useful feedback (``test_all.py:109-115``).
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

from ..model import CypherSyntaxError
from . import ast as A

KEYWORDS = {
    "MATCH", "OPTIONAL", "WHERE", "WITH", "RETURN", "DISTINCT", "AS", "LIMIT", "SKIP", "ORDER", "BY",
    "ASC", "ASCENDING", "DESC", "DESCENDING", "AND", "OR", "XOR", "NOT", "IN", "CONTAINS", "STARTS",
    "ENDS", "IS", "NULL", "TRUE", "FALSE", "UNWIND", "CASE", "WHEN", "THEN", "ELSE", "END",
}
UNSUPPORTED = {"CREATE", "MERGE", "DELETE", "DETACH", "SET", "REMOVE", "CALL", "FOREACH", "LOAD", "UNION", "YIELD"}

_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<num>\d+\.\d+(?:[eE][+-]?\d+)?|\d+(?:[eE][+-]?\d+)?)
  | (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<param>\$[A-Za-z_][A-Za-z_0-9]*|\$\d+)
  | (?P<ident>[A-Za-z_][A-Za-z_0-9]*|`[^`]*`)
  | (?P<op>->|<-|\.\.|<>|!=|<=|>=|=~|[-+*/%^=<>(){}\[\],.:;|])
""", re.VERBOSE | re.DOTALL)

_ESC = {"n": "\n", "t": "\t", "r": "\r", "b": "\b", "f": "\f", "'": "'", '"': '"', "\\": "\\"}


class Tok:
    __slots__ = ("kind", "value", "pos", "end")

    def __init__(self, kind, value, pos, end):
        self.kind, self.value, self.pos, self.end = kind, value, pos, end

    def __repr__(self):
        return f"Tok({self.kind},{self.value!r})"


def _unescape(s: str) -> str:
    out = []
    i = 0
    while i < len(s):
        c = s[i]
        if c == "\\" and i + 1 < len(s):
            n = s[i + 1]
            if n == "u" and i + 5 < len(s) + 0:
                try:
                    out.append(chr(int(s[i + 2:i + 6], 16)))
                    i += 6
                    continue
                except ValueError:
                    pass
            out.append(_ESC.get(n, "\\" + n))
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)


def tokenize(q: str) -> List[Tok]:
    toks: List[Tok] = []
    pos = 0
    n = len(q)
    while pos < n:
        m = _TOKEN_RE.match(q, pos)
        if m is None:
            raise CypherSyntaxError(_err(q, pos, f"Invalid input '{q[pos]}'"))
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "num" and pos + len(text) < n and q[pos + len(text)] == "." and text.isdigit() is False:
            pass
        if kind != "ws":
            if kind == "str":
                toks.append(Tok("str", _unescape(text[1:-1]), pos, m.end()))
            elif kind == "num":
                toks.append(Tok("num", float(text) if any(c in text for c in ".eE") else int(text), pos, m.end()))
            elif kind == "ident":
                if text.startswith("`"):
                    toks.append(Tok("ident", text[1:-1], pos, m.end()))
                elif text.upper() in KEYWORDS:
                    toks.append(Tok("kw", text.upper(), pos, m.end()))
                else:
                    toks.append(Tok("ident", text, pos, m.end()))
            elif kind == "param":
                toks.append(Tok("param", text[1:], pos, m.end()))
            else:
                toks.append(Tok("op", text, pos, m.end()))
        pos = m.end()
    toks.append(Tok("eof", None, n, n))
    return toks


def _err(q: str, pos: int, msg: str) -> str:
    line = q.count("\n", 0, pos) + 1
    col = pos - (q.rfind("\n", 0, pos) + 1) + 1
    return f"{msg} (line {line}, column {col} (offset: {pos}))"


class Parser:
    def __init__(self, q: str):
        self.q = q
        self.toks = tokenize(q)
        self.i = 0

    # ------------------------------------------------------------ helpers
    @property
    def t(self) -> Tok:
        return self.toks[self.i]

    def peek(self, k=1) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def fail(self, expected: str):
        t = self.t
        got = "end of input" if t.kind == "eof" else repr(self.q[t.pos:t.end])
        raise CypherSyntaxError(_err(self.q, t.pos, f"Invalid input {got}: expected {expected}"))

    def is_kw(self, *kws) -> bool:
        return self.t.kind == "kw" and self.t.value in kws

    def is_op(self, *ops) -> bool:
        return self.t.kind == "op" and self.t.value in ops

    def eat_kw(self, kw) -> Tok:
        if not self.is_kw(kw):
            self.fail(kw)
        t = self.t
        self.i += 1
        return t

    def eat_op(self, op) -> Tok:
        if not self.is_op(op):
            self.fail(f"'{op}'")
        t = self.t
        self.i += 1
        return t

    def ident(self, what="an identifier") -> str:
        t = self.t
        if t.kind == "ident":
            self.i += 1
            return t.value
        if t.kind == "kw" and t.value not in ("WHERE", "RETURN", "WITH", "MATCH"):
            # keywords are allowed as labels / property keys (e.g. n.end, :END)
            self.i += 1
            return self.q[t.pos:t.end]
        self.fail(what)

    def text_from(self, start_tok_index: int) -> str:
        a = self.toks[start_tok_index].pos
        b = self.toks[self.i - 1].end
        return self.q[a:b]

    # ------------------------------------------------------------- query
    def parse(self) -> A.Query:
        clauses = []
        if self.t.kind == "eof":
            raise CypherSyntaxError("Unexpected end of input: expected a query")
        while self.t.kind != "eof":
            if self.is_op(";"):
                self.i += 1
                if self.t.kind != "eof":
                    self.fail("end of input")
                break
            clauses.append(self.clause())
        if not clauses:
            raise CypherSyntaxError("Empty query")
        last = clauses[-1]
        if not (isinstance(last, A.Projection) and last.kind == "return"):
            raise CypherSyntaxError("Query cannot conclude with %s (must be a RETURN clause)" % type(last).__name__.upper())
        for c in clauses[:-1]:
            if isinstance(c, A.Projection) and c.kind == "return":
                raise CypherSyntaxError("RETURN can only be used at the end of the query")
        return A.Query(clauses)

    def clause(self):
        t = self.t
        if t.kind == "ident" and t.value.upper() in UNSUPPORTED or (t.kind == "kw" and t.value in UNSUPPORTED):
            raise CypherSyntaxError(_err(self.q, t.pos, f"Unsupported clause '{t.value}': this engine is read-only"))
        if self.is_kw("OPTIONAL"):
            self.i += 1
            self.eat_kw("MATCH")
            return self.match(optional=True)
        if self.is_kw("MATCH"):
            self.i += 1
            return self.match()
        if self.is_kw("WITH"):
            self.i += 1
            return self.projection("with")
        if self.is_kw("RETURN"):
            self.i += 1
            return self.projection("return")
        if self.is_kw("UNWIND"):
            self.i += 1
            e = self.expr()
            self.eat_kw("AS")
            return A.Unwind(e, self.ident())
        self.fail("one of MATCH, OPTIONAL MATCH, WITH, UNWIND, RETURN")

    def match(self, optional=False) -> A.Match:
        pats = [self.pattern_path()]
        while self.is_op(","):
            self.i += 1
            pats.append(self.pattern_path())
        where = None
        if self.is_kw("WHERE"):
            self.i += 1
            where = self.expr()
        return A.Match(pats, where, optional)

    def pattern_path(self) -> A.PatternPath:
        var = None
        if self.t.kind == "ident" and self.peek().kind == "op" and self.peek().value == "=":
            var = self.t.value
            self.i += 2
        nodes = [self.node_pat()]
        rels = []
        while self.is_op("-", "<-"):
            rels.append(self.rel_pat())
            nodes.append(self.node_pat())
        return A.PatternPath(var, nodes, rels)

    def node_pat(self) -> A.NodePat:
        self.eat_op("(")
        var = None
        if self.t.kind == "ident":
            var = self.ident()
        labels = []
        while self.is_op(":"):
            self.i += 1
            labels.append(self.ident("a label"))
        props = self.props() if self.is_op("{") else {}
        self.eat_op(")")
        return A.NodePat(var, labels, props)

    def props(self):
        self.eat_op("{")
        out = {}
        if not self.is_op("}"):
            while True:
                k = self.ident("a property key")
                self.eat_op(":")
                out[k] = self.expr()
                if self.is_op(","):
                    self.i += 1
                    continue
                break
        self.eat_op("}")
        return out

    def rel_pat(self) -> A.RelPat:
        left_arrow = self.is_op("<-")
        self.i += 1
        r = A.RelPat(None)
        if self.is_op("["):
            self.i += 1
            if self.t.kind == "ident":
                r.var = self.ident()
            if self.is_op(":"):
                self.i += 1
                r.types.append(self.ident("a relationship type"))
                while self.is_op("|"):
                    self.i += 1
                    if self.is_op(":"):
                        self.i += 1
                    r.types.append(self.ident("a relationship type"))
            if self.is_op("*"):
                self.i += 1
                r.var_length = True
                r.min_hops, r.max_hops = 1, 16
                if self.t.kind == "num":
                    r.min_hops = int(self.t.value)
                    r.max_hops = r.min_hops
                    self.i += 1
                if self.is_op(".."):
                    self.i += 1
                    r.max_hops = 16
                    if self.t.kind == "num":
                        r.max_hops = int(self.t.value)
                        self.i += 1
                elif self.t.kind == "num":
                    pass
                if r.min_hops > r.max_hops:
                    raise CypherSyntaxError("Invalid variable-length bounds %d..%d" % (r.min_hops, r.max_hops))
            if self.is_op("{"):
                r.props = self.props()
            self.eat_op("]")
        # closing part: '->' or '-'
        if self.is_op("->"):
            if left_arrow:
                raise CypherSyntaxError(_err(self.q, self.t.pos, "Relationship with both directions is not allowed"))
            self.i += 1
            r.direction = "out"
        elif self.is_op("-"):
            self.i += 1
            r.direction = "in" if left_arrow else "both"
        else:
            self.fail("'-' or '->'")
        return r

    def projection(self, kind: str) -> A.Projection:
        p = A.Projection(kind, [])
        if self.is_kw("DISTINCT"):
            self.i += 1
            p.distinct = True
        if self.is_op("*"):
            self.i += 1
            p.star = True
            if self.is_op(","):
                self.i += 1
                self._items(p)
        else:
            self._items(p)
        if self.is_kw("ORDER"):
            self.i += 1
            self.eat_kw("BY")
            while True:
                e = self.expr()
                desc = False
                if self.is_kw("DESC", "DESCENDING"):
                    desc = True
                    self.i += 1
                elif self.is_kw("ASC", "ASCENDING"):
                    self.i += 1
                p.order.append(A.OrderItem(e, desc))
                if self.is_op(","):
                    self.i += 1
                    continue
                break
        if self.is_kw("SKIP"):
            self.i += 1
            p.skip = self.expr()
        if self.is_kw("LIMIT"):
            self.i += 1
            p.limit = self.expr()
        if kind == "with" and self.is_kw("WHERE"):
            self.i += 1
            p.where = self.expr()
        return p

    def _items(self, p: A.Projection):
        while True:
            start = self.i
            e = self.expr()
            text = self.text_from(start)
            alias = None
            if self.is_kw("AS"):
                self.i += 1
                alias = self.ident()
            p.items.append(A.ReturnItem(e, alias, alias or text))
            if self.is_op(","):
                self.i += 1
                continue
            break

    # -------------------------------------------------------- expressions
    def expr(self) -> A.Expr:
        return self.or_expr()

    def _bin(self, sub, ops_kw, name_map=None):
        start = self.i
        left = sub()
        while self.is_kw(*ops_kw):
            op = self.t.value.lower()
            self.i += 1
            right = sub()
            left = A.BinOp(op, left, right, text=self.text_from(start))
        return left

    def or_expr(self):
        return self._bin(self.xor_expr, ("OR",))

    def xor_expr(self):
        return self._bin(self.and_expr, ("XOR",))

    def and_expr(self):
        return self._bin(self.not_expr, ("AND",))

    def not_expr(self):
        if self.is_kw("NOT"):
            start = self.i
            self.i += 1
            e = self.not_expr()
            return A.UnaryOp("not", e, text=self.text_from(start))
        return self.cmp_expr()

    def cmp_expr(self):
        start = self.i
        left = self.add_expr()
        while True:
            if self.is_op("=", "<>", "!=", "<", "<=", ">", ">=", "=~"):
                op = self.t.value
                op = "<>" if op == "!=" else op
                self.i += 1
                right = self.add_expr()
                left = A.BinOp(op, left, right, text=self.text_from(start))
            elif self.is_kw("IN"):
                self.i += 1
                right = self.add_expr()
                left = A.BinOp("in", left, right, text=self.text_from(start))
            elif self.is_kw("CONTAINS"):
                self.i += 1
                right = self.add_expr()
                left = A.BinOp("contains", left, right, text=self.text_from(start))
            elif self.is_kw("STARTS"):
                self.i += 1
                self.eat_kw("WITH")
                right = self.add_expr()
                left = A.BinOp("starts", left, right, text=self.text_from(start))
            elif self.is_kw("ENDS"):
                self.i += 1
                self.eat_kw("WITH")
                right = self.add_expr()
                left = A.BinOp("ends", left, right, text=self.text_from(start))
            elif self.is_kw("IS"):
                self.i += 1
                neg = False
                if self.is_kw("NOT"):
                    neg = True
                    self.i += 1
                self.eat_kw("NULL")
                left = A.IsNull(left, neg, text=self.text_from(start))
            else:
                return left

    def add_expr(self):
        start = self.i
        left = self.mul_expr()
        while self.is_op("+", "-"):
            op = self.t.value
            self.i += 1
            right = self.mul_expr()
            left = A.BinOp(op, left, right, text=self.text_from(start))
        return left

    def mul_expr(self):
        start = self.i
        left = self.pow_expr()
        while self.is_op("*", "/", "%"):
            op = self.t.value
            self.i += 1
            right = self.pow_expr()
            left = A.BinOp(op, left, right, text=self.text_from(start))
        return left

    def pow_expr(self):
        start = self.i
        left = self.unary_expr()
        while self.is_op("^"):
            self.i += 1
            right = self.unary_expr()
            left = A.BinOp("^", left, right, text=self.text_from(start))
        return left

    def unary_expr(self):
        if self.is_op("-", "+"):
            start = self.i
            op = "neg" if self.t.value == "-" else "pos"
            self.i += 1
            e = self.unary_expr()
            if op == "neg" and isinstance(e, A.Literal) and isinstance(e.value, (int, float)):
                return A.Literal(-e.value, text=self.text_from(start))
            return A.UnaryOp(op, e, text=self.text_from(start))
        return self.postfix_expr()

    def postfix_expr(self):
        start = self.i
        e = self.atom()
        while True:
            if self.is_op("."):
                self.i += 1
                key = self.ident("a property key")
                e = A.Prop(e, key, text=self.text_from(start))
            elif self.is_op("["):
                self.i += 1
                lo = hi = None
                if self.is_op(".."):
                    self.i += 1
                    if not self.is_op("]"):
                        hi = self.expr()
                    self.eat_op("]")
                    e = A.Slice(e, None, hi, text=self.text_from(start))
                    continue
                lo = self.expr()
                if self.is_op(".."):
                    self.i += 1
                    if not self.is_op("]"):
                        hi = self.expr()
                    self.eat_op("]")
                    e = A.Slice(e, lo, hi, text=self.text_from(start))
                else:
                    self.eat_op("]")
                    e = A.Index(e, lo, text=self.text_from(start))
            else:
                return e

    def atom(self):
        t = self.t
        start = self.i
        if t.kind == "num":
            self.i += 1
            return A.Literal(t.value, text=self.text_from(start))
        if t.kind == "str":
            self.i += 1
            return A.Literal(t.value, text=self.text_from(start))
        if t.kind == "param":
            self.i += 1
            return A.Param(t.value, text=self.text_from(start))
        if t.kind == "kw":
            if t.value in ("TRUE", "FALSE"):
                self.i += 1
                return A.Literal(t.value == "TRUE", text=self.text_from(start))
            if t.value == "NULL":
                self.i += 1
                return A.Literal(None, text=self.text_from(start))
            if t.value == "CASE":
                return self.case_expr()
            if t.value in ("CONTAINS", "END", "ASC", "DESC") and self.peek().kind == "op" and self.peek().value != "(":
                pass
        if self.is_op("("):
            self.i += 1
            e = self.expr()
            self.eat_op(")")
            return e
        if self.is_op("["):
            return self.list_expr()
        if self.is_op("{"):
            items = {}
            self.i += 1
            if not self.is_op("}"):
                while True:
                    k = self.ident("a map key")
                    self.eat_op(":")
                    items[k] = self.expr()
                    if self.is_op(","):
                        self.i += 1
                        continue
                    break
            self.eat_op("}")
            return A.MapLit(items, text=self.text_from(start))
        if t.kind == "ident":
            name = t.value
            if self.peek().kind == "op" and self.peek().value == "(":
                return self.func_call()
            self.i += 1
            return A.Var(name, text=self.text_from(start))
        self.fail("an expression")

    def case_expr(self):
        start = self.i
        self.eat_kw("CASE")
        subject = None
        if not self.is_kw("WHEN"):
            subject = self.expr()
        whens = []
        while self.is_kw("WHEN"):
            self.i += 1
            c = self.expr()
            self.eat_kw("THEN")
            whens.append((c, self.expr()))
        default = None
        if self.is_kw("ELSE"):
            self.i += 1
            default = self.expr()
        self.eat_kw("END")
        return A.CaseExpr(subject, whens, default, text=self.text_from(start))

    def list_expr(self):
        start = self.i
        self.eat_op("[")
        # list comprehension: [x IN list WHERE pred | expr]
        if self.t.kind == "ident" and self.peek().kind == "kw" and self.peek().value == "IN":
            var = self.t.value
            self.i += 2
            src = self.expr()
            where = mapping = None
            if self.is_kw("WHERE"):
                self.i += 1
                where = self.expr()
            if self.is_op("|"):
                self.i += 1
                mapping = self.expr()
            self.eat_op("]")
            return A.ListComprehension(var, src, where, mapping, text=self.text_from(start))
        items = []
        if not self.is_op("]"):
            while True:
                items.append(self.expr())
                if self.is_op(","):
                    self.i += 1
                    continue
                break
        self.eat_op("]")
        return A.ListLit(items, text=self.text_from(start))

    def func_call(self):
        start = self.i
        name = self.t.value.lower()
        self.i += 1
        self.eat_op("(")
        if name in ("all", "any", "none", "single") and self.t.kind == "ident" and \
                self.peek().kind == "kw" and self.peek().value == "IN":
            var = self.t.value
            self.i += 2
            src = self.expr()
            self.eat_kw("WHERE")
            cond = self.expr()
            self.eat_op(")")
            return A.ListPredicate(name, var, src, cond, text=self.text_from(start))
        if self.is_op("*"):
            self.i += 1
            self.eat_op(")")
            return A.FuncCall(name, [], star=True, text=self.text_from(start))
        distinct = False
        if self.is_kw("DISTINCT"):
            distinct = True
            self.i += 1
        args = []
        if not self.is_op(")"):
            while True:
                args.append(self.expr())
                if self.is_op(","):
                    self.i += 1
                    continue
                break
        self.eat_op(")")
        return A.FuncCall(name, args, distinct=distinct, text=self.text_from(start))


_CACHE = {}


def parse(q: str) -> A.Query:
    """Parse (cached by query text)."""
    r = _CACHE.get(q)
    if r is None:
        r = Parser(q).parse()
        if len(_CACHE) > 4096:
            _CACHE.clear()
        _CACHE[q] = r
    return r
