"""Row-wise expression evaluation with Cypher's three-valued logic (null = None)."""
from __future__ import annotations

import math
import re
from typing import Any, Callable, Dict, List, Optional

from ..model import CypherError, CypherTypeError, Entity, Node, Path, Relationship
from . import ast as A

AGGREGATES = {"count", "collect", "sum", "avg", "min", "max"}


def is_num(x) -> bool:
    return isinstance(x, (int, float)) and not isinstance(x, bool)


def cy_eq(a, b):
    """Cypher equality: None if either side is null."""
    if a is None or b is None:
        return None
    if is_num(a) and is_num(b):
        return a == b
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        if len(a) != len(b):
            return False
        res = True
        for x, y in zip(a, b):
            r = cy_eq(x, y)
            if r is False:
                return False
            if r is None:
                res = None
        return res
    if type(a) is not type(b) and not (isinstance(a, Entity) and isinstance(b, Entity)):
        if isinstance(a, bool) or isinstance(b, bool) or isinstance(a, str) or isinstance(b, str):
            return False
    return a == b


def cy_cmp(op: str, a, b):
    if a is None or b is None:
        return None
    if is_num(a) and is_num(b):
        pass
    elif isinstance(a, str) and isinstance(b, str):
        pass
    elif isinstance(a, bool) and isinstance(b, bool):
        pass
    else:
        return None
    if op == "<":
        return a < b
    if op == "<=":
        return a <= b
    if op == ">":
        return a > b
    return a >= b


def cy_and(a, b):
    if a is False or b is False:
        return False
    if a is None or b is None:
        return None
    return True


def cy_or(a, b):
    if a is True or b is True:
        return True
    if a is None or b is None:
        return None
    return False


def cy_not(a):
    return None if a is None else (not a)


def _bool(v, what="predicate"):
    if v is None or isinstance(v, bool):
        return v
    raise CypherTypeError(f"Type mismatch: expected Boolean but was {type(v).__name__} in {what}")


def cy_in(x, lst):
    if lst is None:
        return None
    if not isinstance(lst, (list, tuple)):
        raise CypherTypeError(f"Type mismatch: expected List but was {type(lst).__name__}")
    saw_null = x is None
    for y in lst:
        r = cy_eq(x, y)
        if r is True:
            return True
        if r is None:
            saw_null = True
    return None if saw_null else False


class Env:
    """Variable scope chain; the root resolves variables through a callback."""

    __slots__ = ("vars", "parent", "resolve", "params")

    def __init__(self, resolve: Optional[Callable[[str], Any]], params: Dict[str, Any],
                 parent: "Env" = None, vars: Optional[Dict[str, Any]] = None):
        self.resolve = resolve
        self.params = params
        self.parent = parent
        self.vars = vars or {}

    def lookup(self, name: str):
        e = self
        while e is not None:
            if name in e.vars:
                return e.vars[name]
            if e.resolve is not None:
                return e.resolve(name)
            e = e.parent
        raise CypherError(f"Variable `{name}` not defined")

    def child(self, vars: Dict[str, Any]) -> "Env":
        return Env(None, self.params, self, vars)


def _prop(obj, key):
    if obj is None:
        return None
    if isinstance(obj, Entity):
        return obj[key]
    if isinstance(obj, dict):
        return obj.get(key)
    raise CypherTypeError(f"Type mismatch: expected a map, node or relationship but was {type(obj).__name__}")


def _index(obj, idx):
    if obj is None or idx is None:
        return None
    if isinstance(obj, (list, tuple)):
        if not isinstance(idx, int) or isinstance(idx, bool):
            raise CypherTypeError("list index must be an integer")
        try:
            return obj[idx]
        except IndexError:
            return None
    if isinstance(obj, (dict, Entity)) and isinstance(idx, str):
        return _prop(obj, idx)
    raise CypherTypeError(f"cannot index {type(obj).__name__}")


def _to_list(x):
    if x is None:
        return None
    if isinstance(x, Path):
        return list(x.nodes)
    if isinstance(x, (list, tuple)):
        return list(x)
    raise CypherTypeError(f"Type mismatch: expected List but was {type(x).__name__}")


def _func(name: str, args: List[Any]):
    n = len(args)
    a0 = args[0] if n else None
    if name == "size":
        if a0 is None:
            return None
        if isinstance(a0, (list, tuple, str)):
            return len(a0)
        raise CypherTypeError("size() expects a list or string")
    if name == "length":
        if a0 is None:
            return None
        return len(a0)
    if name == "nodes":
        return None if a0 is None else list(a0.nodes)
    if name in ("relationships", "rels"):
        return None if a0 is None else list(a0.relationships)
    if name == "type":
        return None if a0 is None else a0.type
    if name == "labels":
        return None if a0 is None else sorted(a0.labels)
    if name in ("id",):
        return None if a0 is None else a0.id
    if name in ("elementid",):
        return None if a0 is None else a0.element_id
    if name == "keys":
        if a0 is None:
            return None
        return list(a0.keys())
    if name == "properties":
        return None if a0 is None else dict(a0.items())
    if name == "startnode":
        return None if a0 is None else a0.start_node
    if name == "endnode":
        return None if a0 is None else a0.end_node
    if name == "coalesce":
        for x in args:
            if x is not None:
                return x
        return None
    if name == "head":
        return None if not a0 else a0[0]
    if name == "last":
        return None if not a0 else a0[-1]
    if name == "tail":
        return None if a0 is None else list(a0[1:])
    if name == "reverse":
        return None if a0 is None else (a0[::-1] if isinstance(a0, str) else list(reversed(a0)))
    if name == "range":
        step = args[2] if n > 2 else 1
        return list(range(args[0], args[1] + (1 if step > 0 else -1), step))
    if name in ("tolower", "lower"):
        return None if a0 is None else str(a0).lower()
    if name in ("toupper", "upper"):
        return None if a0 is None else str(a0).upper()
    if name == "trim":
        return None if a0 is None else str(a0).strip()
    if name == "ltrim":
        return None if a0 is None else str(a0).lstrip()
    if name == "rtrim":
        return None if a0 is None else str(a0).rstrip()
    if name == "tostring":
        if a0 is None:
            return None
        if isinstance(a0, bool):
            return "true" if a0 else "false"
        return str(a0)
    if name == "tointeger":
        try:
            return None if a0 is None else int(float(a0))
        except (TypeError, ValueError):
            return None
    if name == "tofloat":
        try:
            return None if a0 is None else float(a0)
        except (TypeError, ValueError):
            return None
    if name == "split":
        return None if a0 is None or args[1] is None else a0.split(args[1])
    if name == "replace":
        return None if None in args else args[0].replace(args[1], args[2])
    if name == "substring":
        if a0 is None:
            return None
        return a0[args[1]:] if n == 2 else a0[args[1]:args[1] + args[2]]
    if name == "left":
        return None if a0 is None else a0[:args[1]]
    if name == "right":
        return None if a0 is None else a0[-args[1]:] if args[1] else ""
    if name == "abs":
        return None if a0 is None else abs(a0)
    if name == "exists":
        return a0 is not None
    if name in ("sqrt",):
        return None if a0 is None else math.sqrt(a0)
    raise CypherError(f"Unknown function '{name}'")


def evaluate(e: A.Expr, env: Env):
    t = type(e)
    if t is A.Literal:
        return e.value
    if t is A.Var:
        return env.lookup(e.name)
    if t is A.Prop:
        return _prop(evaluate(e.target, env), e.key)
    if t is A.Param:
        if e.name not in env.params:
            raise CypherError(f"Expected parameter(s): {e.name}")
        return env.params[e.name]
    if t is A.BinOp:
        op = e.op
        if op == "and":
            left = _bool(evaluate(e.left, env))
            if left is False:
                return False
            return cy_and(left, _bool(evaluate(e.right, env)))
        if op == "or":
            left = _bool(evaluate(e.left, env))
            if left is True:
                return True
            return cy_or(left, _bool(evaluate(e.right, env)))
        if op == "xor":
            a, b = _bool(evaluate(e.left, env)), _bool(evaluate(e.right, env))
            return None if a is None or b is None else (a != b)
        a = evaluate(e.left, env)
        b = evaluate(e.right, env)
        if op == "=":
            return cy_eq(a, b)
        if op == "<>":
            r = cy_eq(a, b)
            return None if r is None else (not r)
        if op in ("<", "<=", ">", ">="):
            return cy_cmp(op, a, b)
        if op == "in":
            return cy_in(a, b)
        if op in ("contains", "starts", "ends"):
            if not isinstance(a, str) or not isinstance(b, str):
                return None
            return (b in a) if op == "contains" else (a.startswith(b) if op == "starts" else a.endswith(b))
        if op == "=~":
            if not isinstance(a, str) or not isinstance(b, str):
                return None
            return re.fullmatch(b, a) is not None
        if a is None or b is None:
            return None
        if op == "+":
            if isinstance(a, list) or isinstance(b, list):
                return (a if isinstance(a, list) else [a]) + (b if isinstance(b, list) else [b])
            if isinstance(a, str) or isinstance(b, str):
                return str(a) + str(b)
            return a + b
        if op == "-":
            return a - b
        if op == "*":
            return a * b
        if op == "/":
            if isinstance(a, int) and isinstance(b, int):
                if b == 0:
                    raise CypherError("/ by zero")
                q = abs(a) // abs(b)
                return q if (a >= 0) == (b >= 0) else -q
            return a / b
        if op == "%":
            return math.fmod(a, b) if (isinstance(a, float) or isinstance(b, float)) else int(math.fmod(a, b))
        if op == "^":
            return float(a) ** float(b)
        raise CypherError(f"unsupported operator {op}")
    if t is A.UnaryOp:
        v = evaluate(e.operand, env)
        if e.op == "not":
            return cy_not(_bool(v))
        if v is None:
            return None
        return -v if e.op == "neg" else v
    if t is A.IsNull:
        v = evaluate(e.operand, env)
        return (v is not None) if e.negate else (v is None)
    if t is A.ListLit:
        return [evaluate(x, env) for x in e.items]
    if t is A.MapLit:
        return {k: evaluate(v, env) for k, v in e.items.items()}
    if t is A.Index:
        return _index(evaluate(e.target, env), evaluate(e.index, env))
    if t is A.Slice:
        lst = evaluate(e.target, env)
        if lst is None:
            return None
        lo = evaluate(e.lo, env) if e.lo is not None else None
        hi = evaluate(e.hi, env) if e.hi is not None else None
        if (e.lo is not None and lo is None) or (e.hi is not None and hi is None):
            return None
        return list(lst[lo:hi]) if not isinstance(lst, str) else lst[lo:hi]
    if t is A.ListPredicate:
        lst = _to_list(evaluate(e.source, env))
        if lst is None:
            return None
        n_true = 0
        n_null = 0
        for x in lst:
            r = _bool(evaluate(e.where, env.child({e.var: x})))
            if r is True:
                n_true += 1
                if e.kind == "any":
                    return True
                if e.kind == "none":
                    return False
            elif r is None:
                n_null += 1
            elif e.kind == "all":
                return False
        if e.kind == "all":
            return None if n_null else True
        if e.kind == "any":
            return None if n_null else False
        if e.kind == "none":
            return None if n_null else True
        # single
        if n_true > 1:
            return False
        if n_null:
            return None
        return n_true == 1
    if t is A.ListComprehension:
        lst = _to_list(evaluate(e.source, env))
        if lst is None:
            return None
        out = []
        for x in lst:
            sub = env.child({e.var: x})
            if e.where is not None and _bool(evaluate(e.where, sub)) is not True:
                continue
            out.append(evaluate(e.mapping, sub) if e.mapping is not None else x)
        return out
    if t is A.CaseExpr:
        if e.subject is not None:
            s = evaluate(e.subject, env)
            for c, v in e.whens:
                if cy_eq(s, evaluate(c, env)) is True:
                    return evaluate(v, env)
        else:
            for c, v in e.whens:
                if _bool(evaluate(c, env)) is True:
                    return evaluate(v, env)
        return evaluate(e.default, env) if e.default is not None else None
    if t is A.FuncCall:
        if e.name in AGGREGATES:
            raise CypherError(f"Aggregation function '{e.name}' not allowed here")
        return _func(e.name, [evaluate(a, env) for a in e.args])
    raise CypherError(f"cannot evaluate {t.__name__}")


def has_aggregate(e: A.Expr) -> bool:
    if isinstance(e, A.FuncCall):
        if e.name in AGGREGATES:
            return True
        return any(has_aggregate(a) for a in e.args)
    for f in ("left", "right", "operand", "target", "index", "lo", "hi", "source", "where", "mapping"):
        sub = getattr(e, f, None)
        if isinstance(sub, A.Expr) and has_aggregate(sub):
            return True
    if isinstance(e, A.ListLit):
        return any(has_aggregate(x) for x in e.items)
    return False


def free_vars(e, bound=frozenset()) -> set:
    """Variables an expression reads (excluding list-predicate locals)."""
    out = set()

    def walk(x, b):
        if x is None:
            return
        tx = type(x)
        if tx is A.Var:
            if x.name not in b:
                out.add(x.name)
        elif tx in (A.ListPredicate, A.ListComprehension):
            walk(x.source, b)
            nb = b | {x.var}
            walk(x.where, nb)
            walk(getattr(x, "mapping", None), nb)
        elif tx is A.ListLit:
            for i in x.items:
                walk(i, b)
        elif tx is A.MapLit:
            for i in x.items.values():
                walk(i, b)
        elif tx is A.FuncCall:
            for i in x.args:
                walk(i, b)
        elif tx is A.CaseExpr:
            walk(x.subject, b)
            for c, v in x.whens:
                walk(c, b)
                walk(v, b)
            walk(x.default, b)
        else:
            for f in ("left", "right", "operand", "target", "index", "lo", "hi"):
                walk(getattr(x, f, None), b)

    walk(e, set(bound))
    return out
