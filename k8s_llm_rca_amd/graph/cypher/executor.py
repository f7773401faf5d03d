"""Columnar executor for the Cypher subset over a :class:`PropertyGraph`.

Plan shape: each MATCH pattern is anchored on its most selective node (an
already-bound variable, a hash-index equality, a ``CONTAINS`` scan or the
smallest label) and expanded hop by hop through the CSR with the relationship
type / ``key`` filters pushed into the expand operator.  Single-variable
conjuncts of the WHERE clause (``v.p = c``, ``v.p CONTAINS c``, ``v.p IN c``)
are applied during expansion; the rest is evaluated row-wise afterwards with
Cypher null semantics.  Relationship isomorphism (a relationship is bound at
most once per MATCH) is enforced per clause, as Neo4j does.

The binding table is columnar: node / relationship columns are int64 id
arrays, so hop expansion, index lookups and substring scans run on whole
frontiers (and on the GPU via :mod:`k8s_llm_rca_amd.graph.device` when the
graph is mirrored to HBM).
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..model import CypherError, Node, Path, Record, Relationship
from ..store import PropertyGraph
from . import ast as A
from .evaluator import Env, _bool, cy_eq, evaluate, free_vars, has_aggregate
from .parser import parse

# the stored timestamp form (graph/store.py TS_FORMAT, millisecond fraction)
_TS_FIXED = re.compile(r"\d{4}-\d{2}-\d{2} \d{2}:\d{2}:\d{2}\.\d{3}")

NODE, REL, RELS, PATH, VALUE = "node", "rel", "rels", "path", "value"


class Table:
    __slots__ = ("cols", "types", "n")

    def __init__(self, n: int = 1):
        self.cols: Dict[str, Any] = {}
        self.types: Dict[str, str] = {}
        self.n = n

    def take(self, idx: np.ndarray) -> "Table":
        t = Table(len(idx))
        for k, c in self.cols.items():
            t.cols[k] = c[idx]
            t.types[k] = self.types[k]
        return t

    def add(self, name: str, col, typ: str):
        self.cols[name] = col
        self.types[name] = typ


def _obj_array(items: List[Any]) -> np.ndarray:
    a = np.empty(len(items), dtype=object)
    a[:] = items
    return a


class Executor:
    def __init__(self, graph: PropertyGraph):
        self.g = graph

    # ----------------------------------------------------------------- entry
    def run(self, query: str, params: Optional[Dict[str, Any]] = None) -> List[Record]:
        q = parse(query)
        params = dict(params or {})
        table = Table(1)
        out: List[Record] = []
        for ci, clause in enumerate(q.clauses):
            if isinstance(clause, A.Match):
                table = self._match(table, clause, params, ci)
            elif isinstance(clause, A.Unwind):
                table = self._unwind(table, clause, params)
            elif isinstance(clause, A.Projection):
                table, names = self._project(table, clause, params)
                if clause.kind == "return":
                    out = self._records(table, names)
        return out

    # ------------------------------------------------------------ row access
    def _value(self, table: Table, name: str, i: int):
        typ = table.types[name]
        v = table.cols[name][i]
        if typ == NODE:
            return None if v < 0 else Node(self.g, v)
        if typ == REL:
            return None if v < 0 else Relationship(self.g, v)
        if typ == RELS:
            return None if v is None else [Relationship(self.g, e) for e in v]
        if typ == PATH:
            if v is None:
                return None
            nodes, rels = v
            return Path([Node(self.g, n) for n in nodes], [Relationship(self.g, e) for e in rels])
        return v

    def _env(self, table: Table, i: int, params) -> Env:
        def resolve(name):
            if name not in table.cols:
                raise CypherError(f"Variable `{name}` not defined")
            return self._value(table, name, i)
        return Env(resolve, params)

    # ----------------------------------------------------------------- MATCH
    def _match(self, table: Table, m: A.Match, params, ci: int) -> Table:
        fast = self._state_pattern(table, m, params)
        if fast is not None:
            return fast
        conjuncts = _split_and(m.where) if m.where is not None else []
        pushed = [False] * len(conjuncts)
        in_rows = table.n
        if m.optional:
            table = table.take(np.arange(table.n))
            table.add(" optrow", np.arange(table.n, dtype=np.int64), VALUE)
        base = table
        new_vars: List[str] = []
        rel_cols: List[str] = []
        for pi, pat in enumerate(m.patterns):
            table = self._match_path(table, pat, conjuncts, pushed, params, f"{ci}_{pi}", new_vars, rel_cols)
        # relationship isomorphism inside one MATCH clause
        if len(rel_cols) > 1 and table.n:
            keep = np.ones(table.n, dtype=bool)
            singles = [c for c in rel_cols if table.types[c] == REL]
            multis = [c for c in rel_cols if table.types[c] == RELS]
            for a in range(len(singles)):
                for b in range(a + 1, len(singles)):
                    keep &= table.cols[singles[a]] != table.cols[singles[b]]
            if multis:
                for i in np.nonzero(keep)[0].tolist():
                    seen = set()
                    ok = True
                    for c in rel_cols:
                        v = table.cols[c][i]
                        es = v if table.types[c] == RELS else (v,)
                        for e in es:
                            if e in seen:
                                ok = False
                                break
                            seen.add(e)
                        if not ok:
                            break
                    keep[i] = ok
            if not keep.all():
                table = table.take(np.nonzero(keep)[0])
        # residual WHERE
        residual = [c for c, p in zip(conjuncts, pushed) if not p]
        if residual and table.n:
            keep = np.zeros(table.n, dtype=bool)
            for i in range(table.n):
                env = self._env(table, i, params)
                ok = True
                for c in residual:
                    if _bool(evaluate(c, env)) is not True:
                        ok = False
                        break
                keep[i] = ok
            table = table.take(np.nonzero(keep)[0])
        # drop hidden columns
        for k in [k for k in table.cols if k.startswith("  ")]:
            del table.cols[k]
            del table.types[k]
        if m.optional:
            matched = set(table.cols[" optrow"].tolist())
            missing = [r for r in range(in_rows) if r not in matched]
            if missing:
                extra = base.take(np.asarray(missing, dtype=np.int64))
                for v in new_vars:
                    if v in table.cols and v not in extra.cols:
                        typ = table.types[v]
                        if typ in (NODE, REL):
                            extra.add(v, np.full(len(missing), -1, dtype=np.int64), typ)
                        else:
                            extra.add(v, _obj_array([None] * len(missing)), typ)
                table = _concat(table, extra)
            del table.cols[" optrow"]
            del table.types[" optrow"]
        return table

    # temporal STATE lookup (G6) ------------------------------------------
    STATE_LIMIT = 64

    def _state_pattern(self, table: Table, m: A.Match, params) -> Optional[Table]:
        """The check_state queries (``analyze_root_cause.py:51-79``)::

            MATCH (n1:Kind)-[r1:HasState]->(n2:KIND)
            WHERE n1.id = 'uid' AND r1.tmin <= 'ts_a' AND r1.tmax > 'ts_b'

        run as one temporal-interval operator (``PropertyGraph.state_lookup``:
        the HIP ``state_kernel`` on a mirrored graph, batched across the
        concurrent pipelines) instead of a generic expand + filter.  The
        timestamp literals must be the fixed-width format the store parses:
        then int64-ms comparison == Cypher's lexicographic string comparison.
        Anything else returns None (generic path)."""
        if table.n != 1 or table.cols or m.optional or m.where is None or len(m.patterns) != 1:
            return None
        pat = m.patterns[0]
        if pat.var or len(pat.nodes) != 2 or len(pat.rels) != 1:
            return None
        a, b, r = pat.nodes[0], pat.nodes[1], pat.rels[0]
        if (r.types != ["HasState"] or r.direction != "out" or r.var_length or r.props or a.props or b.props
                or len(a.labels) != 1 or len(b.labels) > 1 or not (a.var and b.var and r.var)
                or len({a.var, b.var, r.var}) != 3):
            return None
        want = {}
        for c in _split_and(m.where):
            if not (isinstance(c, A.BinOp) and isinstance(c.left, A.Prop) and isinstance(c.left.target, A.Var)
                    and _is_const(c.right)):
                return None
            try:
                val = evaluate(c.right, Env(None, params))
            except CypherError:
                return None
            key = (c.left.target.name, c.left.key, c.op)
            if key in want or not isinstance(val, str):
                return None
            want[key] = val
        uid = want.pop((a.var, "id", "="), None)
        t_lo = want.pop((r.var, "tmin", "<="), None)
        t_hi = want.pop((r.var, "tmax", ">"), None)
        if want or uid is None or t_lo is None or t_hi is None:
            return None
        from ..store import ts_to_ms
        # Cypher compares these strings lexicographically; the int64-ms fast path is
        # the same order only for the stored fixed-width form (an unpadded field, a
        # 1-2 or 4-6 digit fraction would compare differently): anything else takes
        # the generic path
        if not (_TS_FIXED.fullmatch(t_lo) and _TS_FIXED.fullmatch(t_hi)):
            return None
        try:
            q_lo, q_hi = ts_to_ms(t_lo), ts_to_ms(t_hi)
        except (ValueError, TypeError):
            return None
        ents = self.g.index_lookup(a.labels[0], "id", uid)
        n1s, es = [], []
        if len(ents):
            res = self.g.state_lookup(ents, np.full(len(ents), q_hi, dtype=np.int64), b.labels[0] if b.labels else None,
                                      "loose", np.full(len(ents), q_lo, dtype=np.int64), self.STATE_LIMIT)
            for n, e in zip(ents.tolist(), res):
                if len(e) >= self.STATE_LIMIT:
                    return None  # more valid STATEs than the operator returns: generic path
                n1s += [n] * len(e)
                es += list(e)
        t = Table(len(es))
        e_arr = np.asarray(es, dtype=np.int64)
        t.add(a.var, np.asarray(n1s, dtype=np.int64), NODE)
        t.add(r.var, e_arr, REL)
        t.add(b.var, self.g.e_dst[e_arr] if len(e_arr) else np.zeros(0, dtype=np.int64), NODE)
        return t

    def _pushdown(self, var: str, conjuncts, pushed, params) -> List[Tuple[str, str, Any]]:
        """Collect single-variable filters ``(op, key, value)`` for ``var``."""
        out = []
        for j, c in enumerate(conjuncts):
            if pushed[j] or not isinstance(c, A.BinOp):
                continue
            op = c.op
            lhs, rhs = c.left, c.right
            if op == "=" and _is_prop_of(rhs, var) and _is_const(lhs):
                lhs, rhs = rhs, lhs
            if op in ("=", "contains", "in") and _is_prop_of(lhs, var) and _is_const(rhs):
                try:
                    val = evaluate(rhs, Env(None, params))
                except CypherError:
                    continue
                if op == "in" and not isinstance(val, (list, tuple)):
                    continue
                if op == "contains" and not isinstance(val, str):
                    continue
                out.append((op, lhs.key, val))
                pushed[j] = True
        return out

    def _filter_nodes(self, ids: np.ndarray, labels: Sequence[str], filters) -> np.ndarray:
        """Mask of ids satisfying labels + pushed filters."""
        m = np.ones(len(ids), dtype=bool)
        for lab in labels:
            m &= self.g.has_label(ids, lab)
        for op, key, val in filters:
            if not m.any():
                break
            sel = np.nonzero(m)[0]
            if op == "contains":
                sub = self.g.contains_scan(ids[sel], key, val)
            else:
                col = self.g.node_column(key)[ids[sel]]
                if op == "=":
                    sub = np.fromiter((cy_eq(v, val) is True for v in col), dtype=bool, count=len(sel))
                else:
                    sub = np.fromiter((any(cy_eq(v, x) is True for x in val) for v in col), dtype=bool,
                                      count=len(sel))
            m[sel] = sub
        return m

    def _anchor_ids(self, npat: A.NodePat, filters) -> np.ndarray:
        eq = [f for f in filters if f[0] == "="]
        if eq:
            op, key, val = eq[0]
            ids = self.g.index_lookup(npat.labels[0] if npat.labels else None, key, val)
            rest = [f for f in filters if f is not eq[0]]
            lab = npat.labels[1:] if npat.labels else []
            return ids[self._filter_nodes(ids, lab, rest)] if (rest or lab) else ids
        if npat.labels:
            # smallest label first
            best = min(npat.labels, key=lambda l: len(self.g.label_scan(l)))
            ids = self.g.label_scan(best)
            others = [l for l in npat.labels if l != best]
        else:
            ids = self.g.all_nodes()
            others = []
        if not filters and not others:
            return ids
        return ids[self._filter_nodes(ids, others, filters)]

    def _match_path(self, table: Table, pat: A.PatternPath, conjuncts, pushed, params, tag: str,
                    new_vars: List[str], rel_cols: List[str]) -> Table:
        nn = len(pat.nodes)
        nvars = [p.var if p.var else f"  n{tag}_{i}" for i, p in enumerate(pat.nodes)]
        rvars = [r.var if r.var else f"  r{tag}_{i}" for i, r in enumerate(pat.rels)]
        for v in nvars + rvars:
            if v in table.cols and table.types.get(v) not in (NODE, REL, RELS):
                raise CypherError(f"Variable `{v}` already declared as another type")
        node_filters = []
        for i, p in enumerate(pat.nodes):
            fl = [("=", k, evaluate(v, Env(None, params))) for k, v in p.props.items()]
            if p.var and p.var not in table.cols:
                fl += self._pushdown(p.var, conjuncts, pushed, params)
            node_filters.append(fl)
        rel_filters = []
        for i, r in enumerate(pat.rels):
            fl = [("=", k, evaluate(v, Env(None, params))) for k, v in r.props.items()]
            if r.var and r.var not in table.cols and not r.var_length:
                fl += [f for f in self._pushdown(r.var, conjuncts, pushed, params)]
            rel_filters.append(fl)

        # anchor choice
        bound = [i for i in range(nn) if nvars[i] in table.cols]
        if bound:
            a = bound[0]
        else:
            def score(i):
                f = node_filters[i]
                if any(x[0] == "=" for x in f):
                    return (0, 0)
                if pat.nodes[i].labels:
                    return (2 - (1 if f else 0), min(len(self.g.label_scan(l)) for l in pat.nodes[i].labels))
                return (3 - (1 if f else 0), self.g.num_nodes)
            a = min(range(nn), key=score)
        if nvars[a] in table.cols:
            col = table.cols[nvars[a]]
            ok = col >= 0
            if pat.nodes[a].labels or node_filters[a]:
                ok2 = np.zeros(table.n, dtype=bool)
                sel = np.nonzero(ok)[0]
                ok2[sel] = self._filter_nodes(col[sel], pat.nodes[a].labels, node_filters[a])
                ok = ok2
            table = table.take(np.nonzero(ok)[0])
        else:
            ids = self._anchor_ids(pat.nodes[a], node_filters[a])
            table = _cross(table, nvars[a], ids)
            new_vars.append(nvars[a])
        vl_cols: Dict[int, str] = {}
        # expand right then left
        order = [(i, i + 1, "right") for i in range(a, nn - 1)] + [(i, i - 1, "left") for i in range(a, 0, -1)]
        for cur, nxt, side in order:
            ri = cur if side == "right" else nxt
            r = pat.rels[ri]
            direction = r.direction
            if side == "left" and direction != "both":
                direction = "in" if direction == "out" else "out"
            cur_ids = table.cols[nvars[cur]]
            if r.var_length:
                table = self._expand_var(table, nvars[cur], nvars[nxt], rvars[ri], r, direction, side,
                                         pat.nodes[nxt], node_filters[nxt], vl_cols, ri, tag)
            else:
                if rvars[ri] in table.cols:
                    raise CypherError(f"relationship variable `{rvars[ri]}` re-bound (not supported)")
                key = None
                extra_rf = []
                for f in rel_filters[ri]:
                    if f[0] == "=" and f[1] == "key" and isinstance(f[2], str) and key is None:
                        key = f[2]
                    else:
                        extra_rf.append(f)
                valid = cur_ids >= 0
                src_rows = np.nonzero(valid)[0]
                row, eid, nbr = self.g.expand(cur_ids[src_rows], direction, r.types or None, key)
                row = src_rows[row]
                keep = np.ones(len(row), dtype=bool)
                for op, k, val in extra_rf:
                    col = self.g.edge_column(k)[eid]
                    if op == "=":
                        keep &= np.fromiter((cy_eq(v, val) is True for v in col), dtype=bool, count=len(col))
                    elif op == "contains":
                        keep &= np.fromiter((isinstance(v, str) and val in v for v in col), dtype=bool, count=len(col))
                    else:
                        keep &= np.fromiter((any(cy_eq(v, x) is True for x in val) for v in col), dtype=bool,
                                            count=len(col))
                if nvars[nxt] in table.cols:
                    keep &= table.cols[nvars[nxt]][row] == nbr
                    if pat.nodes[nxt].labels or node_filters[nxt]:
                        sel = np.nonzero(keep)[0]
                        keep[sel] = self._filter_nodes(nbr[sel], pat.nodes[nxt].labels, node_filters[nxt])
                    sel = np.nonzero(keep)[0]
                    table = table.take(row[sel])
                    table.add(rvars[ri], eid[sel], REL)
                else:
                    if pat.nodes[nxt].labels or node_filters[nxt]:
                        sel = np.nonzero(keep)[0]
                        keep[sel] = self._filter_nodes(nbr[sel], pat.nodes[nxt].labels, node_filters[nxt])
                    sel = np.nonzero(keep)[0]
                    table = table.take(row[sel])
                    table.add(rvars[ri], eid[sel], REL)
                    table.add(nvars[nxt], nbr[sel], NODE)
                    new_vars.append(nvars[nxt])
            if rvars[ri] not in new_vars:
                new_vars.append(rvars[ri])
            rel_cols.append(rvars[ri])
        if pat.var:
            paths = []
            for i in range(table.n):
                nodes = [int(table.cols[nvars[0]][i])]
                rels: List[int] = []
                for ri, r in enumerate(pat.rels):
                    if r.var_length:
                        seg_nodes, seg_edges = table.cols[vl_cols[ri]][i]
                        nodes.extend(seg_nodes[1:])
                        rels.extend(seg_edges)
                    else:
                        rels.append(int(table.cols[rvars[ri]][i]))
                        nodes.append(int(table.cols[nvars[ri + 1]][i]))
                paths.append((tuple(nodes), tuple(rels)))
            table.add(pat.var, _obj_array(paths), PATH)
            new_vars.append(pat.var)
        return table

    def _expand_var(self, table: Table, cur: str, nxt: str, rvar: str, r: A.RelPat, direction: str,
                    side: str, npat: A.NodePat, nfilters, vl_cols, ri, tag) -> Table:
        cur_ids = table.cols[cur]
        valid = np.nonzero(cur_ids >= 0)[0]
        uniq, inv = np.unique(cur_ids[valid], return_inverse=True)
        end_label = npat.labels[0] if (len(npat.labels) == 1 and nxt not in table.cols) else None
        walks = self.g.var_length(uniq, r.min_hops, r.max_hops, direction, r.types or None, end_label)
        by_start: Dict[int, List[Tuple[List[int], List[int]]]] = {}
        for srow, nodes, edges in walks:
            by_start.setdefault(srow, []).append((nodes, edges))
        rows, segs, rels, ends = [], [], [], []
        for j, trow in enumerate(valid.tolist()):
            for nodes, edges in by_start.get(int(inv[j]), ()):
                if side == "left":
                    nodes = nodes[::-1]
                    edges = edges[::-1]
                rows.append(trow)
                segs.append((tuple(nodes), tuple(edges)))
                rels.append(tuple(edges))
                ends.append(nodes[0] if side == "left" else nodes[-1])
        rows_a = np.asarray(rows, dtype=np.int64)
        ends_a = np.asarray(ends, dtype=np.int64)
        keep = np.ones(len(rows_a), dtype=bool)
        if nxt in table.cols:
            keep &= table.cols[nxt][rows_a] == ends_a
        if npat.labels or nfilters:
            sel = np.nonzero(keep)[0]
            keep[sel] = self._filter_nodes(ends_a[sel], npat.labels, nfilters)
        sel = np.nonzero(keep)[0]
        out = table.take(rows_a[sel])
        out.add(rvar, _obj_array([rels[k] for k in sel.tolist()]), RELS)
        if nxt not in table.cols:
            out.add(nxt, ends_a[sel], NODE)
        name = f"  vl{tag}_{ri}"
        out.add(name, _obj_array([segs[k] for k in sel.tolist()]), VALUE)
        vl_cols[ri] = name
        return out

    # ---------------------------------------------------------------- UNWIND
    def _unwind(self, table: Table, u: A.Unwind, params) -> Table:
        rows, vals = [], []
        for i in range(table.n):
            v = evaluate(u.expr, self._env(table, i, params))
            if v is None:
                continue
            if not isinstance(v, (list, tuple)):
                v = [v]
            for x in v:
                rows.append(i)
                vals.append(x)
        out = table.take(np.asarray(rows, dtype=np.int64))
        out.add(u.alias, _obj_array(vals), VALUE)
        return out

    # ------------------------------------------------------------ projection
    def _project(self, table: Table, p: A.Projection, params) -> Tuple[Table, List[str]]:
        items = list(p.items)
        names: List[str] = []
        if p.star:
            names = [k for k in table.cols if not k.startswith(" ")]
        aggregate = any(has_aggregate(it.expr) for it in items)
        out = Table(table.n)
        for k in names:
            out.add(k, table.cols[k], table.types[k])
        if aggregate:
            out, agg_names = self._aggregate(table, items, params)
            names = names + agg_names
        else:
            for it in items:
                col, typ = self._eval_column(table, it.expr, params)
                out.add(it.name, col, typ)
                names.append(it.name)
        if p.distinct and out.n:
            seen = set()
            keep = []
            for i in range(out.n):
                key = tuple(_hashable(out.cols[k][i]) for k in names)
                if key not in seen:
                    seen.add(key)
                    keep.append(i)
            out = out.take(np.asarray(keep, dtype=np.int64))
            if not aggregate and p.order:
                table = table.take(np.asarray(keep, dtype=np.int64))
        if p.order and out.n:
            keys = []
            for i in range(out.n):
                def resolve(name, i=i):
                    if name in out.cols:
                        return self._value(out, name, i)
                    if not aggregate and name in table.cols:
                        return self._value(table, name, i)
                    raise CypherError(f"Variable `{name}` not defined")
                env = Env(resolve, params)
                keys.append([_sort_key(evaluate(o.expr, env)) for o in p.order])
            idx = list(range(out.n))
            for j in range(len(p.order) - 1, -1, -1):
                idx.sort(key=lambda i: keys[i][j], reverse=p.order[j].descending)
            out = out.take(np.asarray(idx, dtype=np.int64))
        lo = 0
        if p.skip is not None:
            lo = int(evaluate(p.skip, Env(None, params)))
        hi = out.n
        if p.limit is not None:
            lim = evaluate(p.limit, Env(None, params))
            if not isinstance(lim, int) or lim < 0:
                raise CypherError("LIMIT expects a non-negative integer")
            hi = min(out.n, lo + lim)
        if lo or hi < out.n:
            out = out.take(np.arange(lo, max(lo, hi), dtype=np.int64))
        if p.where is not None and out.n:
            keep = [i for i in range(out.n)
                    if _bool(evaluate(p.where, self._env(out, i, params))) is True]
            out = out.take(np.asarray(keep, dtype=np.int64))
        return out, names

    def _eval_column(self, table: Table, e: A.Expr, params):
        if isinstance(e, A.Var) and e.name in table.cols:
            return table.cols[e.name], table.types[e.name]
        if isinstance(e, A.Prop) and isinstance(e.target, A.Var) and table.types.get(e.target.name) in (NODE, REL):
            ids = table.cols[e.target.name]
            src = self.g.node_column(e.key) if table.types[e.target.name] == NODE else self.g.edge_column(e.key)
            col = np.empty(table.n, dtype=object)
            ok = ids >= 0
            col[ok] = src[ids[ok]]
            col[~ok] = None
            return col, VALUE
        vals = [evaluate(e, self._env(table, i, params)) for i in range(table.n)]
        return _obj_array(vals), VALUE

    def _aggregate(self, table: Table, items: List[A.ReturnItem], params):
        keys = [it for it in items if not has_aggregate(it.expr)]
        aggs = [it for it in items if has_aggregate(it.expr)]
        key_cols = [self._eval_column(table, it.expr, params) for it in keys]
        groups: Dict[tuple, List[int]] = {}
        for i in range(table.n):
            k = tuple(_hashable(c[0][i]) for c in key_cols)
            groups.setdefault(k, []).append(i)
        if not keys and not groups:
            groups[()] = []
        out = Table(len(groups))
        gl = list(groups.values())
        for it, (col, typ) in zip(keys, key_cols):
            out.add(it.name, col[np.asarray([g[0] for g in gl], dtype=np.int64)] if gl and gl[0] else
                    _obj_array([]), typ)
        for it in aggs:
            vals = []
            for g in gl:
                vals.append(self._agg_value(table, it.expr, g, params))
            out.add(it.name, _obj_array(vals), VALUE)
        return out, [it.name for it in items]

    def _agg_value(self, table: Table, e: A.Expr, rows: List[int], params):
        if not isinstance(e, A.FuncCall) or e.name not in ("count", "collect", "sum", "avg", "min", "max"):
            raise CypherError("only top-level aggregate functions are supported")
        if e.star:
            return len(rows)
        vals = [evaluate(e.args[0], self._env(table, i, params)) for i in rows]
        vals = [v for v in vals if v is not None]
        if e.distinct:
            uniq, seen = [], set()
            for v in vals:
                h = _hashable(v)
                if h not in seen:
                    seen.add(h)
                    uniq.append(v)
            vals = uniq
        if e.name == "count":
            return len(vals)
        if e.name == "collect":
            return vals
        if not vals:
            return None
        if e.name == "sum":
            return sum(vals)
        if e.name == "avg":
            return sum(vals) / len(vals)
        if e.name == "min":
            return min(vals, key=_sort_key)
        return max(vals, key=_sort_key)

    def _records(self, table: Table, names: List[str]) -> List[Record]:
        recs = []
        for i in range(table.n):
            recs.append(Record(names, [self._value(table, k, i) for k in names]))
        return recs


# --------------------------------------------------------------------- utils
def _split_and(e: A.Expr) -> List[A.Expr]:
    if isinstance(e, A.BinOp) and e.op == "and":
        return _split_and(e.left) + _split_and(e.right)
    return [e]


def _is_prop_of(e, var: str) -> bool:
    return isinstance(e, A.Prop) and isinstance(e.target, A.Var) and e.target.name == var


def _is_const(e) -> bool:
    if isinstance(e, (A.Literal, A.Param)):
        return True
    if isinstance(e, A.ListLit):
        return all(_is_const(x) for x in e.items)
    return False


def _cross(table: Table, name: str, ids: np.ndarray) -> Table:
    n, m = table.n, len(ids)
    rows = np.repeat(np.arange(n, dtype=np.int64), m)
    out = table.take(rows)
    out.add(name, np.tile(ids.astype(np.int64), n), NODE)
    return out


def _concat(a: Table, b: Table) -> Table:
    out = Table(a.n + b.n)
    for k in a.cols:
        ca, cb = a.cols[k], b.cols[k]
        if ca.dtype == object or cb.dtype == object:
            col = _obj_array(list(ca) + list(cb))
        else:
            col = np.concatenate([ca, cb])
        out.add(k, col, a.types[k])
    return out


def _hashable(v):
    if isinstance(v, list):
        return tuple(_hashable(x) for x in v)
    if isinstance(v, dict):
        return tuple(sorted((k, _hashable(x)) for k, x in v.items()))
    if isinstance(v, np.integer):
        return int(v)
    return v


def _sort_key(v):
    # Cypher orders: maps < nodes < rels < lists < paths < strings < booleans < numbers < null
    if v is None:
        return (9, 0)
    if isinstance(v, bool):
        return (7, v)
    if isinstance(v, (int, float)):
        return (8, v)
    if isinstance(v, str):
        return (6, v)
    if isinstance(v, (list, tuple)):
        return (4, tuple(_sort_key(x) for x in v))
    if isinstance(v, Node):
        return (2, v.id)
    if isinstance(v, Relationship):
        return (3, v.id)
    return (5, str(v))
