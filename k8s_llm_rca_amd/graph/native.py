"""Dispatch layer for the host-side graph operators.

The hot host operators (CSR build, filtered hop expansion, substring scan and
relationship-unique walk enumeration) live in the C++ extension
``k8s_llm_rca_amd/_graphcore*.so`` (source ``csrc/graph/graphcore.cpp``).
NumPy implementations of the same contracts are kept here as the oracle for
tests and as the fallback when the extension has not been built (CPU-only
containers that never ran ``__graft_entry__.build()``).
"""
from __future__ import annotations

from ..knobs import KNOBS
import importlib
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

_core = None
_tried = False


def core():
    """The compiled ``_graphcore`` module or None."""
    global _core, _tried
    if not _tried:
        _tried = True
        if not KNOBS.no_native:
            try:
                _core = importlib.import_module("k8s_llm_rca_amd._graphcore")
            except ImportError:
                _core = None
    return _core


def have_native() -> bool:
    return core() is not None


# --------------------------------------------------------------------- CSR
def build_csr_np(n: int, src: np.ndarray, dst: np.ndarray):
    order = np.argsort(src, kind="stable")
    counts = np.bincount(src, minlength=n) if len(src) else np.zeros(n, dtype=np.int64)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    return indptr, dst[order].astype(np.int64), order.astype(np.int64)


def build_csr(n: int, src: np.ndarray, dst: np.ndarray):
    c = core()
    if c is not None:
        return c.build_csr(int(n), np.ascontiguousarray(src, dtype=np.int64),
                           np.ascontiguousarray(dst, dtype=np.int64))
    return build_csr_np(n, src, dst)


# ------------------------------------------------------------------ expand
def expand_np(indptr, nbr, eid, ids, e_type, e_key, tids, kid):
    ids = np.asarray(ids, dtype=np.int64)
    starts = indptr[ids]
    ends = indptr[ids + 1]
    cnt = ends - starts
    total = int(cnt.sum())
    if total == 0:
        z = np.zeros(0, dtype=np.int64)
        return z, z, z
    row = np.repeat(np.arange(len(ids), dtype=np.int64), cnt)
    base = np.repeat(starts - np.concatenate(([0], np.cumsum(cnt)[:-1])), cnt)
    pos = base + np.arange(total, dtype=np.int64)
    e = eid[pos]
    nb = nbr[pos]
    m = np.ones(total, dtype=bool)
    if tids is not None:
        m &= np.isin(e_type[e], tids)
    if kid >= -1 and kid != -2:
        m &= e_key[e] == kid
    return row[m], e[m], nb[m]


def expand(indptr, nbr, eid, ids, e_type, e_key, tids, kid):
    c = core()
    if c is not None:
        t = np.zeros(0, dtype=np.int32) if tids is None else np.ascontiguousarray(tids, dtype=np.int32)
        return c.expand(indptr, nbr, eid, np.ascontiguousarray(ids, dtype=np.int64), e_type, e_key,
                        t, tids is not None, int(kid))
    return expand_np(indptr, nbr, eid, ids, e_type, e_key, tids, kid)


# ------------------------------------------------------------- substring
def substr_mask_np(offs: np.ndarray, buf: np.ndarray, ids: np.ndarray, needle: bytes) -> np.ndarray:
    out = np.zeros(len(ids), dtype=bool)
    raw = buf.tobytes()
    for j, n in enumerate(np.asarray(ids).tolist()):
        a, b = int(offs[n]), int(offs[n + 1])
        out[j] = raw.find(needle, a, b) >= 0 if (b - a) >= len(needle) else (len(needle) == 0)
    return out


def substr_mask(offs, buf, ids, needle: bytes) -> np.ndarray:
    c = core()
    if c is not None:
        return c.substr_mask(offs, buf, np.ascontiguousarray(ids, dtype=np.int64), needle)
    return substr_mask_np(offs, buf, ids, needle)


# ------------------------------------------------------ var-length walks
def var_length_np(g, starts, min_hops: int, max_hops: int, direction: str,
                  tids: Optional[np.ndarray]) -> List[Tuple[int, List[int], List[int]]]:
    results: List[Tuple[int, List[int], List[int]]] = []
    tset = None if tids is None else set(int(t) for t in tids)

    def nbrs(n):
        out = []
        if direction in ("out", "both"):
            a, b = g.out_indptr[n], g.out_indptr[n + 1]
            out.extend(zip(g.out_eid[a:b].tolist(), g.out_nbr[a:b].tolist()))
        if direction in ("in", "both"):
            a, b = g.in_indptr[n], g.in_indptr[n + 1]
            for e, m in zip(g.in_eid[a:b].tolist(), g.in_nbr[a:b].tolist()):
                if direction == "both" and g.e_src[e] == g.e_dst[e]:
                    continue
                out.append((e, m))
        if tset is not None:
            out = [(e, m) for e, m in out if int(g.e_type[e]) in tset]
        return out

    for row, s in enumerate(np.asarray(starts).tolist()):
        stack = [(s, [s], [])]
        while stack:
            n, nodes, edges = stack.pop()
            if min_hops <= len(edges) <= max_hops and len(edges) > 0:
                results.append((row, nodes, edges))
            elif len(edges) == 0 and min_hops == 0:
                results.append((row, nodes, edges))
            if len(edges) == max_hops:
                continue
            for e, m in reversed(nbrs(n)):
                if e in edges:
                    continue
                stack.append((m, nodes + [m], edges + [e]))
    return results


def var_length(g, starts, min_hops, max_hops, direction, tids):
    c = core()
    if c is not None:
        dcode = {"out": 0, "in": 1, "both": 2}[direction]
        t = np.zeros(0, dtype=np.int32) if tids is None else np.ascontiguousarray(tids, dtype=np.int32)
        rows, nodes_flat, edges_flat, hops = c.var_length(
            g.out_indptr, g.out_nbr, g.out_eid, g.in_indptr, g.in_nbr, g.in_eid,
            g.e_src, g.e_dst, g.e_type, np.ascontiguousarray(starts, dtype=np.int64),
            int(min_hops), int(max_hops), dcode, t, tids is not None)
        out = []
        npos = 0
        epos = 0
        for r, h in zip(rows.tolist(), hops.tolist()):
            out.append((r, nodes_flat[npos:npos + h + 1].tolist(), edges_flat[epos:epos + h].tolist()))
            npos += h + 1
            epos += h
        return out
    return var_length_np(g, starts, min_hops, max_hops, direction, tids)
