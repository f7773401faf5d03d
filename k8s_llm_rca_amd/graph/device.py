"""HBM mirror of a :class:`PropertyGraph` + dispatch to the HIP graph kernels.

The CSR arrays (int32 ids), edge type / key / validity-interval columns, node
labels and the packed ``message`` heap are uploaded once; the store then
routes large operator calls here (``min_gpu_rows``), small ones stay on the
host where a kernel launch + sync would cost more than the work:

* ``contains``    -> ``k8s_substr_search`` (multi-needle: :meth:`contains_many`)
* ``expand``      -> ``k8s_graph_expand2`` (count, device scan, fill)
* ``state_lookup``-> ``k8s_state_lookup``
* ``var_length``  -> ``k8s_walks`` (1..3 hops, relationship-unique, end-label pushdown)

Every op runs on the mirror's own HIP stream (non-blocking w.r.t. the LLM
engine's stream, so a graph query never queues behind a forward) and returns
its results through pinned host buffers with an async copy + event wait that
waits for this stream only.  :class:`..batcher.GraphBatcher` coalesces the
concurrent pipelines' calls into one launch per op.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from ..knobs import KNOBS
from ..ops._lib import check, lib, ptr, stream_ptr


class DeviceGraph:
    def __init__(self, g, device, min_gpu_rows: int = 2048):
        self.g = g
        self.device = torch.device(device)
        self.min_gpu_rows = min_gpu_rows

        def up32(a):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(self.device)

        def up64(a):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(self.device)

        if g.num_nodes >= 2 ** 31 or g.num_edges >= 2 ** 31:
            raise ValueError("device mirror uses int32 ids")
        self.oip, self.onb, self.oei = up32(g.out_indptr), up32(g.out_nbr), up32(g.out_eid)
        self.iip, self.inb, self.iei = up32(g.in_indptr), up32(g.in_nbr), up32(g.in_eid)
        self.esrc, self.edst = up32(g.e_src), up32(g.e_dst)
        self.etype, self.ekey = up32(g.e_type), up32(g.e_key)
        self.tmin, self.tmax = up64(g.e_tmin), up64(g.e_tmax)
        self.nlabel = up32(g.node_label)
        self._heaps = {}
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.batcher = None  # graph/batcher.py, attached by enable_batching()
        self.launches = 0
        self.bytes = sum(t.numel() * t.element_size() for t in (
            self.oip, self.onb, self.oei, self.iip, self.inb, self.iei, self.esrc, self.edst, self.etype,
            self.ekey, self.tmin, self.tmax, self.nlabel))

    def _ctx(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _up(self, a, dtype) -> torch.Tensor:
        """Pinned host staging + async upload on the graph stream."""
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=dtype))
        if self.device.type == "cuda":
            t = t.pin_memory()
        return t.to(self.device, non_blocking=True)

    def _fetch(self, *ts: torch.Tensor):
        """Device -> pinned host copies of ``ts``; waits for THIS stream only."""
        if self.device.type != "cuda":
            return [t.numpy() for t in ts]
        hs = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in ts]
        for h, t in zip(hs, ts):
            h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event(blocking=KNOBS.blocking_sync)
        ev.record(self.stream)
        ev.synchronize()
        return [h.numpy() for h in hs]

    def _heap(self, key: str):
        h = self._heaps.get(key)
        if h is None:
            offs, buf = self.g.string_heap(key)
            with self._ctx():  # uploaded on the mirror's stream, read there (never the engine's)
                h = (self._up(offs, offs.dtype), self._up(buf if len(buf) else np.zeros(1, np.uint8), np.uint8))
                (_,) = self._fetch(h[0][:1])  # the heap is resident before the first kernel reads it
            self.bytes += h[0].numel() * 8 + h[1].numel()
            self._heaps[key] = h
        return h

    def _type_mask(self, rel_types: Optional[Sequence[str]]) -> int:
        if not rel_types:
            return -1  # 0xFFFFFFFF
        m = 0
        for t in rel_types:
            tid = self.g.rel_types.lookup(t)
            if tid >= 0:
                if tid >= 31:
                    return -1
                m |= 1 << tid
        return m

    # ------------------------------------------------------------ CONTAINS
    def contains_many(self, ids: np.ndarray, key: str, needles: List[str]) -> np.ndarray:
        """[len(needles), len(ids)] bool: node[key] CONTAINS needle (one launch)."""
        offs, heap = self._heap(key)
        enc = [n.encode("utf-8") for n in needles]
        noff = np.zeros(len(enc) + 1, dtype=np.int32)
        np.cumsum([len(e) for e in enc], out=noff[1:])
        nbuf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
        with self._ctx():
            d_ids = self._up(ids, np.int64)
            d_nd = self._up(nbuf, np.uint8)
            d_noff = self._up(noff, np.int32)
            out = torch.empty(len(needles) * len(ids), dtype=torch.uint8, device=self.device)
            check(lib().k8s_substr_search(ptr(offs), ptr(heap), ptr(d_ids), len(ids), ptr(d_nd), len(needles),
                                          ptr(d_noff), ptr(out), stream_ptr(d_ids)), "substr_search")
            self.launches += 1
            (o,) = self._fetch(out)
        return o.reshape(len(needles), len(ids)).astype(bool)

    def contains(self, ids: np.ndarray, key: str, needle: str) -> np.ndarray:
        return self.contains_many(ids, key, [needle])[0]

    # -------------------------------------------------------------- expand
    def expand(self, ids: np.ndarray, direction: str, rel_types, key: Optional[str]):
        kid = -2 if key is None else self.g.keys.lookup(key)
        tm = self._type_mask(rel_types)
        outs = []
        n = len(ids)
        # on the mirror's stream like every other op: on the caller's (default) stream
        # the count read-back waited for the LLM engine's queued forward, and the
        # engine's next kernels queued behind these
        with self._ctx():
            d_ids = self._up(ids, np.int64)
            for side in (("out",) if direction == "out" else ("in",) if direction == "in" else ("out", "in")):
                ip, nb, ei = (self.oip, self.onb, self.oei) if side == "out" else (self.iip, self.inb, self.iei)
                skip = 1 if (direction == "both" and side == "in") else 0
                counts = torch.empty(n, dtype=torch.int32, device=self.device)
                check(lib().k8s_graph_expand2(ptr(ip), ptr(nb), ptr(ei), ptr(self.etype), ptr(self.ekey),
                                              ptr(self.esrc), ptr(self.edst), ptr(d_ids), n, tm, kid, skip,
                                              ptr(counts), 0, 0, 0, 0, stream_ptr(d_ids)), "graph_expand")
                offsets = torch.zeros(n + 1, dtype=torch.int64, device=self.device)
                torch.cumsum(counts, 0, out=offsets[1:])
                (tot,) = self._fetch(offsets[-1:])
                total = int(tot[0])
                o = [torch.empty(max(total, 1), dtype=torch.int64, device=self.device) for _ in range(3)]
                check(lib().k8s_graph_expand2(ptr(ip), ptr(nb), ptr(ei), ptr(self.etype), ptr(self.ekey),
                                              ptr(self.esrc), ptr(self.edst), ptr(d_ids), n, tm, kid, skip,
                                              ptr(counts), ptr(offsets), ptr(o[0]), ptr(o[1]), ptr(o[2]),
                                              stream_ptr(d_ids)), "graph_expand")
                self.launches += 2
                outs.append(tuple(self._fetch(*[t[:total] for t in o])))
        if len(outs) == 1:
            return outs[0]
        row = np.concatenate([x[0] for x in outs])
        order = np.argsort(row, kind="stable")
        return row[order], np.concatenate([x[1] for x in outs])[order], np.concatenate([x[2] for x in outs])[order]

    # -------------------------------------------------------- STATE lookup
    def state_lookup(self, entity_ids, ts_ms, state_label, mode, tmax_ms, limit):
        n = len(entity_ids)
        lid = -1 if state_label is None else self.g.labels.lookup(state_label)
        if state_label is not None and lid < 0:
            return [np.zeros(0, dtype=np.int64) for _ in range(n)]
        with self._ctx():
            d_e = self._up(entity_ids, np.int64)
            d_t = self._up(ts_ms, np.int64)
            d_q = self._up(tmax_ms if tmax_ms is not None else ts_ms, np.int64)
            out = torch.full((n * limit,), -1, dtype=torch.int64, device=self.device)
            counts = torch.empty(n, dtype=torch.int32, device=self.device)
            check(lib().k8s_state_lookup(ptr(self.oip), ptr(self.onb), ptr(self.oei), ptr(self.etype),
                                         ptr(self.nlabel), ptr(self.tmin), ptr(self.tmax),
                                         self.g.rel_types.lookup("HasState"), lid, 1 if mode != "strict" else 0,
                                         limit, ptr(d_e), ptr(d_t), ptr(d_q), n, ptr(out), ptr(counts),
                                         stream_ptr(d_e)), "state_lookup")
            self.launches += 1
            o, c = self._fetch(out, counts)
        o = o.reshape(n, limit)
        return [o[i, :c[i]] for i in range(n)]

    # ------------------------------------------------------------- walks
    def walks(self, starts: np.ndarray, min_h: int, max_h: int, direction: str,
              rel_types=None, end_label: Optional[str] = None) -> np.ndarray:
        """Records [W, 9] int32: row, hops, n0..n3, e0..e2 (-1 padded), in the
        host enumeration's order.  Starts whose frontier overflows the
        kernel's LDS (hubs) are enumerated on the host instead."""
        n = len(starts)
        dcode = {"out": 0, "in": 1, "both": 2}[direction]
        el = -1 if end_label is None else self.g.labels.lookup(end_label)
        if end_label is not None and el < 0:
            return np.zeros((0, 9), dtype=np.int32)
        tm = self._type_mask(rel_types)
        with self._ctx():
            d_s = self._up(starts, np.int64)
            counts = torch.empty(n, dtype=torch.int32, device=self.device)
            args = [ptr(self.oip), ptr(self.onb), ptr(self.oei), ptr(self.iip), ptr(self.inb), ptr(self.iei),
                    ptr(self.esrc), ptr(self.edst), ptr(self.etype), ptr(self.nlabel), ptr(d_s), n, min_h, max_h,
                    dcode, tm, el]
            check(lib().k8s_walks(*args, ptr(counts), 0, 0, stream_ptr(d_s)), "walks")
            offsets = torch.zeros(n + 1, dtype=torch.int64, device=self.device)
            torch.cumsum(counts.clamp(min=0), 0, out=offsets[1:])
            (tot, c_host) = self._fetch(offsets[-1:], counts)
            total = int(tot[0])
            out = torch.empty(max(total, 1) * 12, dtype=torch.int32, device=self.device)
            check(lib().k8s_walks(*args, ptr(counts), ptr(offsets), ptr(out), stream_ptr(d_s)), "walks")
            self.launches += 2
            (rec,) = self._fetch(out[: total * 12])
        rec = rec.reshape(total, 12)
        over = np.nonzero(c_host < 0)[0]
        if len(over):  # hubs: the host path, merged back in enumeration order
            extra = []
            tids = None
            if rel_types:
                tids = np.asarray([self.g.rel_types.lookup(t) for t in rel_types], dtype=np.int32)
            from . import native as _native
            for j in over.tolist():
                for _, nodes, edges in _native.var_length(self.g, np.asarray([starts[j]]), min_h, max_h, direction,
                                                           tids):
                    if el >= 0 and self.g.node_label[nodes[-1]] != el:
                        continue
                    h = len(edges)
                    r = [j, h] + list(nodes) + [-1] * (4 - len(nodes)) + list(edges) + [-1] * (3 - h)
                    extra.append(r + [len(extra), -1, -1])  # k: host order within the start
            if extra:
                rec = np.concatenate([rec, np.asarray(extra, dtype=np.int32)])
        order = np.lexsort((rec[:, 11], rec[:, 10], rec[:, 9], rec[:, 0]))
        return np.ascontiguousarray(rec[order, :9])


def to_device(g, device, min_gpu_rows: int = 2048) -> DeviceGraph:
    g.device = DeviceGraph(g, device, min_gpu_rows)
    return g.device
