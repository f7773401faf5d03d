"""Cross-pipeline batching of graph queries onto the HBM mirror (G3 / G4 / G6).

With 128 concurrent RCA pipelines (one thread each) the graph queries arrive
as a steady trickle of tiny, independent operator calls: a ``CONTAINS`` scan of
every EVENT message per ``find_srcKind`` (``find_srckind_metapath_neo4j.py:75-90``),
a temporal STATE lookup per entity of every statepath (``analyze_root_cause.py:
70-79``), the var-length metapath cascade (``:95-150``).  Run one by one, each
is a kernel launch plus a round trip -- or host work under the GIL.  The
batcher collects whatever calls are pending across all pipeline threads and
runs them as ONE kernel per (op, shape class):

* ``contains``  -> one multi-needle ``substr_kernel`` launch for every pending
  needle over the same row set (all EVENT nodes);
* ``state``     -> one ``state_kernel`` launch over the concatenated entities;
* ``walks``     -> one ``walks_kernel`` count + fill over the concatenated starts.

Callers block on a future (GIL released); the batcher thread issues on the
mirror's own stream and fetches through pinned buffers, so neither the LLM
engine's stream nor its thread ever waits for a graph query.
"""
from __future__ import annotations

import threading
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np


class _Req:
    __slots__ = ("op", "key", "args", "done", "result", "error")

    def __init__(self, op: str, key: Tuple, args: Tuple):
        self.op, self.key, self.args = op, key, args
        self.done = threading.Event()
        self.result = None
        self.error: Optional[BaseException] = None


class GraphBatcher:
    def __init__(self, dev, window_s: float = 200e-6):
        self.dev = dev
        self.window_s = window_s
        self._q: List[_Req] = []
        self._cv = threading.Condition()
        self._stop = False
        self._dead: Optional[BaseException] = None
        self.stats: Dict[str, float] = {"requests": 0, "batches": 0, "launches": 0, "busy_s": 0.0, "max_batch": 0}
        self._t = threading.Thread(target=self._loop, name="graph-batcher", daemon=True)
        self._t.start()

    # ------------------------------------------------------------- callers
    def _call(self, op: str, key: Tuple, args: Tuple) -> Any:
        r = _Req(op, key, args)
        with self._cv:
            if self._dead is not None:
                raise RuntimeError(f"graph batcher thread died: {self._dead!r}")
            if self._stop:  # the worker drains what is queued, then exits: nothing would serve this
                raise RuntimeError("graph batcher is closed")
            self._q.append(r)
            self._cv.notify()
        r.done.wait()
        if r.error is not None:
            raise r.error
        return r.result

    def contains(self, ids: np.ndarray, key: str, needle: str) -> np.ndarray:
        return self._call("contains", (key,), (np.asarray(ids, np.int64), needle))

    def state_lookup(self, entity_ids, ts_ms, state_label, mode, tmax_ms, limit) -> List[np.ndarray]:
        return self._call("state", (state_label, mode, limit),
                          (np.asarray(entity_ids, np.int64), np.asarray(ts_ms, np.int64),
                           None if tmax_ms is None else np.asarray(tmax_ms, np.int64)))

    def walks(self, starts, min_h, max_h, direction, rel_types, end_label) -> np.ndarray:
        return self._call("walks", (min_h, max_h, direction, tuple(rel_types or ()), end_label),
                          (np.asarray(starts, np.int64),))

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()

    # -------------------------------------------------------------- worker
    def _loop(self) -> None:
        try:
            import torch
            if self.dev.device.type == "cuda" and self.dev.device.index is not None:
                torch.cuda.set_device(self.dev.device)
            self._serve()
        except BaseException as e:  # noqa: BLE001 - never leave a caller waiting on a dead thread
            with self._cv:
                self._dead = e
                pending, self._q = self._q, []
            for r in pending:
                r.error = e
                r.done.set()
            raise

    def _serve(self) -> None:
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait(0.1)
                if self._stop and not self._q:
                    return
            time.sleep(self.window_s)  # let the other pipelines' calls of this tick arrive
            with self._cv:
                batch, self._q = self._q, []
            t0 = time.perf_counter()
            groups: Dict[Tuple, List[_Req]] = {}
            for r in batch:
                groups.setdefault((r.op,) + r.key, []).append(r)
            for (op, *_), reqs in groups.items():
                try:
                    getattr(self, "_run_" + op)(reqs)
                except BaseException as e:  # noqa: BLE001 - surfaces in every waiting caller
                    for r in reqs:
                        r.error = e
                for r in reqs:
                    r.done.set()
            self.stats["requests"] += len(batch)
            self.stats["batches"] += 1
            self.stats["launches"] += len(groups)
            self.stats["max_batch"] = max(self.stats["max_batch"], len(batch))
            self.stats["busy_s"] += time.perf_counter() - t0

    def _run_contains(self, reqs: List[_Req]) -> None:
        """Every pending needle against the union of the requests' rows (in
        the pipeline the row set is the same for all: every EVENT node)."""
        key = reqs[0].key[0]
        first = reqs[0].args[0]
        same = all(r.args[0] is first or np.array_equal(r.args[0], first) for r in reqs[1:])
        rows = first if same else np.unique(np.concatenate([r.args[0] for r in reqs]))
        needles = list(dict.fromkeys(r.args[1] for r in reqs))
        res = self.dev.contains_many(rows, key, needles)
        row = {n: i for i, n in enumerate(needles)}
        for r in reqs:
            hit = res[row[r.args[1]]]
            r.result = hit if same else hit[np.searchsorted(rows, r.args[0])]

    def _run_state(self, reqs: List[_Req]) -> None:
        state_label, mode, limit = reqs[0].key
        ents = np.concatenate([r.args[0] for r in reqs])
        ts = np.concatenate([r.args[1] for r in reqs])
        tq = None
        if mode != "strict":
            tq = np.concatenate([r.args[2] if r.args[2] is not None else r.args[1] for r in reqs])
        out = self.dev.state_lookup(ents, ts, state_label, mode, tq, limit)
        o = 0
        for r in reqs:
            n = len(r.args[0])
            r.result = out[o:o + n]
            o += n

    def _run_walks(self, reqs: List[_Req]) -> None:
        min_h, max_h, direction, rel_types, end_label = reqs[0].key
        starts = np.concatenate([r.args[0] for r in reqs])
        rec = self.dev.walks(starts, min_h, max_h, direction, list(rel_types) or None, end_label)
        o = 0
        rows = rec[:, 0] if len(rec) else np.zeros(0, np.int32)
        for r in reqs:
            n = len(r.args[0])
            lo, hi = np.searchsorted(rows, o), np.searchsorted(rows, o + n)
            part = rec[lo:hi].copy()
            part[:, 0] -= o
            r.result = part
            o += n


def enable_batching(g, window_s: float = 200e-6) -> GraphBatcher:
    """Route ``g``'s device-mirrored operators through one batcher thread
    (``g.device`` must be a :class:`..device.DeviceGraph`)."""
    dev = g.device
    if dev.batcher is None:
        dev.batcher = GraphBatcher(dev, window_s)
    return dev.batcher
