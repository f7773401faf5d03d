"""GraphBatcher (graph/batcher.py) on CPU with a fake device: concurrent
callers are coalesced into one call per (op, shape class) and each gets its
own slice back; a closed or dead batcher fails callers instead of hanging."""
import threading

import numpy as np
import pytest

from k8s_llm_rca_amd.graph.batcher import GraphBatcher


class FakeDev:
    """contains_many / state_lookup / walks with the DeviceGraph signatures."""

    def __init__(self, texts):
        self.texts = texts
        self.calls = {"contains": 0, "state": 0, "walks": 0}
        self.device = type("D", (), {"type": "cpu", "index": None})()

    def contains_many(self, rows, key, needles):
        self.calls["contains"] += 1
        return [np.array([n in self.texts[r] for r in rows]) for n in needles]

    def state_lookup(self, ents, ts, label, mode, tq, limit):
        self.calls["state"] += 1
        return [np.array([e * 10 + t], np.int64) for e, t in zip(ents, ts)]

    def walks(self, starts, min_h, max_h, direction, rel_types, end_label):
        self.calls["walks"] += 1
        # one record per start and hop count: [start row, hops, node...]
        recs = [[i, h, int(s)] + [0] * 9 for i, s in enumerate(starts) for h in range(min_h, max_h + 1)]
        return np.array(recs, np.int64).reshape(-1, 12)


def _run_threads(fn, n):
    out, errs = [None] * n, []

    def go(i):
        try:
            out[i] = fn(i)
        except BaseException as e:  # noqa: BLE001 - collected for the assert
            errs.append(e)
    ts = [threading.Thread(target=go, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert not errs, errs
    return out


def test_batched_contains_state_walks_match_direct():
    texts = ["secret db-creds not found", "nfs path missing", "quota exceeded", "pvc unbound"] * 8
    dev = FakeDev(texts)
    b = GraphBatcher(dev, window_s=0.02)
    rows = np.arange(len(texts))
    needles = ["secret", "nfs", "quota", "pvc", "missing", "none"]
    try:
        got = _run_threads(lambda i: b.contains(rows, "message", needles[i % len(needles)]), 12)
        for i, g in enumerate(got):
            assert np.array_equal(g, np.array([needles[i % len(needles)] in t for t in texts]))
        st = _run_threads(lambda i: b.state_lookup([i, i + 100], [1, 2], "STATE", "loose", None, 10), 8)
        for i, res in enumerate(st):
            assert [int(x[0]) for x in res] == [i * 10 + 1, (i + 100) * 10 + 2]
        wk = _run_threads(lambda i: b.walks([i, i + 50], 1, 2, "out", None, None), 8)
        for i, rec in enumerate(wk):
            assert rec.shape == (4, 12) and set(rec[:, 0]) == {0, 1}  # rows renumbered per caller
            assert sorted(rec[rec[:, 0] == 1][:, 2]) == [i + 50, i + 50]
        # coalescing: fewer device calls than requests
        assert b.stats["requests"] == 28 and b.stats["batches"] < 28
        assert dev.calls["contains"] < 12
    finally:
        b.close()


def test_closed_batcher_rejects_calls():
    b = GraphBatcher(FakeDev(["x"]), window_s=0.0)
    b.close()
    with pytest.raises(RuntimeError, match="closed"):
        b.contains(np.arange(1), "message", "x")


@pytest.mark.filterwarnings("ignore::pytest.PytestUnhandledThreadExceptionWarning")
def test_dead_batcher_fails_waiting_callers():
    class Broken(FakeDev):
        @property
        def device(self):
            raise SystemExit("boom")  # kills the worker thread at start-up

        @device.setter
        def device(self, v):
            pass

    b = GraphBatcher(Broken(["x"]), window_s=0.0)
    b._t.join(5)
    with pytest.raises(RuntimeError, match="died"):
        b.contains(np.arange(1), "message", "x")
