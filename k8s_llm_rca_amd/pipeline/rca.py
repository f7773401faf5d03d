"""End-to-end RCA driver: the equivalent of ``test_all.py`` / ``test_with_file.py``.

:class:`RCAPipeline` owns the three assistants (locator, cypher generator,
semantic analyzer) and two graph executors, and :meth:`RCAPipeline.analyze`
runs one incident through locate -> generate_query -> analyze with the
reference's repair loops (``test_with_file.py:77-155``):

* locator: up to ``max_attempts`` runs; JSON / other errors are fed back to
  the same thread (``:78-97``);
* cypher: up to ``max_attempts`` runs per metapath; ``CypherSyntaxError`` /
  other errors fed back (``:118-141``);
* deterministic template fallback when the last attempt was used or no record
  survived filtering (``:149-155``).

The result dict has the reference's keys in the reference's order
(``error_message, locator_attempts, analysis[extend_metapath, cypher_query,
cypher_attempts, human_cypher_query?, statepath[report, clue]], time_cost,
token_usage``) and is appended to the output as pretty JSON + ``\\n``
(``:202-204``).

:func:`run_batch` is the multi-incident form: ``concurrency`` worker threads,
each with its own pipeline (its own three threads, as if that many reference
drivers ran side by side) feeding one shared engine, which batches every
active run into the same GPU steps.

Reference quirks are reproduced only behind :class:`Compat` flags:
``shared_statepath_dict`` (every statepath entry aliases one dict,
``test_with_file.py:158``), ``int_token_window`` (``int()`` of the window
bounds, ``:179-180``) and ``fallback_after_last_attempt`` (fallback even when
the last attempt succeeded, ``:149``; on by default -- it is observable in the
output's ``human_cypher_query`` key).
"""
from __future__ import annotations

import csv
import json
import logging
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..graph.model import CypherSyntaxError
from ..utils import tracing
from . import check_state as CS
from . import find_metapath as FM
from . import formats as F
from . import generate_query as GQ
from . import prompts

log = logging.getLogger(__name__)


@dataclass
class Compat:
    shared_statepath_dict: bool = False
    int_token_window: bool = False
    fallback_after_last_attempt: bool = True


@dataclass
class RCAConfig:
    model: str = "llama3-8b"
    max_attempts: int = 3
    constrained: bool = True     # hand the engine a grammar per stage
    hints: bool = False          # oracle hints from the incident ground truth
    budget: F.GenerationBudget = field(default_factory=F.GenerationBudget)
    compat: Compat = field(default_factory=Compat)
    # token-usage `limit`s per assistant (test_with_file.py:182-188)
    usage_limits: tuple = (10, 20, 30)


class RCAPipeline:
    def __init__(self, service, metagraph_qe, stategraph_qe, config: Optional[RCAConfig] = None):
        self.service = service
        self.meta = metagraph_qe
        self.state = stategraph_qe
        self.cfg = config or RCAConfig()
        m = self.cfg.model
        self.locator = FM.setup_root_cause_locator(service, m)
        self.native, self.external = FM.find_native_external_kinds(self.meta)
        self.prompt_template = FM.build_prompt_template(self.native, self.external)
        self.generator = GQ.setup_cypher_generator(service, m)
        self.analyzer = CS.setup_state_semantic_analyzer(service, m)
        self.last_failed_runs = 0  # LLM runs of the last analyze() that failed / expired / were cancelled
        self.n_analyses = 0  # incidents this pipeline's three threads have carried (thread age)

    # ------------------------------------------------------------ formats
    def _locator_fmt(self, src: str, truth) -> Any:
        if not self.cfg.constrained:
            return None
        t = (truth.src_kind, truth.dest_kind, truth.path_kinds) if (truth is not None and self.cfg.hints) else None
        return F.locator_grammar(self.native + self.external, src, self.cfg.budget, t)

    def _cypher_fmt(self, mp: str, msg: str) -> Any:
        return F.cypher_grammar(mp, msg, hint=self.cfg.hints) if self.cfg.constrained else None

    def _semantic_fmt(self) -> Any:
        return F.semantic_grammar(self.cfg.budget) if self.cfg.constrained else None

    def _summary_fmt_fn(self, truth) -> Optional[Callable]:
        if not self.cfg.constrained:
            return None
        dest = truth.dest_kind if (truth is not None and self.cfg.hints) else None
        return lambda kinds: F.summary_grammar(kinds, self.cfg.budget, dest)

    # -------------------------------------------------------------- analyze
    def analyze(self, errorMessage: str, truth=None) -> Dict[str, Any]:
        t0 = time.time()
        result: Dict[str, Any] = {"error_message": errorMessage}
        with tracing.span("rca.locate"):
            src = FM.find_srcKind(self.state, errorMessage)
            dest_relevant = None
            attempt = 0
            for attempt in range(self.cfg.max_attempts):
                try:
                    dest_relevant = FM.find_destKind_relevantResources(
                        errorMessage, src, self.prompt_template, self.locator,
                        response_format=self._locator_fmt(src, truth))
                    break
                except json.JSONDecodeError as e:
                    self.locator.add_message(prompts.locator_json_error(str(e)))
                except Exception as e:  # noqa: BLE001 - mirrors the reference's catch-all
                    self.locator.add_message(prompts.locator_other_error(str(e)))
            result["locator_attempts"] = attempt + 1
            result["analysis"] = []
            metapaths = []
            if isinstance(dest_relevant, dict):
                try:
                    dest = dest_relevant["DestinationKind"]
                    relevant = dest_relevant.get("RelevantResources") or []
                    inter = FM.intermediate_kinds(relevant, src, dest, self.native, self.external)
                    metapaths = FM.find_metapath(self.meta, src, dest, inter)
                except (KeyError, ValueError, TypeError) as e:
                    log.warning("no metapath for %r: %s", errorMessage[:60], e)
                    result["locate_error"] = repr(e)
        shared_sp: Dict[str, Any] = {}
        for mp in metapaths:
            with tracing.span("rca.query"):
                ext = GQ.extend_metapath_construct_string(mp)
                analysis: Dict[str, Any] = {"extend_metapath": ext}
                records: list = []
                cypher = None
                attempt = 0
                for attempt in range(self.cfg.max_attempts):
                    try:
                        cypher = GQ.generate_cypher_query(ext, errorMessage, self.generator,
                                                          response_format=self._cypher_fmt(ext, errorMessage))
                        records = GQ.run_and_filter_query(self.state, cypher)
                        break
                    except CypherSyntaxError as e:
                        self.generator.add_message(prompts.cypher_syntax_error(str(e)))
                    except Exception as e:  # noqa: BLE001
                        self.generator.add_message(prompts.cypher_other_error(str(e)))
                analysis["cypher_query"] = cypher
                analysis["cypher_attempts"] = attempt + 1
                last = attempt == self.cfg.max_attempts - 1
                if (last and self.cfg.compat.fallback_after_last_attempt) or not records:
                    try:
                        human = GQ.human_generate_cypher_query(ext, errorMessage)
                        records = GQ.run_and_filter_query(self.state, human)
                        analysis["human_cypher_query"] = human
                    except Exception as e:  # noqa: BLE001
                        analysis["human_cypher_query_error"] = repr(e)
                        records = []
            with tracing.span("rca.analyze"):
                analysis["statepath"] = []
                for rec in records:
                    report, clues = CS.check_statepath(self.state, self.analyzer, rec,
                                                       semantic_format=self._semantic_fmt(),
                                                       summary_format_fn=self._summary_fmt_fn(truth))
                    sp = shared_sp if self.cfg.compat.shared_statepath_dict else {}
                    sp["report"] = report
                    sp["clue"] = clues
                    analysis["statepath"].append(sp)
            result["analysis"].append(analysis)
        t1 = time.time()
        self.n_analyses += 1
        self.last_failed_runs = sum(
            1 for a in (self.locator, self.generator, self.analyzer)
            for run in self.service.list_runs(a.thread.id, limit=64)
            if run.created_at >= t0 and run.status in ("failed", "cancelled", "expired"))
        result["time_cost"] = t1 - t0
        tmin, tmax = (int(t0), int(t1)) if self.cfg.compat.int_token_window else (t0, t1 + 1e-6)
        usage = {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0}
        for a, lim in zip((self.locator, self.generator, self.analyzer), self.cfg.usage_limits):
            u = a.get_token_usage(tmin, tmax, lim)
            for k in usage:
                usage[k] += u[k]
        result["token_usage"] = usage
        return result


def read_messages_csv(path: str) -> List[str]:
    """Column 0 of a CSV, header skipped (test_with_file.py:45-53)."""
    with open(path, newline="") as f:
        r = csv.reader(f)
        next(r, None)
        return [row[0] for row in r if row]


def append_result(path: str, result: Dict[str, Any]) -> None:
    with open(path, "a") as f:
        f.write(json.dumps(result, indent=4) + "\n")


def read_results(path: str) -> List[Dict[str, Any]]:
    """Parse the concatenated pretty-JSON stream written by :func:`append_result`."""
    dec = json.JSONDecoder()
    txt = open(path).read()
    out, i = [], 0
    while True:
        while i < len(txt) and txt[i].isspace():
            i += 1
        if i >= len(txt):
            return out
        obj, i = dec.raw_decode(txt, i)
        out.append(obj)


@dataclass
class BatchStats:
    results: List[Dict[str, Any]]
    latencies: List[float]
    wall_s: float
    errors: List[str]

    @property
    def n_ok(self) -> int:
        """Analyses that completed; an incident that raised is in ``results`` as
        an ``{"error": ...}`` record (the batch output keeps one line per input)
        but is not throughput."""
        return sum(1 for r in self.results if "error" not in r)

    @property
    def analyses_per_s(self) -> float:
        return self.n_ok / self.wall_s if self.wall_s > 0 else 0.0

    def pct(self, q: float) -> float:
        if not self.latencies:
            return 0.0
        s = sorted(self.latencies)
        k = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
        return s[k]


def run_batch(make_pipeline: Callable[[], RCAPipeline], messages: List[str], concurrency: int = 1,
              truths: Optional[List[Any]] = None, output_path: Optional[str] = None,
              pipelines: Optional[List[RCAPipeline]] = None) -> BatchStats:
    """Analyze ``messages`` with ``concurrency`` concurrent pipelines."""
    work: "queue.Queue" = queue.Queue()
    for i, m in enumerate(messages):
        work.put((i, m))
    results: List[Optional[Dict[str, Any]]] = [None] * len(messages)
    lat: List[float] = [0.0] * len(messages)
    errors: List[str] = []
    out_lock = threading.Lock()
    if pipelines is None:
        pipelines = [make_pipeline() for _ in range(max(1, concurrency))]

    def worker(p: RCAPipeline):
        while True:
            try:
                i, m = work.get_nowait()
            except queue.Empty:
                return
            t = time.perf_counter()
            try:
                r = p.analyze(m, truths[i] if truths else None)
            except Exception as e:  # noqa: BLE001 - one bad incident must not stop the batch
                log.exception("incident %d failed", i)
                r = {"error_message": m, "error": repr(e)}
                with out_lock:
                    errors.append(repr(e))
            lat[i] = time.perf_counter() - t
            results[i] = r
            if output_path:
                with out_lock:
                    append_result(output_path, r)

    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(p,), daemon=True) for p in pipelines]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    wall = time.perf_counter() - t0
    return BatchStats([r for r in results if r is not None], lat, wall, errors)


class IncidentStream:
    """Steady-state multi-incident driver: one worker thread per pipeline pulls
    the next incident from a cyclic source the moment it finishes one, so the
    engine always sees ``len(pipelines)`` concurrent analyses (the CLI's
    ``run --concurrency`` as an unbounded stream).  Every completion is
    timestamped, so a caller can time a window of N completed analyses
    (``bench/rca_bench.py``'s steps) without draining the stream.

    An analysis counts as completed only if it raised nothing and none of its
    LLM runs failed, expired or was cancelled (an engine fault that fails every
    in-flight run must not show up as fast throughput)."""

    def __init__(self, pipelines: List[RCAPipeline], incidents: List[Any], hints: bool = True):
        self.pipelines = pipelines
        self.incidents = incidents
        self.hints = hints
        self._cv = threading.Condition()
        self._next = 0
        self._stop = False
        self.done: List[tuple] = []   # (t_done, latency_s, ok, stage3, fault) in completion order
        self.n_ok = 0
        self.n_err = 0
        self.n_abandoned = 0
        self.errors: List[str] = []
        self._threads: List[threading.Thread] = []
        self.ok_by_pipeline: List[int] = [0] * len(pipelines)  # successful stream analyses per pipeline

    def pre_age(self, n: int, workers: int = 8) -> None:
        """Drive every pipeline through ``n`` incidents of the stream's source
        before :meth:`start` (the stream then continues with the incidents
        after them), so its threads carry ``n`` incidents of history -- the
        reference's regime, where one driver pushes every incident of its CSV
        through the same three threads (``test_with_file.py:28-38,64``).  The
        caller puts the backend in replay mode first (``EngineBackend.set_replay``)."""
        jobs: "queue.Queue" = queue.Queue()
        for p in self.pipelines:
            jobs.put(p)
        errs: List[BaseException] = []

        def work():
            while True:
                try:
                    p = jobs.get_nowait()
                except queue.Empty:
                    return
                for _ in range(n):
                    with self._cv:
                        i = self._next
                        self._next += 1
                    inc = self.incidents[i % len(self.incidents)]
                    try:
                        p.analyze(inc.message, inc if self.hints else None)
                    except BaseException as e:  # noqa: BLE001 - re-raised below
                        errs.append(e)
                        return

        ths = [threading.Thread(target=work, daemon=True, name="rca-preage") for _ in range(max(1, workers))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]

    def start(self) -> None:
        for j, p in enumerate(self.pipelines):
            t = threading.Thread(target=self._worker, args=(p, j), daemon=True, name="rca-stream")
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        """Stop admitting incidents (in-flight analyses finish or are abandoned)."""
        with self._cv:
            self._stop = True
            self._cv.notify_all()

    def join(self, timeout: float) -> bool:
        """Wait for the workers to exit (after :meth:`stop`); True if all did."""
        end = time.perf_counter() + timeout
        for t in self._threads:
            t.join(max(0.0, end - time.perf_counter()))
        return not any(t.is_alive() for t in self._threads)

    def _worker(self, p: RCAPipeline, j: int) -> None:
        while True:
            with self._cv:
                if self._stop:
                    return
                i = self._next
                self._next += 1
            inc = self.incidents[i % len(self.incidents)]
            t = time.perf_counter()
            ok, err, stage3 = True, None, False
            try:
                r = p.analyze(inc.message, inc if self.hints else None)
                # reached stage 3: some metapath's query left a statepath to analyze
                stage3 = any(a.get("statepath") for a in r.get("analysis", []))
                if p.last_failed_runs:
                    ok, err = False, f"{p.last_failed_runs} LLM run(s) failed: {r.get('error_message', '')[:60]!r}"
            except Exception as e:  # noqa: BLE001 - counted, never fatal to the stream
                if not self._stop:  # after stop() the service is closing under the analysis
                    log.exception("incident %d failed", i)
                ok, err = False, repr(e)
            t1 = time.perf_counter()
            with self._cv:
                if self._stop and not ok:  # cut short by the shutdown (service closed), not a failure
                    self.n_abandoned += 1
                    return
                self.done.append((t1, t1 - t, ok, stage3, getattr(inc, "fault", "")))
                if ok:
                    self.n_ok += 1
                    self.ok_by_pipeline[j] += 1
                else:
                    self.n_err += 1
                    self.errors.append(err)
                self._cv.notify_all()

    def wait_ok(self, n: int, deadline: Optional[float] = None, poll: Optional[Callable[[], None]] = None) -> bool:
        """Block until ``n`` analyses completed successfully (False at ``deadline``,
        a ``time.perf_counter()`` value).  ``poll`` runs every ~0.5 s (e.g. to
        re-raise an engine fault)."""
        with self._cv:
            while self.n_ok < n:
                if deadline is not None and time.perf_counter() >= deadline:
                    return False
                self._cv.wait(0.5)
                if poll is not None:
                    poll()
            return True

    def wait_each(self, n_each: int, deadline: Optional[float] = None,
                  poll: Optional[Callable[[], None]] = None) -> bool:
        """Block until every pipeline has completed ``n_each`` analyses of the
        stream (False at ``deadline``)."""
        with self._cv:
            while min(self.ok_by_pipeline, default=n_each) < n_each:
                if deadline is not None and time.perf_counter() >= deadline:
                    return False
                self._cv.wait(0.5)
                if poll is not None:
                    poll()
            return True

    def window(self, t0: float, t1: float) -> List[float]:
        """Latencies of the successful analyses completed in ``[t0, t1)``."""
        with self._cv:
            return [lat for t, lat, ok, *_ in self.done if ok and t0 <= t < t1]

    def stage3(self, t0: float, t1: float) -> Dict[str, Any]:
        """Of the successful analyses completed in ``[t0, t1)``: the fraction
        that reached stage 3 (analyze_root_cause ran on at least one statepath),
        and ``{fault: [reached, total]}``."""
        by: Dict[str, List[int]] = {}
        with self._cv:
            rows = [(s3, f) for t, _, ok, s3, f in self.done if ok and t0 <= t < t1]
        for s3, f in rows:
            c = by.setdefault(f or "?", [0, 0])
            c[0] += int(s3)
            c[1] += 1
        n = len(rows)
        return {"fraction": round(sum(int(s3) for s3, _ in rows) / n, 4) if n else 0.0,
                "by_fault": dict(sorted(by.items()))}
