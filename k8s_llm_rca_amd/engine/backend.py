"""Assistant-service backend that executes runs on the :class:`LLMEngine`.

Each service thread maps to one engine sequence.  The thread's token list is
kept as per-message segments in the chat template::

    <|begin_of_text|> system(instructions) user(m1) user(m2) assistant(reply) ...
    <|start_header_id|>assistant<|end_header_id|>\\n\\n          <- generation prompt

Assistant replies keep their *generated* token ids (not a re-encoding of the
text), so the next run's prompt shares the whole cached prefix and only the
new messages are prefilled.  When a thread would overflow the model context,
the oldest non-seed messages are dropped (the system prompt and the first
``keep_seed`` messages -- the reference's seeding messages -- are kept) and
the engine's longest-common-prefix logic re-prefills from the first change.
Truncation has hysteresis: an overflowing thread drops old turns down to
``trunc_low`` of its window and that cut point is sticky, so the next runs
append to a stable prefix (one re-prefill per ~half window of new history
instead of one per run once a thread sits at the window edge).
"""
from __future__ import annotations

import logging
import threading
from typing import Dict, List, Optional

from ..api.service import Backend, RunState, ThreadState
from .engine import LLMEngine

log = logging.getLogger(__name__)


class _ThreadTokens:
    __slots__ = ("sid", "sys_text", "sys_ids", "segments", "lock", "dropped", "prompt_len", "truncations")

    def __init__(self, sid: int):
        self.sid = sid
        self.sys_text: Optional[str] = None
        self.sys_ids: List[int] = []
        self.segments: Dict[str, List[int]] = {}  # message id -> token ids
        self.lock = threading.Lock()
        self.dropped = 0  # non-seed messages cut from the front (sticky truncation point)
        self.prompt_len = 0  # tokens of the last run's prompt (the thread's live context)
        self.truncations = 0  # times this thread's history was cut at the window


class _Replay:
    """Host-only generation for pre-aging threads (``EngineBackend.replay``).

    Walks the run's grammar exactly as the engine does (forced literal text,
    choice tries, repeat decisions, hints) and draws every sampled token
    uniformly from the step's allow-set -- what the random-init model's
    sampling amounts to (a terminator is one token out of ~32k, so free text
    runs to its budget, as measured on the GPU: ``work_per_analysis``).  The
    reply's token ids become the thread's assistant segment, so a replayed
    history has the token count and structure of a generated one; its KV is
    computed by the engine's real prefill on the thread's first engine run."""

    def __init__(self, grt, eos_ids, use_hints: bool, seed: int):
        import numpy as np
        self.np = np
        self.grt = grt
        self.eos = list(eos_ids)
        self.use_hints = use_hints
        self.rng = np.random.default_rng(seed)
        self._rows: Dict[int, "np.ndarray"] = {}

    def _allowed(self, row: int, drop=()):
        key = (row, tuple(drop))
        ids = self._rows.get(key)
        if ids is None:
            words = self.grt.masks.rows[row]
            bits = self.np.unpackbits(words.view(self.np.uint8), bitorder="little")
            ids = self.np.flatnonzero(bits).astype(self.np.int64)
            if drop:
                ids = self.np.setdiff1d(ids, self.np.asarray(drop, self.np.int64))
            self._rows[key] = ids
        return ids

    def generate(self, grammar, max_new: int) -> List[int]:
        from .structured import GrammarState
        gs = GrammarState(self.grt, grammar, self.eos, max_tokens=max_new, use_hints=self.use_hints)
        out: List[int] = []
        while True:
            act, arg = gs.action()
            if act == "force":
                out.extend(arg)
                continue
            if act != "sample" or len(out) >= max_new * 4 + 64:  # the engine's runaway bound (_drive)
                return out
            kind, m = arg
            sub = gs.sub
            if kind == "bitmap" and sub is not None and sub[0] == "free":
                # a free-text run: draw the rest of its budget at once (terminators
                # excluded -- with ~32k allowed tokens the engine ends one early in
                # <1 % of runs); the state then closes the run as at its budget
                _, op, n, term_ids = sub
                k = op.max_tokens - n
                if k > 0:
                    pool = self._allowed(m, term_ids)
                    out.extend(pool[self.rng.integers(len(pool), size=k)].tolist())
                    gs.sub = ("free", op, op.max_tokens, term_ids)
                    gs.n_generated += k
                    continue
            pool = m if kind == "list" else self._allowed(m)
            t = int(pool[int(self.rng.integers(len(pool)))])
            if t in self.eos:
                gs.advance(t)
                return out
            out.append(t)
            gs.advance(t)


class EngineBackend(Backend):
    def __init__(self, engine: LLMEngine, default_max_tokens: int = 512, keep_seed: int = 2,
                 temperature: Optional[float] = None, trunc_low: float = 0.5, top_k: int = 0, top_p: float = 1.0):
        self.engine = engine
        self.top_k = top_k  # defaults for runs that do not set them (run_assistant(sampling=...))
        self.top_p = top_p
        self.tok = engine.tok
        self.default_max_tokens = default_max_tokens
        self.keep_seed = keep_seed
        self.temperature = temperature
        self.trunc_low = trunc_low
        self._gen_tokens: Dict[str, List[int]] = {}  # run id -> generated ids (for the reply segment)
        self._lock = threading.Lock()
        self._replay: Optional[_Replay] = None
        self._threads: List[_ThreadTokens] = []
        self.truncations = 0  # history cuts over every thread (sticky truncation events)

    # ------------------------------------------------------------ replay
    def set_replay(self, on: bool, seed: int = 0) -> None:
        """Pre-aging mode: runs complete on the host (grammar walk with uniform
        draws, :class:`_Replay`) instead of on the engine.  Threads driven
        through prior incidents this way carry the history a long-lived
        reference thread has (``test_with_file.py:28-38,64``: three threads
        per driver, reused for every incident of the batch)."""
        self._replay = _Replay(self.engine.grt, self.engine.eos_ids, self.engine.cfg.use_hints, seed) if on else None

    def thread_stats(self) -> Dict[str, float]:
        """Live context of every thread (tokens of its last prompt) and how
        many threads have been cut at the window at least once."""
        with self._lock:
            ths = list(self._threads)
        lens = sorted(t.prompt_len for t in ths if t.prompt_len)
        if not lens:
            return {"threads": 0}
        return {"threads": len(lens), "ctx_mean": round(sum(lens) / len(lens), 1), "ctx_p50": lens[len(lens) // 2],
                "ctx_max": lens[-1], "truncated_threads": sum(1 for t in ths if t.truncations),
                "truncations": self.truncations}

    def _state(self, ts: ThreadState) -> _ThreadTokens:
        if ts.backend_state is None:
            ts.backend_state = _ThreadTokens(self.engine.new_sequence())
            with self._lock:
                self._threads.append(ts.backend_state)
        return ts.backend_state

    def _segment(self, st: _ThreadTokens, m) -> List[int]:
        seg = st.segments.get(m.id)
        if seg is None:
            if m.role == "assistant" and m.run_id is not None:
                with self._lock:
                    gen = self._gen_tokens.pop(m.run_id, None)
                if gen is not None:
                    seg = self.tok.header("assistant") + gen + [self.tok.eot_id]
            if seg is None:
                seg = self.tok.message(m.role, m.text)
            st.segments[m.id] = seg
        return seg

    def build_prompt(self, rs: RunState, max_new: int) -> List[int]:
        st = self._state(rs.thread)
        sys_text = rs.run.instructions or rs.assistant.instructions
        if st.sys_text != sys_text:
            st.sys_text = sys_text
            st.sys_ids = self.tok.system_prefix(sys_text)
        msgs = list(rs.thread.messages)
        gen_prompt = self.tok.header("assistant")
        budget = self.engine.max_context - max_new - len(gen_prompt) - len(st.sys_ids)
        n_seed = min(self.keep_seed, len(msgs))
        seeds = [self._segment(st, m) for m in msgs[:n_seed]]
        st.dropped = min(st.dropped, len(msgs) - n_seed)
        rest = [self._segment(st, m) for m in msgs[n_seed + st.dropped:]]
        n_seed_tok = sum(len(s) for s in seeds)
        total = n_seed_tok + sum(len(s) for s in rest)
        if total > budget:
            # cut down to the low-water mark (never the newest message) and remember the cut
            low = max(n_seed_tok, int(budget * self.trunc_low))
            while len(rest) > 1 and total > low:
                total -= len(rest.pop(0))
                st.dropped += 1
            st.truncations += 1
            with self._lock:
                self.truncations += 1
        segs = seeds + rest
        if total > budget:  # a single message larger than the window: keep its tail
            flat = [t for s in segs for t in s]
            segs = [flat[-budget:]] if budget > 0 else []
        out = list(st.sys_ids)
        for s in segs:
            out.extend(s)
        out.extend(gen_prompt)
        st.prompt_len = len(out)
        return out

    def submit(self, rs: RunState) -> None:
        max_new = rs.max_tokens or self.default_max_tokens
        st = self._state(rs.thread)
        with st.lock:
            prompt = self.build_prompt(rs, max_new)
        self.service.run_started(rs)
        rep = self._replay
        if rep is not None:  # pre-aging: the reply is produced on the host, nothing runs on the engine
            gen = rep.generate(rs.response_format, max_new)
            with self._lock:
                self._gen_tokens[rs.run.id] = gen
            self.service.run_completed(rs, self.tok.decode(gen), len(prompt), len(gen), metrics={"replayed": 1.0})
            return
        temp = rs.sampling.get("temperature", self.temperature)
        seed = rs.sampling.get("seed", hash(rs.run.id) & 0x7FFFFFFF)

        def on_done(gen: Optional[List[int]], stats: Dict[str, float]):
            if gen is None:
                self.service.run_failed(rs, stats.get("error", "engine failure"))
                return
            text = self.tok.decode(gen)
            with self._lock:
                self._gen_tokens[rs.run.id] = gen
            self.service.run_completed(rs, text, len(prompt), len(gen), metrics=stats)

        self.engine.submit(st.sid, prompt, grammar=rs.response_format, max_new=max_new, temperature=temp,
                           seed=seed, on_done=on_done, top_k=rs.sampling.get("top_k", self.top_k),
                           top_p=rs.sampling.get("top_p", self.top_p))

    def cancel(self, rs: RunState) -> None:
        """A cancelled / expired run (service.cancel_run, wait_run timeout) stops
        generating in the engine; other runs are unaffected."""
        st = rs.thread.backend_state
        if st is not None:
            self.engine.cancel(st.sid)

    def release_thread(self, ts: ThreadState) -> None:
        st = ts.backend_state
        if st is not None:
            self.engine.release_sequence(st.sid)
            ts.backend_state = None
