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
    __slots__ = ("sid", "sys_text", "sys_ids", "segments", "lock", "dropped")

    def __init__(self, sid: int):
        self.sid = sid
        self.sys_text: Optional[str] = None
        self.sys_ids: List[int] = []
        self.segments: Dict[str, List[int]] = {}  # message id -> token ids
        self.lock = threading.Lock()
        self.dropped = 0  # non-seed messages cut from the front (sticky truncation point)


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

    def _state(self, ts: ThreadState) -> _ThreadTokens:
        if ts.backend_state is None:
            ts.backend_state = _ThreadTokens(self.engine.new_sequence())
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
        segs = seeds + rest
        if total > budget:  # a single message larger than the window: keep its tail
            flat = [t for s in segs for t in s]
            segs = [flat[-budget:]] if budget > 0 else []
        out = list(st.sys_ids)
        for s in segs:
            out.extend(s)
        out.extend(gen_prompt)
        return out

    def submit(self, rs: RunState) -> None:
        max_new = rs.max_tokens or self.default_max_tokens
        st = self._state(rs.thread)
        with st.lock:
            prompt = self.build_prompt(rs, max_new)
        self.service.run_started(rs)
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
