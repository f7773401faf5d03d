"""LLM engine, part 1 of 4: scheduling (``LLMEngine`` = these mixins + the
lifecycle in ``engine.py``).

Admission of submitted runs (grammar driving / jump-forward; the KV side --
prefix reuse, sharing, allocation, eviction, swap, preemption -- is the
``KVCacheManager`` in ``kv_manager.py``, ``self.kvm``), prompt-prefill
batching, and ``step()``: which decode rows and prefill chunks go into the
next forward, overlapped with the host processing of the previous step.  The reference has no scheduler: its
driver loops run one GPT-4 call at a time (``/root/reference/test_with_file.py:64,111,159``).
"""
from __future__ import annotations

import json
import logging
import math
import os
import threading
import time
from typing import Callable, Dict, List, Optional, Sequence as Seq, Tuple

import numpy as np
import torch

from ..knobs import KNOBS
from ..ops import attention as A
from ..ops import sampling as SMP
from ..ops._lib import scratch
from ..utils import tracing
from .structured import GrammarState
from .types import PART_MIN, SPEC, InFlight, Request, Sequence, _LazySample, _spec_tok

log = logging.getLogger("k8s_llm_rca_amd.engine.engine")


class SchedulerMixin:
    def _apply_releases(self) -> None:
        with self._lock:
            rel, self._releases = self._releases, []
            keep = []
            for sid in rel:
                s = self.seqs.get(sid)
                if s is not None and s.req is not None:
                    keep.append(sid)  # still generating: release after it finishes
                    continue
                s = self.seqs.pop(sid, None)
                if s is not None:
                    self.kvm.drop(s, gone=True)
            self._releases = keep + self._releases

    def _apply_cancels(self, in_flight: set) -> None:
        """Requests in ``in_flight`` (their sample is on the device) are only
        flagged: :meth:`_process_tokens` fails them when their token lands."""
        with self._lock:
            cl, self._cancels = self._cancels, []
        now = time.perf_counter()
        lim = self.cfg.max_run_s
        for s in (self.seqs.get(sid) for sid in cl):
            if s is not None and s.req is not None:
                s.req.cancelled = True
        if lim is not None:
            for s in self._snapshot():
                if s.req is not None and not s.req.cancelled and now - s.req.t_submit > lim:
                    s.req.cancelled = True
                    self.stats["timeouts"] += 1
        for s in self._snapshot():
            r = s.req
            if r is not None and r.cancelled and s.id not in in_flight:
                self._fail_req(r, "cancelled")

    # ---------------------------------------------------------------- steps
    def _admit(self) -> None:
        with self._lock:
            inc, self._incoming = self._incoming, []
            seqs = {sid: self.seqs[sid] for sid, *_ in inc}
        deferred = []
        for item in inc:
            sid, toks, grammar, max_new, temp, seed, on_done, top_k, top_p = item
            s = seqs[sid]
            if self._fault is not None:  # the TP communicator is dead: nothing can run any more
                if on_done:
                    on_done(None, {"error": self._fault})
                continue
            if s.req is not None:
                if s.req.cancelled:  # the cancelled request still drains its in-flight sample: next step
                    deferred.append(item)
                elif on_done:  # one bad submit fails alone, never the engine
                    on_done(None, {"error": f"sequence {sid} already has an active request"})
                continue
            # longest common prefix with what is cached -> keep that KV
            lcp = 0
            n = min(s.n_cached, len(toks))
            cur = s.tokens
            while lcp < n and cur[lcp] == toks[lcp]:
                lcp += 1
            # cached positions the new prompt re-prefills (history truncation, divergence)
            self.stats["recompute_tokens"] += max(0, n - lcp)
            s.tokens = toks
            s.n_cached = lcp
            self.kvm.keep_prefix(s, lcp)  # KV of the common prefix kept (or swapped back in)
            gs = GrammarState(self.grt, grammar, self.eos_ids, max_tokens=max_new, use_hints=self.cfg.use_hints)
            r = Request(s, gs, max_new, temp, seed, on_done, len(toks), top_k, top_p)
            s.req = r
            self.stats["requests"] += 1
            self._drive(r)
        if deferred:
            with self._lock:
                self._incoming[:0] = deferred

    def _drive(self, r: Request) -> None:
        """Run grammar actions until a sample is needed (forced text is appended)."""
        s = r.seq
        while True:
            act, arg = r.gs.action()
            if act == "force":
                s.tokens.extend(arg)
                r.generated.extend(arg)
                r.n_forced += len(arg)
                self.stats["forced_tokens"] += len(arg)
                continue
            if act == "sample":
                if len(r.generated) >= r.max_new * 4 + 64:
                    self.stats["end_cap"] += 1
                    self._finish(r)
                    return
                r.mask = arg
                return
            self.stats["end_grammar"] += 1
            self._finish(r)
            return

    def _finish(self, r: Request) -> None:
        s = r.seq
        s.req = None
        s.tokens.append(self.tok.eot_id)  # end of the assistant message; prefilled with the next run
        s.last_used = time.perf_counter()
        st = {"prompt_tokens": r.n_prompt, "completion_tokens": len(r.generated), "forced_tokens": r.n_forced,
              "sampled_tokens": r.n_sampled, "latency_s": time.perf_counter() - r.t_submit,
              "ttft_s": (r.t_first - r.t_submit) if r.t_first else 0.0}
        if r.on_done:
            r.on_done(list(r.generated), st)

    def _defer_prefill(self, cands: List["Sequence"]) -> bool:
        """Hold this step's prefill back (``EngineConfig.prefill_min_tokens``):
        only when every candidate is a new run's prompt (no token generated
        yet), together they are short of the minimum, and the oldest was
        submitted less than ``prefill_max_defer_s`` ago."""
        tot, oldest = 0, None
        for s in cands:
            r = s.req
            if r is None or r.t_first is not None or s.pending <= self.cfg.tiny_chunk_tokens:
                return False
            tot += s.pending
            oldest = r.t_submit if oldest is None else min(oldest, r.t_submit)
        return tot < self.cfg.prefill_min_tokens and time.perf_counter() - oldest < self.cfg.prefill_max_defer_s

    def step(self) -> bool:
        """One engine step.  In async mode the sequences sampled by the previous
        step (still in flight: their tokens are on the device only) join this
        step as decode rows fed straight from the device tokens, and the host
        processes those tokens while this step's forward runs on the GPU."""
        t_host0 = self._t_step0 = time.perf_counter()
        if self._cancels or self.cfg.max_run_s is not None:
            ps0 = self._pending_sample
            self._apply_cancels(set(s.id for s in ps0[1]) if ps0 is not None else set())
        self._admit()
        self.stats["admit_s"] += time.perf_counter() - t_host0
        if self._releases:
            self._apply_releases()
        self.kvm.tick()  # KV host tier: landed swap-outs, swap ahead of need
        # The previous forward's sampling is launched only now, AFTER this
        # step is scheduled, so sample(k) and forward(k+1) reach the GPU back
        # to back while it is still busy with forward(k): the host's
        # scheduling never leaves the GPU idle.
        ps = self._pending_sample
        self._pending_sample = None
        if ps is not None:
            for s in ps[1]:
                s.tokens.append(SPEC)
        snap = self._snapshot()
        active = [s for s in snap if s.req is not None and s.pending > 0 and not self.kvm.loading(s)]
        if not active:
            if ps is not None:  # nothing else to run: just finish the pending sample
                for s in ps[1]:
                    s.tokens.pop()
                self._process_tokens(self._launch_sample(*ps))
                return True
            loading = [s for s in snap if s.req is not None and s.loading is not None]
            if loading:  # only swap-ins are pending: wait for the oldest
                loading[0].loading.synchronize()
                return True
            return False
        BS = self.kv.block_size
        decode, prefill = [], []
        budget = self.cfg.max_batch_tokens
        protect = set(s.id for s in active)
        active.sort(key=lambda s: s.req.t_submit)  # oldest first: they keep their KV under pressure
        placed: set = set()
        for s in active:
            if s.pending == 1 and len(decode) < self.cfg.max_decode_seqs:
                if (self.kvm.ensure_blocks(s, s.n_cached + 1, protect)
                        or self.kvm.preempt_for(s, s.n_cached + 1, placed, protect, active)):
                    decode.append(s)
                    placed.add(s.id)
        budget -= len(decode)
        chunks: List[Tuple[Sequence, int]] = []
        cands = [s for s in active if (s.pending > 1 or (s.pending == 1 and s.id not in placed))
                 and s.tokens[-1] != SPEC]
        if (cands and self.cfg.prefill_min_tokens > 0 and len(decode) >= max(1, self.cfg.prefill_defer_min_rows)
                and self._defer_prefill(cands)):
            cands = []
            self.stats["prefill_deferred_steps"] += 1
        for s in cands:
            if budget <= 0:
                break
            if s.req is None:  # failed below (longer than the pool)
                continue
            q = min(s.pending, budget)
            if len(s.tokens) > self.kv.num_blocks * BS:
                self._fail_req(s.req, "context longer than the whole KV pool")
                continue
            if self.cfg.prefix_sharing and s.n_cached % BS == 0 and len(s.blocks) == s.n_cached // BS:
                self.kvm.attach_prefix(s)
                q = min(s.pending, budget)
            if not (self.kvm.ensure_blocks(s, s.n_cached + q, protect)
                    or self.kvm.preempt_for(s, s.n_cached + q, placed, protect, active)):
                continue
            chunks.append((s, q))
            placed.add(s.id)
            budget -= q
        if not decode and not chunks:
            if ps is not None:  # only the in-flight sample can progress: finish it
                for s in ps[1]:
                    s.tokens.pop()
                self._process_tokens(self._launch_sample(*ps))
                return True
            # nothing fits even after preemption: fail the youngest request alone
            young = [s for s in active if s.req is not None]
            if young:
                self._fail_req(young[-1].req, "KV pool exhausted")
            return True
        tiny = [(s, q) for s, q in chunks if q <= self.cfg.tiny_chunk_tokens]
        big = [(s, q) for s, q in chunks if q > self.cfg.tiny_chunk_tokens]
        if len(decode) + sum(q for _, q in tiny) > max(self.cfg.max_decode_seqs, 1):
            tiny, big = [], chunks
        # decode-attention rows (sequence, token offset past n_cached): the decode
        # rows, then every token of the tiny chunks; token order = decode, tiny, big
        drows = [(s, 0) for s in decode] + [(s, j) for s, q in tiny for j in range(q)]
        rows = [(s, 1) for s in decode] + tiny + big
        if self._shape_trace:
            with open(self._shape_trace, "a") as f:
                f.write(json.dumps({"d": [s.n_cached + j + 1 for s, j in drows],
                                    "p": [[s.n_cached + q, q] for s, q in big]}) + "\n")
        sample_rows = []  # (row index in batch, seq)
        off = 0
        for s, q in rows:
            off += q
            if s.n_cached + q == len(s.tokens):
                sample_rows.append((off - 1, s))
        spec = lazy = None
        if ps is not None:
            # the previous step's sampling is launched from inside the forward,
            # after this step's inputs are packed and uploaded and right before
            # its first kernel: the GPU goes sample(k) -> forward(k+1) with no
            # host packing time between them
            pos_in = {s.id: j for j, s in enumerate(ps[1])}
            src = np.array([pos_in.get(s.id, -1) if s.tokens[s.n_cached] == SPEC else -1 for s in decode]
                           + [-1] * (len(drows) - len(decode)), dtype=np.int32)
            lazy = _LazySample(self, ps)
            spec = (src, lazy)
        self.stats["host_s"] += time.perf_counter() - t_host0
        logits = self._forward(drows, big, [i for i, _ in sample_rows], spec)
        infl = lazy.launch() if lazy is not None else None
        spec_pos = {}
        for s, q in rows:
            if q == 1 and s.tokens[s.n_cached] == SPEC:
                spec_pos[s.id] = s.n_cached
            s.n_cached += q
            s.last_used = time.perf_counter()
        if self.cfg.prefix_sharing:
            for s, _ in chunks:  # publish the pages this prefill completed (their KV write is enqueued)
                self.kvm.register_blocks(s)
        self.stats["steps"] += 1
        n_rows = len(drows) + sum(q for _, q in big)
        if n_rows <= 256:  # decode-size step: the projections stream every weight once (M <= 256 kernels)
            self.stats["small_steps"] += 1
            self.stats["small_rows"] += n_rows
        else:
            self.stats["big_rows"] += n_rows
        self.stats["prefill_tokens"] += sum(q for _, q in chunks)
        self.stats["tiny_chunk_tokens"] += len(drows) - len(decode)
        self.stats["decode_tokens"] += len(decode)
        self.stats["decode_ctx_tokens"] += sum(s.n_cached for s in decode)
        self.stats["prefill_ctx_tokens"] += sum(s.n_cached * q for s, q in chunks)
        # (query, key) pairs the prefill attention computes: the cached keys plus the causal chunk
        self.stats["prefill_attn_pairs"] += sum((s.n_cached - q) * q + q * (q + 1) // 2 for s, q in chunks)
        if infl is not None:
            # host side of the previous step, overlapped with this step's forward
            toks = self._process_tokens(infl, placeholders=True)
            for s, t in zip(infl.seqs, toks):
                p = spec_pos.get(s.id)
                if p is not None and (len(s.tokens) <= p or s.tokens[p] != t):
                    s.n_cached = p  # the speculative KV at p is not this sequence's token (it finished)
                    self.kvm.truncate_chain(s, p)
        # rows still waiting for a sample (a finished or newly-forced sequence is not)
        keep = [(i, s) for i, (ri, s) in enumerate(sample_rows)
                if s.req is not None and s.n_cached == len(s.tokens)]
        if keep:
            rows_sel = [i for i, _ in keep] if len(keep) != len(sample_rows) else None
            pend = (logits, [s for _, s in keep], rows_sel)
            if self._async:
                self._pending_sample = pend
            else:
                self._process_tokens(self._launch_sample(*pend))
        return True
