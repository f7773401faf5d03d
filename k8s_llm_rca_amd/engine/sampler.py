"""LLM engine, part 4 of 4: sampling and token processing.

Grammar-masked sampling of each step's logits (TP: the vocab-parallel sampler
of ``tp_sampler.py``, ``self.tps``), the async device -> host copy of the
tokens, and the host side that appends them, advances grammars and finishes
requests (NON_FINITE rows fail their request).
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

# knob token_flag: the host's poll period while the GPU finishes a step, and the
# smallest sampled batch that polls (a few-row step is latency-bound: a 50 us poll
# period would be ~2 % of a concurrency-1 decode token, so it keeps the event wait)
TOKEN_FLAG_SLEEP_S = 50e-6
TOKEN_FLAG_MIN_ROWS = 16
log = logging.getLogger("k8s_llm_rca_amd.engine.engine")


class SamplerMixin:
    # ------------------------------------------------------------ sampling
    def _mask_table(self) -> Optional[torch.Tensor]:
        if self._mask_ver != self.grt.masks.version:
            ver, arr = self.grt.masks.snapshot()  # version and rows together (MaskTable.snapshot)
            host = torch.from_numpy(arr)
            if self.device.type == "cuda":  # pinned + non-blocking: a pageable copy would wait for the GPU
                host = host.pin_memory()
            self._mask_dev = host.to(self.device, non_blocking=True)
            self._mask_ver = ver
        return self._mask_dev

    def _launch_sample(self, logits: torch.Tensor, seqs: List[Sequence], rows: Optional[List[int]] = None) -> InFlight:
        """Launch masked sampling for ``seqs`` (rows ``rows`` of ``logits``, all
        rows when None) and an async device -> host copy of the tokens; nothing
        waits here (every upload is pinned + non-blocking)."""
        t0 = time.perf_counter()
        B = len(seqs)
        mask_id = np.full(B, -1, dtype=np.int32)
        list_off = np.zeros(B, dtype=np.int32)
        list_len = np.zeros(B, dtype=np.int32)
        lists: List[int] = []
        temps = np.zeros(B, dtype=np.float32)
        seeds = np.zeros(B, dtype=np.int32)
        steps = np.zeros(B, dtype=np.int32)
        topk = np.zeros(B, dtype=np.int32)
        topp = np.ones(B, dtype=np.float32)
        for i, s in enumerate(seqs):
            r = s.req
            kind, m = r.mask
            if kind == "list":
                list_off[i] = len(lists)
                list_len[i] = len(m)
                lists.extend(m)
            else:
                mask_id[i] = m
            temps[i] = r.temperature
            seeds[i] = (r.seed * 2654435761 + s.id) & 0x7FFFFFFF
            steps[i] = len(r.generated)
            topk[i] = r.top_k
            topp[i] = r.top_p
        if not lists:
            lists = [0]
        filt = bool((topk > 0).any() or (topp < 1.0).any())
        status = None
        car = self.pc.custom_ar if self.pc.tp_size > 1 else None
        if self._dist_sample:
            tok = self.tps.sample_leader(logits, mask_id, list_off, list_len, np.asarray(lists, np.int32),
                                         seeds, steps, temps, topk, topp, rows)
        else:
            table = self._mask_table()
            if table is not None and int(mask_id.max(initial=-1)) >= table.shape[0]:
                # a bitmap row the device mirror does not hold: sampling would read past
                # the table (garbage bits, silently ended runs) -- fail loudly instead
                raise RuntimeError(f"grammar mask row {int(mask_id.max())} >= device table rows {table.shape[0]}")
            arrays = [mask_id, list_off, list_len, np.asarray(lists, np.int32), seeds, steps, temps.view(np.int32)]
            if filt:
                arrays += [topk, topp.view(np.int32)]
            if rows is not None:
                arrays.append(np.asarray(rows, np.int32))
            ints = self._to_dev(arrays)
            if rows is not None:
                logits = logits.index_select(0, ints[-1])
            d_temps = ints[6].view(torch.float32)
            tok = SMP.sample(logits, d_temps, ints[4], ints[5], ints[0], table, ints[1], ints[2], ints[3],
                             vocab=self.vocab, top_k=ints[7] if filt else None,
                             top_p=ints[8].view(torch.float32) if filt else None)
        if car is not None and self.device.type == "cuda":
            # the communicator's STATUS, stream-ordered after this step's forward and
            # the sampling collectives (the xGMI all-gather of the TP winners): valid
            # once the sampled tokens are (_process_tokens checks it first)
            status = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            car.status_async(status)
        nf = None
        if self._nf is not None:  # the flags of every forward since the last sampling
            nf = torch.empty(self._nf.numel(), dtype=torch.int32, pin_memory=True)
            nf.copy_(self._nf, non_blocking=True)
            self._nf.zero_()
        seq = 0
        if tok.is_cuda:
            host = torch.empty(B, dtype=torch.int32, pin_memory=True)
            host.copy_(tok, non_blocking=True)
            if KNOBS.token_flag and self.pc.tp_size == 1 and B >= TOKEN_FLAG_MIN_ROWS:
                # stream-ordered after the copy: a one-wave kernel raises the pinned flag
                from ..ops._lib import check, lib, stream_ptr
                if self._tflag is None:
                    self._tflag = torch.zeros(64, dtype=torch.int32, pin_memory=True)
                    self._tflag_np = self._tflag.numpy()
                self._tflag_seq += 1
                seq = self._tflag_seq
                check(lib().k8s_host_flag(self._tflag.data_ptr(), seq, stream_ptr(tok)), "host_flag")
            ev = torch.cuda.Event(blocking=KNOBS.blocking_sync)
            ev.record()
        else:
            host, ev = tok, None
        self.stats["sample_s"] += time.perf_counter() - t0
        return InFlight(seqs, tok, host, ev, t0, status, nf, seq)

    def _wait_flag(self, fl: InFlight) -> None:
        """Sleep-poll the pinned host flag until the step's tokens have landed
        (knob token_flag): the engine thread leaves the CPU and the GIL to the
        pipelines instead of spinning in hipEventSynchronize.  The event is
        recorded after the flag kernel, so a completed event with the flag
        still unseen falls back to it (never a hang)."""
        f = self._tflag_np
        t = time.perf_counter()
        while int(f[0]) < fl.flag_seq:
            time.sleep(TOKEN_FLAG_SLEEP_S)
            if time.perf_counter() - t > 1.0 and fl.event.query():
                fl.event.synchronize()
                return

    def _process_tokens(self, fl: InFlight, placeholders: bool = False) -> List[int]:
        """Host side of a sampled step: wait for its tokens (not for later GPU
        work), append them, advance grammars, jump-forward, finish requests.
        ``placeholders``: the sequences carry a SPEC token that the sampled
        token replaces."""
        t1 = time.perf_counter()
        if fl.flag_seq:
            self._wait_flag(fl)
        elif fl.event is not None:
            fl.event.synchronize()
        self._last_wait_end = time.perf_counter()
        if fl.status is not None and int(fl.status[0]) != 0:
            from ..parallel.xgmi import CommFault
            raise CommFault("xGMI collective timed out: a TP peer never arrived (allreduce STATUS set)")
        toks = fl.tok_host.tolist()
        if fl.nf is not None and bool(fl.nf.any()):
            layer = int(fl.nf.nonzero()[0, 0])
            self.stats["nonfinite_flag_steps"] += 1
            if self.stats["nonfinite_first_layer"] < 0:
                self.stats["nonfinite_first_layer"] = layer
                log.error("non-finite values in layer %d's normed input (knob nonfinite_check; step %d)", layer,
                          self.stats["steps"])
        now = time.perf_counter()
        if self._pending_ev:
            self._collect_timing()
        self.stats["wait_s"] += now - t1
        for s, t in zip(fl.seqs, toks):
            if placeholders and s.tokens and s.tokens[-1] == SPEC:
                s.tokens.pop()
            r = s.req
            if r is None:
                continue
            if r.cancelled:
                self._fail_req(r, "cancelled")
                continue
            if r.t_first is None:
                r.t_first = now
            if t == SMP.NON_FINITE:  # the model's logits went non-finite: fail loudly, never emit garbage
                self.stats["nonfinite_rows"] += 1
                if self.stats["nonfinite_rows"] == 1:
                    log.error("non-finite logits (NaN / inf) in a sampled row (sequence %d): failing its request",
                              s.id)
                self._fail_req(r, "non-finite logits (NaN / inf) in this request's row")
                continue
            if t < 0:  # no allowed token left
                self.stats["end_no_allowed"] += 1
                self._finish(r)
                continue
            r.n_sampled += 1
            self.stats["sampled_tokens"] += 1
            r.generated.append(t)
            if t in self.eos_ids:
                r.generated.pop()
                r.gs.advance(t)
                self.stats["end_eos"] += 1
                self._finish(r)
                continue
            s.tokens.append(t)
            r.gs.advance(t)
            self._drive(r)
        self.stats["post_s"] += time.perf_counter() - now
        return toks
