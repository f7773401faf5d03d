"""LLM engine, part 2 of 4: step packing and execution.

One engine step becomes a header + one int32 payload (token ids, positions,
KV slots, attention metadata and work lists): packed on the host, uploaded in
one pinned copy, unpacked on the device and run eagerly through the native
layer executor.  Under TP the rank-0 scheduler sends the same message to the
workers (``serve_worker``) over the host channel.
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


class StepExecMixin:
    # ------------------------------------------------------------- forward
    def _meta_arrays(self, seqs_q: List[Tuple[Sequence, int]]):
        BS = self.kv.block_size
        n = len(seqs_q)
        maxb = max(len(s.blocks) for s, _ in seqs_q)
        bt = np.zeros((n, maxb), dtype=np.int32)
        ctx = np.zeros(n, dtype=np.int32)
        qs = np.zeros(n + 1, dtype=np.int32)
        for i, (s, q) in enumerate(seqs_q):
            bt[i, : len(s.blocks)] = s.blocks
            ctx[i] = s.n_cached + q
            qs[i + 1] = qs[i] + q
        return bt, ctx, qs

    def _token_arrays(self, rows: List[Tuple[Sequence, int]]):
        BS = self.kv.block_size
        if not rows:
            e = np.zeros(0, np.int32)
            return e, e, e
        ids, pos, slots = [], [], []
        for s, q in rows:
            a = s.n_cached
            ids.extend(s.tokens[a:a + q])
            p = np.arange(a, a + q, dtype=np.int64)
            pos.append(p)
            blk = np.asarray(s.blocks, dtype=np.int64)[p // BS]
            slots.append(blk * BS + p % BS)
        return (np.asarray(ids, dtype=np.int32), np.concatenate(pos).astype(np.int32),
                np.concatenate(slots).astype(np.int32))

    def _decode_token_arrays(self, drows: List[Tuple[Sequence, int]]):
        BS = self.kv.block_size
        n = len(drows)
        ids = np.empty(n, np.int32)
        pos = np.empty(n, np.int32)
        slots = np.empty(n, np.int32)
        for i, (s, j) in enumerate(drows):
            p = s.n_cached + j
            ids[i] = s.tokens[p]
            pos[i] = p
            slots[i] = s.blocks[p // BS] * BS + p % BS
        return ids, pos, slots

    def _decode_chain(self, drows: List[Tuple[Sequence, int]]) -> Optional[np.ndarray]:
        """chain[i]: decode row i is the token after row i-1's (same sequence):
        such rows share multi-token decode-attention items.  None when no row
        continues its predecessor (plain decode steps)."""
        if self._dec_gmax <= 1 or len(drows) == len(set(id(s) for s, _ in drows)):
            return None
        ch = np.zeros(len(drows), dtype=bool)
        for i in range(1, len(drows)):
            ch[i] = drows[i][0] is drows[i - 1][0] and drows[i][1] == drows[i - 1][1] + 1
        return ch

    def _plan_ctx(self, ctx: np.ndarray, chain: Optional[np.ndarray]) -> np.ndarray:
        """Context lengths the split planner sees: one per multi-token item."""
        if chain is None:
            return ctx
        lead, nt = A.decode_groups(ctx, np.arange(ctx.size), chain, self._dec_gmax)
        return ctx[lead + nt - 1]

    def _decode_meta(self, drows: List[Tuple[Sequence, int]]):
        """Block tables / context lengths / q_start of decode-attention rows:
        row (s, j) is the token at n_cached + j and sees keys 0..n_cached + j."""
        n = len(drows)
        maxb = max(len(s.blocks) for s, _ in drows)
        bt = np.zeros((n, maxb), dtype=np.int32)
        ctx = np.zeros(n, dtype=np.int32)
        for i, (s, j) in enumerate(drows):
            bt[i, : len(s.blocks)] = s.blocks
            ctx[i] = s.n_cached + j + 1
        return bt, ctx, np.arange(n + 1, dtype=np.int32)

    def _forward(self, decode: List[Tuple[Sequence, int]], chunks: List[Tuple[Sequence, int]],
                 sample_idx: List[int], spec=None):
        """``spec`` = (src[nd], tok): decode row i takes its input id from the
        device tensor ``tok[src[i]]`` when ``src[i] >= 0`` (tokens sampled by
        the in-flight step, not yet on the host)."""
        t0 = time.perf_counter()
        timed = (self._step_timing or self._trace is not None) and self.device.type == "cuda"
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            if self._trace is not None and self._trace_base is None:
                self._trace_base = (torch.cuda.Event(enable_timing=True), t0)
                self._trace_base[0].record()
            ev[0].record()
        if spec is not None and self._chan is not None:
            _spec_tok(spec)  # TP: sample(k) -- a message + an all-gather -- goes before forward(k+1) on every rank
        if (not chunks and self.cfg.use_graphs and self.device.type == "cuda" and decode and self._graphs_ok()
                and self.kv.block_size % 64 == 0):
            out = self._forward_graph(decode, spec, sample_idx)
            self.stats["graph_steps"] += 1
            self.stats["decode_steps"] += 1
            kind = "graph"
        else:
            out = self._forward_eager(decode, chunks, sample_idx, spec)
            if not chunks:
                self.stats["decode_steps"] += 1
            kind = "eager"
        t1 = time.perf_counter()
        dt = t1 - t0
        self.stats["forward_s"] += dt
        if timed:
            ev[1].record()
            rec = None
            if self._trace is not None:
                ek, self._trace_evk = getattr(self, "_trace_evk", None), None
                rec = {"step": self.stats["steps"], "kind": kind, "nd": len(decode), "_ek": ek,
                       "np": sum(q for _, q in chunks), "t_enq0": t0, "t_enq1": t1, "t_wait": self._last_wait_end,
                       "t_step": getattr(self, "_t_step0", None)}
            self._pending_ev.append((kind, dt, ev, rec))
        return out

    def _collect_timing(self) -> None:
        """Fold completed step events into stats (with overlapped steps the
        newest forward may still be running: its events stay pending)."""
        keep = []
        for kind, dt, (e0, e1), rec in self._pending_ev:
            if not e1.query():
                keep.append((kind, dt, (e0, e1), rec))
                continue
            self.stats[kind + "_issue_s"] += dt
            self.stats[kind + "_gpu_s"] += e0.elapsed_time(e1) / 1e3
            if rec is not None:
                base, tb = self._trace_base
                rec["g0"] = round(base.elapsed_time(e0), 4)   # ms on the GPU clock since the first traced forward
                rec["g1"] = round(base.elapsed_time(e1), 4)
                ek = rec.pop("_ek")
                rec["gk"] = round(base.elapsed_time(ek), 4) if ek is not None else None  # upload landed
                for k in ("t_enq0", "t_enq1", "t_wait", "t_step"):
                    rec[k] = None if rec[k] is None else round((rec[k] - tb) * 1e3, 4)  # ms, host clock
                self._trace_buf.append(json.dumps(rec))
        self._pending_ev = keep
        if len(self._trace_buf) >= 256:
            self.flush_trace()

    def flush_trace(self) -> None:
        if self._trace is not None and self._trace_buf:
            with open(self._trace, "a") as f:
                f.write("\n".join(self._trace_buf) + "\n")
            self._trace_buf = []

    def _to_dev(self, arrays: List[np.ndarray]) -> List[torch.Tensor]:
        """One H2D copy for all int32 metadata arrays."""
        sizes = [a.size for a in arrays]
        flat = np.concatenate([a.reshape(-1).astype(np.int32, copy=False) for a in arrays]) if arrays else \
            np.zeros(0, np.int32)
        host = torch.from_numpy(flat)
        if self.device.type == "cuda":
            host = host.pin_memory()
            dev = host.to(self.device, non_blocking=True)
        else:
            dev = host
        out, o = [], 0
        for a, n in zip(arrays, sizes):
            out.append(dev[o:o + n].view(*a.shape))
            o += n
        return out

    # Step wire format (also the TP broadcast): header int64[12] + one int32 payload
    # = ids[T] pos[T] slots[T] sidx[ns] | bt_d ctx_d qs_d | bt_p ctx_p qs_p tseq ttok0 tlen
    HDR = 14

    def _pack_step(self, decode, chunks, sample_idx):
        """``decode``: decode-attention rows (sequence, token offset past n_cached)."""
        ids_d, pos_d, slots_d = self._decode_token_arrays(decode)
        ids, pos, slots = self._token_arrays(list(chunks))
        ids, pos, slots = np.concatenate([ids_d, ids]), np.concatenate([pos_d, pos]), np.concatenate([slots_d, slots])
        arrays = [ids, pos, slots, np.asarray(sample_idx, dtype=np.int32)]
        nd = len(decode)
        maxb_d = maxb_p = n_tiles = n_merge = n_items = 0
        n_parts, part = 1, PART_MIN
        if decode:
            bt_d, ctx_d, qs_d = self._decode_meta(decode)
            maxb_d = bt_d.shape[1]
            chain = self._decode_chain(decode)
            n_parts, part = A.plan_decode_split(self._plan_ctx(ctx_d, chain), self.model.nkv,
                                                max_parts=self._n_parts(self.max_context))
            n_parts = max(n_parts, -(-int(ctx_d.max()) // part))
            arrays += [bt_d, ctx_d, qs_d]
            if self.kv.block_size % 64 == 0:
                items = A.build_decode_items(ctx_d, np.arange(nd), part, chain, self._dec_gmax)
                n_items = items.shape[0]
                arrays.append(items)
            else:
                n_parts = 1 << (n_parts - 1).bit_length()
        if chunks:
            bt_p, ctx_p, qs_p = self._meta_arrays(chunks)
            maxb_p = bt_p.shape[1]
            plan = A.plan_prefill(qs_p.tolist(), self.model.nq // self.model.nkv, self.kv.block_size,
                                  ctx_p.tolist(), nkv=self.model.nkv)
            n_tiles, n_merge = plan.n_tiles, plan.n_merge
            arrays += [bt_p, ctx_p, qs_p] + [np.asarray(x, np.int32) for x in plan.arrays()]
        flat = np.concatenate([x.reshape(-1).astype(np.int32, copy=False) for x in arrays])
        header = np.array([1, flat.size, len(ids), nd, nd, maxb_d, len(chunks), maxb_p, n_tiles,
                           len(sample_idx), n_parts, n_merge, part, n_items], dtype=np.int64)
        return header, flat

    def _exec_step(self, header: np.ndarray, flat_host: Optional[np.ndarray], flat_dev: torch.Tensor,
                   spec=None):
        """Build StepInputs from the wire format and run the forward (every TP rank)."""
        from ..models.llama import StepInputs

        (_, _, T, nd, n_dec, maxb_d, n_pre, maxb_p, n_tiles, ns, n_parts, n_merge, part,
         n_items) = [int(v) for v in header]
        if self._sim:
            self.sim_rows[T] = self.sim_rows.get(T, 0) + 1
        o = 0

        def take(n, shape=None):
            nonlocal o
            d = flat_dev[o:o + n]
            h = flat_host[o:o + n] if flat_host is not None else None
            o += n
            if shape is not None:
                d = d.view(*shape)
            return d, h

        d_ids, _ = take(T)
        if spec is not None:
            d_ids = d_ids.clone()
            self._apply_spec(d_ids, spec[0], _spec_tok(spec))
        d_pos, _ = take(T)
        d_slots, _ = take(T)
        d_sidx, _ = take(ns)
        dmeta = pmeta = None
        if n_dec:
            bt, _ = take(n_dec * maxb_d, (n_dec, maxb_d))
            ctx, ctx_h = take(n_dec)
            qs, qs_h = take(n_dec + 1)
            items = take(n_items * 4, (n_items, 4))[0] if n_items else None
            dmeta = A.AttnMeta(block_tables=bt, ctx_lens=ctx, q_start=qs, num_seqs=n_dec, decode=True,
                               n_parts=n_parts, part_size=part, items=items, n_items=n_items,
                               ctx_lens_host=None if ctx_h is None else ctx_h.tolist(),
                               q_start_host=None if qs_h is None else qs_h.tolist())
            if n_parts > 1:
                dmeta.part_o = scratch(n_dec * self.model.nq * n_parts * self.model.D, torch.float32,
                                       self.device)
                dmeta.part_ml = scratch(n_dec * self.model.nq * n_parts * 2, torch.float32, self.device)
        if n_pre:
            bt, _ = take(n_pre * maxb_p, (n_pre, maxb_p))
            ctx, ctx_h = take(n_pre)
            qs, qs_h = take(n_pre + 1)
            tiles = [take(n_tiles)[0] for _ in range(6)]
            merges = [take(n_merge)[0] for _ in range(4)]
            pmeta = A.AttnMeta(block_tables=bt, ctx_lens=ctx, q_start=qs, num_seqs=n_pre, decode=False,
                               n_tiles=n_tiles, n_merge=n_merge,
                               ctx_lens_host=None if ctx_h is None else ctx_h.tolist(),
                               q_start_host=None if qs_h is None else qs_h.tolist())
            (pmeta.tile_seq, pmeta.tile_tok0, pmeta.tile_len, pmeta.tile_kv0, pmeta.tile_kv1,
             pmeta.tile_slot) = tiles
            pmeta.m_tok0, pmeta.m_len, pmeta.m_slot0, pmeta.m_np = merges
            if n_merge:
                if self._pf_ws is None:
                    self._pf_ws = A.prefill_workspace(self.model.nkv, self.device)
                pmeta.pf_o, pmeta.pf_ml = self._pf_ws
        inp = StepInputs(d_ids, d_pos, d_slots, nd, dmeta, pmeta, d_sidx.long())
        return self._model_fwd(inp)

    def _model_fwd(self, inp):
        """TP with vocab-parallel sampling keeps each rank's logits shard."""
        if self._dist_sample:
            return self.model.forward(inp, self.kv.k, self.kv.v, gather_logits=False)
        return self.model.forward(inp, self.kv.k, self.kv.v)

    # ------------------------------------------------- TP vocab-parallel sampling
    SHDR = 4

    def _forward_eager(self, decode, chunks, sample_idx, spec=None):
        header, flat = self._pack_step(decode, chunks, sample_idx)
        if self._chan is not None:
            from ..parallel.channel import FWD_EAGER
            self._chan.send(FWD_EAGER, [header, flat] + ([spec[0]] if spec is not None else []))
            if self._test_host_stall_s:  # fault injection: the workers' collectives outwait their timeout
                time.sleep(self._test_host_stall_s)
                self._test_host_stall_s = 0.0
        return self._run_eager(header, flat, spec)

    def _run_eager(self, header, flat, spec):
        """Upload a packed step (one pinned async copy) and run its forward
        (rank 0, and every TP worker from the channel's message)."""
        if spec is not None:
            dev, src = self._to_dev([flat, spec[0]])
            spec = (src, spec[1])
        else:
            dev = self._to_dev([flat])[0]
        self._trace_mark()
        return self._exec_step(header, flat, dev, spec)

    def _trace_mark(self) -> None:
        """knob step_trace: a timing event right after the step's upload is
        enqueued (its GPU time minus the forward's start = the GPU waiting for
        the host's packing + upload)."""
        if self._trace is not None and self.device.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._trace_evk = e

    @staticmethod
    def _apply_spec(ids: torch.Tensor, src: torch.Tensor, tok: torch.Tensor) -> None:
        """ids[i] = tok[src[i]] where src[i] >= 0 (device-side, stream-ordered
        after the sampling kernel that produced ``tok``)."""
        n = src.shape[0]
        pick = tok.index_select(0, src.clamp(min=0).long()).clamp(min=0).to(ids.dtype)
        ids[:n] = torch.where(src >= 0, pick, ids[:n])

    def serve_worker(self) -> None:
        """TP ranks > 0: execute every step rank 0 schedules, in rank 0's
        order (sampling / forward messages from the host channel), until STOP.
        The worker never waits for its own GPU: the next message is received
        while the previous forward still runs."""
        assert self.pc.tp_rank > 0
        from ..parallel.channel import FWD_EAGER, FWD_GRAPH, SAMPLE, STOP
        logits = None
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        car = self.pc.custom_ar if self.device.type == "cuda" else None
        status, status_ev = None, None
        while True:
            kind, arrs = self._chan.recv()
            if kind == STOP:
                return
            if self._test_stall or self.comm_dead:  # this peer no longer arrives at the collectives
                continue
            if kind == SAMPLE:
                # the previous step's STATUS (its copy was queued a step ago): once
                # this rank's own wait timed out it skips every later wait but would
                # still publish flags, so rank 0 would mix unsynchronized partials
                # silently.  Stop executing instead: rank 0's next collective then
                # times out and fails every run with CommFault.
                # The check never waits for the GPU: a copy still in flight is
                # read at a later step.
                ready = status_ev is None or status_ev.query()
                if status_ev is not None and ready and int(status[0]) != 0:
                    self.comm_dead = True
                    log.error("TP rank %d: xGMI collective timed out (STATUS set); "
                              "this worker stops executing steps", self.pc.tp_rank)
                    continue
                hdr, flat, rows_a = arrs
                self._last_tok = self.tps.sample_rows(logits, hdr, flat, rows_a)
                if car is not None and ready:
                    if status is None:
                        status = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                        status_ev = torch.cuda.Event()
                    car.status_async(status)
                    status_ev.record()
            elif kind == FWD_EAGER:
                spec = (arrs[2], self._last_tok) if len(arrs) > 2 else None
                logits = self._run_eager(arrs[0], arrs[1], spec)
            elif kind == FWD_GRAPH:
                meta, flat, sel = arrs[0], arrs[1], arrs[2]
                spec = (arrs[3], self._last_tok) if len(arrs) > 3 else None
                logits = self._graph_run(int(meta[0]), int(meta[1]), int(meta[2]), int(meta[3]), int(meta[4]),
                                         flat, spec, sel)
            else:
                raise RuntimeError(f"unknown step message {kind}")

    def stop_workers(self) -> None:
        if self._chan is not None and self.pc.tp_rank == 0:
            from ..parallel.channel import STOP
            self._chan.send(STOP, [])
