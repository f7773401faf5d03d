"""LLM engine, part 3 of 4: HIP-graph decode steps.

Pure-decode steps replay one captured graph per batch bucket; the decode work
list, its item count and the keys per item are read on the device, so one
graph serves every context mix.  Static input buffers are filled from one
pinned staging copy per replay.
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


class GraphRunnerMixin:
    def _graphs_ok(self) -> bool:
        """Decode steps replay HIP graphs at TP=1, and under TP when every
        all-reduce of a decode step runs on the capturable xGMI kernel."""
        if self.pc.tp_size == 1:
            return True
        car = self.pc.custom_ar
        return car is not None and getattr(car, "max_bytes", 0) >= max(self.cfg.graph_batch_sizes) * self.mc.hidden * 2

    @staticmethod
    def _n_parts(max_ctx: int) -> int:
        """Partition count bound at the smallest partition size (buffer sizing)."""
        n = max(1, (max_ctx + PART_MIN - 1) // PART_MIN)
        return 1 << (n - 1).bit_length()

    # ---------------------------------------------------------- HIP graphs
    def _bucket(self, n: int) -> int:
        for b in self.cfg.graph_batch_sizes:
            if b >= n:
                return b
        return n

    def _ensure_static(self):
        if self._static is not None:
            return self._static
        Bmax = max(self.cfg.graph_batch_sizes)
        mb = self.max_blocks_per_seq
        npmax = self._n_parts(self.max_context)
        self._max_items = Bmax * npmax
        dev = self.device
        st = {
            "ids": torch.zeros(Bmax, dtype=torch.int32, device=dev),
            "pos": torch.zeros(Bmax, dtype=torch.int32, device=dev),
            "slots": torch.full((Bmax,), -1, dtype=torch.int32, device=dev),
            "bt": torch.zeros(Bmax, mb, dtype=torch.int32, device=dev),
            "ctx": torch.ones(Bmax, dtype=torch.int32, device=dev),
            "qs": torch.arange(Bmax + 1, dtype=torch.int32, device=dev),
            "sidx": torch.arange(Bmax, dtype=torch.int64, device=dev),
            "part_o": scratch(Bmax * self.model.nq * npmax * self.model.D, torch.float32, dev),
            "part_ml": scratch(Bmax * self.model.nq * npmax * 2, torch.float32, dev),
            "items": torch.zeros(Bmax * npmax, 4, dtype=torch.int32, device=dev),
            "n_items": torch.zeros(2, dtype=torch.int32, device=dev),  # {item count, keys per item}
            # two pinned staging buffers, alternated per graph step; each is
            # reused only after the event recorded behind its last H2D copy
            "host": [torch.zeros(Bmax * (3 + mb + 2) + 2 + Bmax * npmax * 4, dtype=torch.int32).pin_memory()
                     for _ in range(2)],
            "host_ev": [None, None],
            "host_i": 0,
        }
        self._static = st
        return st

    def _graph_inputs(self, B: int, part: int):
        from ..models.llama import StepInputs

        st = self._static
        # work-list decode: the grid is the resident-wave count and the item
        # count is read on the device, so one graph serves every item list
        meta = A.AttnMeta(block_tables=st["bt"][:B], ctx_lens=st["ctx"][:B], q_start=st["qs"][:B + 1], num_seqs=B,
                          decode=True, n_parts=self._n_parts(self.max_context), part_size=part,
                          part_o=st["part_o"], part_ml=st["part_ml"], items=st["items"], n_items=0,
                          d_n_items=st["n_items"], grid_waves=A.DECODE_WAVE_SLOTS)
        return StepInputs(st["ids"][:B], st["pos"][:B], st["slots"][:B], B, meta, None, st["sidx"][:B])

    def _capture(self, B: int, part: int):
        """Graph of a ``B``-row decode step.  ``part`` only seeds the capture:
        the decode kernels read each replay's keys-per-item from the device."""
        key = B
        g = self._graphs.get(key)
        if g is not None:
            return g
        t0 = time.perf_counter()
        inp = self._graph_inputs(B, part)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._model_fwd(inp)
        torch.cuda.current_stream(self.device).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        # thread_local: the graph-query batcher keeps issuing on its own stream from its
        # own thread while a bucket is captured mid-run
        with torch.cuda.graph(graph, pool=self._graph_pool, capture_error_mode="thread_local"):
            out = self._model_fwd(inp)
        self._graphs[key] = (graph, out)
        self.stats["captures"] += 1
        self.stats["capture_s"] += time.perf_counter() - t0
        return self._graphs[key]

    def _forward_graph(self, decode: List[Tuple[Sequence, int]], spec=None, sample_idx: Optional[List[int]] = None):
        """``decode``: decode-attention rows (sequence, token offset past
        n_cached); the logits of the ``sample_idx`` rows are returned (all rows
        when every row samples)."""
        st = self._ensure_static()
        B = len(decode)
        if sample_idx is None:
            sample_idx = list(range(B))
        Bb = self._bucket(B)
        if Bb > max(self.cfg.graph_batch_sizes):
            return self._forward_eager(decode, [], sample_idx, spec)
        BS = self.kv.block_size
        mb = self.max_blocks_per_seq
        ctx = np.ones(Bb, dtype=np.int32)
        ids = np.zeros(Bb, dtype=np.int32)
        pos = np.zeros(Bb, dtype=np.int32)
        slots = np.full(Bb, -1, dtype=np.int32)
        bt = np.zeros((Bb, mb), dtype=np.int32)
        for i, (s, j) in enumerate(decode):
            p = s.n_cached + j
            ids[i] = s.tokens[p]
            pos[i] = p
            slots[i] = s.blocks[p // BS] * BS + p % BS
            ctx[i] = p + 1
            bt[i, : len(s.blocks)] = s.blocks
        # plan on the real rows; padded rows (ctx 1) still get a one-key item
        # (sorted last) so every output row the graph produces is finite
        chain = self._decode_chain(decode)
        _, part = A.plan_decode_split(self._plan_ctx(ctx[:B], chain), self.model.nkv,
                                      max_parts=self._n_parts(self.max_context))
        if self.stats["graph_steps"] % 32 == 0:  # how often decode attention re-reads a shared KV block
            used = np.concatenate([s.blocks[: (s.n_cached + j + BS) // BS] for s, j in decode])
            self.stats["kv_read_blocks_sampled"] += used.size
            self.stats["kv_unique_blocks_sampled"] += np.unique(used).size
        if chain is not None:
            chain = np.concatenate([chain, np.zeros(Bb - B, dtype=bool)])
        items = A.build_decode_items(ctx, np.arange(Bb), part, chain, self._dec_gmax)
        n_items = items.shape[0]
        assert n_items <= self._max_items
        flat = np.concatenate([ids, pos, slots, ctx, bt.reshape(-1), np.array([n_items, part], np.int32),
                               items.reshape(-1).astype(np.int32)])
        sel = np.asarray(sample_idx if len(sample_idx) != B else [], dtype=np.int32)
        if self._chan is not None:
            from ..parallel.channel import FWD_GRAPH
            meta = np.array([B, Bb, part, n_items, mb], dtype=np.int32)
            self._chan.send(FWD_GRAPH, [meta, flat, sel] + ([spec[0]] if spec is not None else []))
        return self._graph_run(B, Bb, part, n_items, mb, flat, spec, sel)

    def _graph_run(self, B: int, Bb: int, part: int, n_items: int, mb: int, flat: np.ndarray, spec=None,
                   sel: Optional[np.ndarray] = None):
        """Upload a packed decode step into the static graph inputs (pinned
        staging, one async copy) and replay bucket ``Bb``'s graph (rank 0, and
        every TP worker from the channel's message).  ``spec`` = (src[B], tok):
        row i's input id is ``tok[src[i]]`` where ``src[i] >= 0``."""
        st = self._ensure_static()
        assert mb == self.max_blocks_per_seq
        if self._sim:
            self.sim_rows[Bb] = self.sim_rows.get(Bb, 0) + 1
        hi = st["host_i"] = st["host_i"] ^ 1
        if st["host_ev"][hi] is not None:
            st["host_ev"][hi].synchronize()  # its previous upload has long completed in practice
        host = st["host"][hi]
        hv = host.numpy()
        n = flat.size
        hv[:n] = flat
        if spec is not None:
            hv[n:n + B] = spec[0]
            n_src = n
            n += B
        n_sel = 0 if sel is None else sel.size
        if n_sel:  # rows that sample (tiny-chunk rows other than a chunk's last do not)
            hv[n:n + n_sel] = sel
            o_sel = n
            n += n_sel
        dev_flat = torch.empty(n, dtype=torch.int32, device=self.device)
        dev_flat.copy_(host[:n], non_blocking=True)
        self._trace_mark()
        ev = st["host_ev"][hi] = st["host_ev"][hi] or torch.cuda.Event(blocking=KNOBS.blocking_sync)
        ev.record()
        # the upload scattered into the graph's static inputs in one launch (csrc/kernels/norm_act.hip),
        # the speculative decode ids (spec) taken from the device tokens in the same launch; before a
        # capture too: its warm-up forwards read these ids
        from ..ops._lib import check, lib, stream_ptr
        tok = _spec_tok(spec) if spec is not None else None  # launches the previous step's sampling
        fused_spec = tok is not None and tok.dtype == torch.int32 and tok.is_contiguous()
        check(lib().k8s_unpack_step(dev_flat.data_ptr(), Bb, mb, n_items, st["ids"].data_ptr(), st["pos"].data_ptr(),
                                    st["slots"].data_ptr(), st["ctx"].data_ptr(), st["bt"].data_ptr(),
                                    st["n_items"].data_ptr(), st["items"].data_ptr(),
                                    dev_flat[n_src:].data_ptr() if fused_spec else None,
                                    tok.data_ptr() if fused_spec else None, B if fused_spec else 0,
                                    stream_ptr(dev_flat)), "unpack_step")
        if tok is not None and not fused_spec:
            self._apply_spec(st["ids"], dev_flat[n_src:n_src + B], tok)
        graph, out = self._capture(Bb, part)  # one graph per bucket: the plan's part size is read on the device
        graph.replay()
        if n_sel:
            return out.index_select(0, dev_flat[o_sel:o_sel + n_sel].long())
        return out[:B]
