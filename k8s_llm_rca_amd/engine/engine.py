"""LLM engine: continuous batching over every active assistant run.

Scheduling model (one step = one forward over a flattened token batch):

* each conversation *thread* owns a :class:`Sequence` whose token list and KV
  pages persist across runs -> a new run only prefills the newly appended
  messages (per-thread prefix reuse; the reference re-sent the whole thread
  to GPT-4 on every run, ``openai_generic_assistant.py:45-51``);
* decode rows (one pending token) go first and use the split-KV decode kernel;
  prefill rows (new prompt text, or literal text forced by the grammar --
  "jump-forward") are chunked under ``max_batch_tokens`` and use the varlen
  prefill kernel in the same step;
* pure-decode steps replay a captured HIP graph per (batch bucket, KV
  partition bucket), so Python/launch overhead is paid once per step;
* sampling is one masked kernel over the logits rows (grammar allow-lists /
  bitmaps), then each row's grammar state advances on the host;
* when the KV pool runs dry, idle threads are evicted LRU (their tokens are
  kept and re-prefilled on their next run);
* full KV blocks written by a prefill are published in the pool's prefix
  table (``kv_cache.py``): a thread whose prompt starts with the same blocks
  -- the three assistants' system prompts and seeding messages are identical
  across every concurrent RCA pipeline -- attaches those pages instead of
  prefilling its own copy.

The engine runs in a background thread (:meth:`start`) or is stepped
explicitly (:meth:`step`); :meth:`submit` is thread-safe.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ..knobs import KNOBS
from ..models.config import ModelConfig, get_config
from ..ops import attention as A
from ..parallel.groups import ParallelContext, single
from .graph_runner import GraphRunnerMixin
from .kv_cache import KVPool
from .kv_manager import KVCacheManager
from .sampler import SamplerMixin
from .scheduler import SchedulerMixin
from .step_exec import StepExecMixin
from .structured import GrammarRuntime
from .tokenizer import get_tokenizer
from .types import PART_MIN, SPEC, EngineConfig, InFlight, Request, Sequence  # noqa: F401 (re-exported)

log = logging.getLogger(__name__)


def _build_model(mc: ModelConfig, device, dtype, pc, seed):
    if mc.arch == "opt":
        from ..models.opt import OPTModel
        return OPTModel(mc, device, dtype, seed=seed)
    from ..models.llama import LlamaModel
    return LlamaModel(mc, device, dtype, pc, seed=seed)


class LLMEngine(SchedulerMixin, StepExecMixin, GraphRunnerMixin, SamplerMixin):
    """The engine: lifecycle, submission API and state; scheduling
    (``scheduler.py``), step packing / execution (``step_exec.py``), HIP-graph
    decode (``graph_runner.py``) and sampling (``sampler.py``) are its mixins.
    The KV side is an object of its own: ``self.kvm`` (``kv_manager.py``) owns
    the page pool, the host tier and every allocation / eviction / swap /
    preemption / prefix-sharing policy, and touches only sequences' cache fields."""

    def __init__(self, cfg: EngineConfig, pc: Optional[ParallelContext] = None, model=None):
        self.cfg = cfg
        self.pc = pc or single()
        self.device = torch.device(cfg.device)
        t0 = time.perf_counter()
        if cfg.weights and model is None:
            from ..models.llama import LlamaModel
            from ..models.weights import config_from_hf, load_safetensors
            self.mc = config_from_hf(cfg.weights)
            model = LlamaModel(self.mc, self.device, cfg.dtype, self.pc, init=False)
            load_safetensors(model, cfg.weights)
        else:
            self.mc = get_config(cfg.model, **cfg.model_overrides)
        self.max_context = cfg.max_context or self.mc.max_position
        self.model = model or _build_model(self.mc, self.device, cfg.dtype, self.pc, cfg.seed)
        if hasattr(self.model, "logits_f32"):
            self.model.logits_f32 = cfg.logits_fp32
        self.gemm_dispatch = False
        if self.device.type == "cuda":
            from ..ops import gemm_tuning
            from ..ops import linear as LIN
            gemm_tuning.load(self.mc.name, self.pc.tp_size)
            from ..ops._lib import stream_ptr
            with torch.cuda.device(self.device):  # the engine's compute stream owns gemm_big's split tail
                LIN.reserve_lib_workspace(self.device, claim_stream=stream_ptr())
            self.lib_algos = LIN.load_lib_algos(LIN.lib_algos_path(self.mc.name, self.pc.tp_size))
            self.gemm_dispatch = LIN.load_dispatch(LIN.dispatch_path(self.mc.name, self.pc.tp_size))
            # prefill-size M ranges where the hand-written gemm_big beats hipBLASLt
            self.big_gemm_ranges = LIN.load_big(LIN.big_path(self.mc.name, self.pc.tp_size))
            if self.gemm_dispatch:  # split-K scratch exists before any HIP-graph capture
                LIN.reserve_dispatch_scratch(self.device)
            else:
                LIN.clear_dispatch()
        self.t_model_init = time.perf_counter() - t0
        tok_path = cfg.tokenizer
        if tok_path is None and cfg.weights and os.path.exists(os.path.join(cfg.weights, "tokenizer.json")):
            tok_path = os.path.join(cfg.weights, "tokenizer.json")
        self.tok = get_tokenizer(tok_path) if tok_path else get_tokenizer()
        self.vocab = min(self.mc.vocab_size, max(self.tok.vocab_size, 1))
        self.grt = GrammarRuntime(self.tok, self.mc.vocab_size)
        self.eos_ids = [self.tok.eot_id, self.tok.eos_id]
        BS = cfg.block_size
        nkv, D = self.model.nkv, self.model.D
        nb = cfg.num_blocks
        if nb is None:
            per = KVPool.bytes_per_block(self.mc.n_layers, nkv, D, BS)
            if self.device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(self.device)
                budget = free * cfg.kv_mem_fraction - self._workspace_bytes()
            else:
                budget = 2 << 30
            if cfg.kv_max_gb is not None:
                budget = min(budget, cfg.kv_max_gb * (1 << 30))
            nb = max(16, int(budget // per))
        self.kv = KVPool(self.mc.n_layers, nkv, D, nb, BS, self.device, cfg.dtype)
        # KV host tier: idle threads are swapped to page-locked host memory instead
        # of dropped (engine/kv_offload.py).  One engine per device: at TP > 1 the
        # ranks' pools would have to swap in lockstep, which the channel does not carry
        self.kv_host = None
        if cfg.kv_host_gb and cfg.kv_host_gb > 0:
            if self.pc.tp_size > 1:
                log.warning("kv_host_gb ignored at TP = %d (host tier is per-device, TP = 1 only)", self.pc.tp_size)
            else:
                from .kv_offload import KVHostTier
                per = KVPool.bytes_per_block(self.mc.n_layers, nkv, D, BS, self.kv.k.element_size())
                self.kv_host = KVHostTier(self.kv, max(1, int(cfg.kv_host_gb * (1 << 30) // per)))
        self.kv_watermark = (cfg.kv_host_watermark if cfg.kv_host_watermark is not None
                             else min(nb // 4, (cfg.max_batch_tokens + self.max_context) // BS + 2))
        self.max_blocks_per_seq = (self.max_context + BS - 1) // BS + 1
        self.seqs: Dict[int, Sequence] = {}
        self.kvm = None  # KVCacheManager: set below, once the stats dict exists
        self._next_sid = 0
        self._incoming: List[tuple] = []
        self._releases: List[int] = []
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self._mask_dev: Optional[torch.Tensor] = None
        self._mask_ver = -1
        self._graphs: Dict[tuple, tuple] = {}
        self._graph_pool = None
        self._static = None
        self._pf_ws = None  # prefill split-KV partials (allocated on first split step)
        # multi-token decode items (a short chunk's tokens read their shared keys
        # once): the decode MFMA's 16 rows hold G q heads per token
        G = getattr(self.model, "nq", 1) // max(1, getattr(self.model, "nkv", 1))
        self._dec_gmax = max(1, 16 // G) if A.DECODE_GROUP_TOKENS and G <= 16 else 1
        self._pending_sample = None  # (logits, seqs, rows): sampled at the start of the next step
        # TP: the leader's host work of step n overlaps step n+1 on every rank too
        # (the workers take the sampled tokens from their own device copy)
        self._chan = None
        self._sim = bool(getattr(self.pc, "sim", False))  # tp-sim: rank 0 alone, collectives stood in
        self.sim_rows: Dict[int, int] = {}  # tp-sim: forwards per row count (collective projection)
        if self.pc.tp_size > 1 and not self._sim:
            from ..parallel.channel import make_channel
            self._chan = make_channel(self.pc)  # host-side step metadata (parallel/channel.py)
        self.tp_tune = self._tune_collectives()
        self._last_tok = None  # TP workers: device tokens of the last sampling (decode inputs of the next step)
        # TP: exact vocab-parallel sampling (B10) instead of all-gathering logits
        self._dist_sample = (self.pc.tp_size > 1 and not self._sim and hasattr(self.model, "vocab_local")
                             and self.model.vocab_local % 8 == 0)
        # TP: every rank needs the sampled tokens on its device to overlap steps
        self._async = cfg.async_steps and (self.pc.tp_size == 1 or self._dist_sample or self._sim)
        # TP: the vocab-parallel sampler (its own object, tp_sampler.py)
        self.tps = None
        if self._dist_sample:
            from .tp_sampler import VocabParallelSampler
            self.tps = VocabParallelSampler(self.pc, self.device, self.vocab, self.model.vocab_local, self.grt,
                                            self._chan, self._to_dev)
        # knob shape_trace=path: append every step's attention shapes as JSON
        # lines (replayed by tools/bench_kernels.py --what replay)
        self._shape_trace = KNOBS.shape_trace
        # knob step_timing: per-path host-issue vs GPU time of the forward
        self._step_timing = KNOBS.step_timing
        self._pending_ev: list = []
        # knob step_trace=path: per-forward GPU start / end + host enqueue vs last token wait (JSONL)
        self._trace = KNOBS.step_trace
        self._trace_base = None
        self._trace_buf: list = []
        self._last_wait_end = None
        # knob token_flag: pinned host flag raised after each step's token copy (engine/sampler.py)
        self._tflag = None
        self._tflag_np = None
        self._tflag_seq = 0
        # debug (knob nonfinite_check): per-layer non-finite flags, read with each sampling
        self._nf = None
        if KNOBS.nonfinite_check and self.device.type == "cuda" and hasattr(self.model, "nf_flags"):
            self._nf = torch.zeros(self.mc.n_layers + 1, dtype=torch.int32, device=self.device)
            self.model.nf_flags = self._nf
        self.stats = {"steps": 0, "decode_steps": 0, "graph_steps": 0, "prefill_tokens": 0, "decode_tokens": 0,
                      "forced_tokens": 0, "sampled_tokens": 0, "forward_s": 0.0, "sample_s": 0.0, "host_s": 0.0,
                      "evictions": 0, "requests": 0, "decode_ctx_tokens": 0, "prefill_ctx_tokens": 0,
                      "prefill_attn_pairs": 0, "small_steps": 0, "small_rows": 0, "big_rows": 0,
                      "wait_s": 0.0, "post_s": 0.0, "admit_s": 0.0, "captures": 0, "capture_s": 0.0,
                      "eager_issue_s": 0.0, "eager_gpu_s": 0.0, "graph_issue_s": 0.0, "graph_gpu_s": 0.0,
                      "prefix_hit_tokens": 0, "prefill_deferred_steps": 0, "preemptions": 0, "cancelled": 0,
                      "nonfinite_rows": 0, "nonfinite_flag_steps": 0, "nonfinite_first_layer": -1,
                      # why requests ended: grammar (complete / budget), eos, no allowed token, length cap
                      "end_grammar": 0, "end_eos": 0, "end_no_allowed": 0, "end_cap": 0,
                      "timeouts": 0,
                      "recompute_tokens": 0, "kv_read_blocks_sampled": 0, "kv_unique_blocks_sampled": 0,
                      "tiny_chunk_tokens": 0, "swap_outs": 0, "swap_ins": 0}
        # where every thread's KV lives and what happens when HBM runs short (kv_manager.py)
        self.kvm = KVCacheManager(self.kv, self.kv_host, self.kv_watermark, self._snapshot, self.stats)
        self._cancels: List[int] = []
        self.error: Optional[BaseException] = None
        self._fault: Optional[str] = None  # a dead communicator: every later request fails at admission
        self._test_stall = False  # tests: a TP worker that receives steps but never executes them
        self._test_host_stall_s = 0.0  # tests: rank 0 sleeps between a step's message and its own launch
        self.comm_dead = False  # a TP worker whose own collective timed out: it stops executing steps

    def _tune_collectives(self) -> Optional[dict]:
        """TP on the xGMI communicator: time the row-parallel epilogue's forms
        (one-/two-shot x staged/push) per decode bucket on this fabric, with
        layer 0's real o / down weights, before any graph is captured
        (``XgmiAllReduce.tune``; knob ``tp_autotune``).  Every rank runs it in
        lockstep and gets the same plan; the report goes into the bench line."""
        car = self.pc.custom_ar if self.pc.tp_size > 1 and not self._sim else None
        if car is None or not hasattr(car, "tune") or not KNOBS.tp_autotune or self.device.type != "cuda":
            return None
        layers = getattr(self.model, "layers", None)
        if not layers or getattr(self.model, "moe", None) is not None:
            return None
        L0 = layers[0]
        buckets = sorted(set(self.cfg.graph_batch_sizes) | {384, 512, 1024, 2048, 4096})
        t0 = time.perf_counter()
        shapes = [("o", L0["wo"]), ("down", L0["w_down"])]
        rep = car.tune(shapes, L0["post_norm"], float(self.mc.rms_eps), buckets)
        log.info("xGMI epilogue plan tuned in %.1f s: %s", time.perf_counter() - t0,
                 {T: r["pick"] for T, r in rep.items()})
        # steps whose all-reduce does not fit the executor's buffer take the Python
        # path's row-chunked GEMM / all-reduce overlap: its depth AND transport (the
        # xGMI kernels vs RCCL) per bucket, timed here.  On a "nccl" group the
        # prefill-size buckets the executor carries are timed too, for the report
        # (RCCL measured against the xGMI kernels on the fabric);
        # the executor keeps its fused xGMI epilogue for them.
        H = int(L0["wo"].shape[0])
        big = [T for T in (1024, 2048, 4096, 8192, 16384)
               if T <= self.cfg.max_batch_tokens and (T * H * 2 + 4 * T > car.max_bytes or self.pc.rccl_ok())]
        ov = self.pc.tune_overlap(shapes, big) if big else {}
        for T, r in ov.items():
            r["executor"] = T * H * 2 + 4 * T <= car.max_bytes
        if ov:
            log.info("GEMM / all-reduce overlap tuned (depth, transport): %s",
                     {T: (r["pick"], r["transport"]) for T, r in ov.items()})
        return {"tune_s": round(time.perf_counter() - t0, 2), "buckets": rep, "overlap": ov}

    def _workspace_bytes(self) -> int:
        mc = self.mc
        t = self.cfg.max_batch_tokens
        act = t * (mc.hidden * 8 + (mc.q_size + 2 * mc.kv_size) * 2 + mc.intermediate * 6)
        if mc.n_experts:
            act += t * mc.top_k * (mc.hidden * 4 + mc.intermediate * 6)
        logits = self.cfg.max_decode_seqs * mc.vocab_size * 4
        return int(act + logits + (4 << 30))

    # ------------------------------------------------------------------ API
    def new_sequence(self) -> int:
        with self._lock:
            sid = self._next_sid
            self._next_sid += 1
            self.seqs[sid] = Sequence(sid)
        return sid

    def release_sequence(self, sid: int) -> None:
        """Drop a sequence and its KV.  Callable from any thread: the engine
        thread performs it (the KV pool is owned by the engine thread), after
        the sequence's active request, if any, has finished."""
        with self._cv:
            self._releases.append(sid)
            self._cv.notify()
        if self._thread is None:  # synchronous use (run_until_idle / tests)
            self._apply_releases()

    def _snapshot(self) -> List[Sequence]:
        with self._lock:
            return list(self.seqs.values())

    def submit(self, sid: int, tokens: List[int], grammar=None, max_new: int = 256,
               temperature: Optional[float] = None, seed: int = 0,
               on_done: Optional[Callable[[List[int], Dict[str, float]], None]] = None,
               top_k: int = 0, top_p: float = 1.0) -> None:
        """Set sequence ``sid``'s desired token list (prompt) and generate a reply
        (``top_k`` <= 0 and ``top_p`` >= 1 disable those filters)."""
        with self._cv:
            self._incoming.append((sid, list(tokens), grammar, max_new,
                                   self.cfg.temperature if temperature is None else temperature, seed, on_done,
                                   top_k, top_p))
            self._cv.notify()

    def cancel(self, sid: int) -> None:
        """Cancel sequence ``sid``'s active request (thread-safe): its run fails
        with "cancelled"; every other request is untouched.  The KV the
        request had written stays cached (the next run of the thread reuses
        the longest common prefix)."""
        with self._cv:
            self._cancels.append(sid)
            self._cv.notify()
        if self._thread is None:  # synchronous use: same rule as a step start
            ps = self._pending_sample
            self._apply_cancels(set(s.id for s in ps[1]) if ps is not None else set())

    def _fail_req(self, r: Request, err: str) -> None:
        s = r.seq
        s.req = None
        s.last_used = time.perf_counter()
        self.stats["cancelled"] += 1
        if r.on_done:
            r.on_done(None, {"error": err})

    def start(self) -> None:
        if self._thread is not None:
            return
        # The engine thread shares the GIL with the callers' pipeline threads;
        # CPython's default 5 ms switch interval can leave the GPU idle while
        # the engine waits to reacquire it after each device sync.
        si = float(KNOBS.switch_interval or self.cfg.gil_switch_interval or 0)
        if si > 0:
            import sys
            sys.setswitchinterval(si)
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self.kv_host is not None:
            self.kv_host.drain()
        if self._trace is not None:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
                if self._pending_ev:
                    self._collect_timing()
            self.flush_trace()

    def _loop(self) -> None:
        prof_path = KNOBS.profile_engine
        if prof_path:  # cProfile of the engine thread only (host turnaround analysis)
            import cProfile
            pr = cProfile.Profile()
            pr.enable()
            try:
                self._loop_inner()
            finally:
                pr.disable()
                pr.dump_stats(prof_path)
            return
        self._loop_inner()

    def _loop_inner(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            with self._cv:
                while (not self._stop and not self._incoming and not self._releases and not self._cancels
                       and not self._has_work()):
                    self._cv.wait(0.05)
                if self._stop:
                    return
            try:
                self.step()
            except BaseException as e:  # surface engine faults as failed runs, never a hang
                log.exception("engine step failed")
                self.error = e
                from ..parallel.xgmi import CommFault
                if isinstance(e, CommFault):
                    self._fault = repr(e)
                self._fail_all(repr(e))

    def _fail_all(self, err: str) -> None:
        self._pending_sample = None
        for s in self._snapshot():
            r = s.req
            if r is not None:
                s.req = None
                self.kvm.drop(s)
                if r.on_done:
                    r.on_done(None, {"error": err})

    def _has_work(self) -> bool:
        return any(s.req is not None for s in self.seqs.values())

    def run_until_idle(self, max_steps: int = 1_000_000) -> None:
        for _ in range(max_steps):
            if not self.step():
                return
