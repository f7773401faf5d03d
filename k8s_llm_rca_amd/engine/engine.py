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

import json
import logging
import math
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence as Seq, Tuple

import numpy as np
import torch

from ..knobs import KNOBS
from ..models.config import ModelConfig, get_config
from ..ops import attention as A
from ..ops import sampling as SMP
from ..ops._lib import scratch
from ..parallel.groups import ParallelContext, single
from ..utils import tracing
from .kv_cache import KVPool, chain_key
from .structured import GrammarRuntime, GrammarState
from .tokenizer import get_tokenizer

log = logging.getLogger(__name__)

PART_MIN = min(A.DECODE_PARTS)  # smallest decode partition: sizes the split-KV buffers
SPEC = -1  # placeholder token: "the token sampled by the in-flight step" (device-side until processed)


def _spec_tok(spec) -> torch.Tensor:
    tok = spec[1]
    return tok.tokens() if isinstance(tok, _LazySample) else tok


class _LazySample:
    """The previous step's sampling, launched on first use (inside the next
    forward, before its first kernel) or at the latest right after it."""
    __slots__ = ("eng", "ps", "infl")

    def __init__(self, eng, ps):
        self.eng, self.ps, self.infl = eng, ps, None

    def launch(self) -> "InFlight":
        if self.infl is None:
            self.infl = self.eng._launch_sample(*self.ps)
        return self.infl

    def tokens(self) -> torch.Tensor:
        return self.launch().tok


class InFlight:
    """A sampled step whose tokens have not been processed on the host yet."""
    __slots__ = ("seqs", "tok", "tok_host", "event", "t0", "status", "nf")

    def __init__(self, seqs, tok, tok_host, event, t0, status=None, nf=None):
        self.seqs = seqs
        self.tok = tok            # [B] int32 on the device (feeds the next forward)
        self.tok_host = tok_host  # [B] int32 host copy (pinned on GPU), valid once `event` completes
        self.event = event
        self.t0 = t0
        self.status = status      # TP: pinned copy of the xGMI STATUS word, taken before the sampling
        self.nf = nf              # knob nonfinite_check: pinned copy of the per-layer non-finite flags


def _knob(name: str, default):
    """An EngineConfig default with its knobs.py override (K8SRCA_<NAME>)."""
    v = getattr(KNOBS, name)
    return default if v is None else v


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    device: str = "cuda"
    dtype: torch.dtype = torch.bfloat16
    block_size: int = 64
    num_blocks: Optional[int] = None
    kv_mem_fraction: float = 0.85
    kv_max_gb: Optional[float] = None
    max_batch_tokens: int = 8192
    max_decode_seqs: int = 256
    # prompt prefill batching: while decode rows are running, a new run's prompt
    # waits (at most prefill_max_defer_s after its submit) until the waiting
    # prompts total prefill_min_tokens, so prefill GEMMs run at a larger M
    # (hipBLASLt per projection: ~900-1300 TFLOP/s at M = 1024 vs ~1300-1500 at
    # 2048, far less below 512) and fewer steps pay a full weight pass for a few
    # hundred prompt rows.  Jump-forward chunks of a running generation are never
    # held back.  Headline A/B, interleaved (profiles/r3/ab/prefill_min_*.json):
    # 0 -> 4.531 / 4.532, 2048 tokens within 0.1 s -> 4.580 / 4.552 analyses/s;
    # then 2048 / 0.1 s -> 4.544 / 4.593 vs 4096 / 0.3 s -> 4.606 / 4.601 (p50
    # 28.0 vs 28.1 s, TTFT p50 68 ms either way).
    # 0 disables
    prefill_min_tokens: int = field(default_factory=lambda: _knob("prefill_min", 4096))
    # ... only while at least this many decode rows run (a busy, throughput-bound
    # engine): at low concurrency a held prompt would only add its wait to the
    # run's latency
    prefill_defer_min_rows: int = field(default_factory=lambda: _knob("prefill_defer_rows", 96))
    prefill_max_defer_s: float = field(default_factory=lambda: _knob("prefill_defer_s", 0.3))
    # prefill chunks of at most this many tokens (grammar jump-forward runs) are
    # run as rows of the decode-attention work list (one row per token, its own
    # causal key count) instead of a prefill tile that walks every page for a
    # few rows and then needs a split-KV merge; 0 disables
    tiny_chunk_tokens: int = field(default_factory=lambda: _knob("tiny_chunk_tokens", 8))
    max_context: Optional[int] = None
    use_graphs: bool = True
    # overlap the host's token processing of step n with the GPU's forward of
    # step n+1 (decode inputs taken from the device-side sampled tokens)
    async_steps: bool = True
    prefix_sharing: bool = True  # attach other threads' published prompt pages (kv_cache.py)
    gil_switch_interval: Optional[float] = None  # seconds; None keeps the interpreter default
    graph_batch_sizes: Tuple[int, ...] = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256)
    seed: int = 0
    # a request running longer than this is cancelled by the engine (its run
    # fails alone, as the reference's expired runs do); None = no limit
    max_run_s: Optional[float] = None
    weights: Optional[str] = None    # HF checkpoint dir (config.json + *.safetensors): real weights
    tokenizer: Optional[str] = None  # tokenizer.json (default: the checkpoint's, else the built-in BPE)
    temperature: float = 0.7
    use_hints: bool = True
    logits_fp32: bool = True   # lm_head writes fp32 logits for the sampler
    model_overrides: dict = field(default_factory=dict)


class Request:
    __slots__ = ("seq", "gs", "max_new", "temperature", "seed", "on_done", "n_prompt", "generated", "mask",
                 "t_submit", "t_first", "n_forced", "n_sampled", "cancelled", "top_k", "top_p")

    def __init__(self, seq, gs, max_new, temperature, seed, on_done, n_prompt, top_k=0, top_p=1.0):
        self.seq = seq
        self.top_k = int(top_k or 0)
        self.top_p = float(1.0 if top_p is None else top_p)
        self.gs: GrammarState = gs
        self.max_new = max_new
        self.temperature = temperature
        self.seed = seed
        self.on_done = on_done
        self.n_prompt = n_prompt
        self.generated: List[int] = []
        self.mask = None
        self.t_submit = time.perf_counter()
        self.t_first = None
        self.n_forced = 0
        self.n_sampled = 0
        self.cancelled = False


class Sequence:
    __slots__ = ("id", "tokens", "n_cached", "blocks", "req", "last_used", "bh")

    def __init__(self, sid: int):
        self.id = sid
        self.tokens: List[int] = []
        self.n_cached = 0
        self.blocks: List[int] = []
        self.bh: List[int] = []  # chain keys of the leading full blocks (prefix table)
        self.req: Optional[Request] = None
        self.last_used = 0.0

    @property
    def pending(self) -> int:
        return len(self.tokens) - self.n_cached


def _build_model(mc: ModelConfig, device, dtype, pc, seed):
    if mc.arch == "opt":
        from ..models.opt import OPTModel
        return OPTModel(mc, device, dtype, seed=seed)
    from ..models.llama import LlamaModel
    return LlamaModel(mc, device, dtype, pc, seed=seed)


class LLMEngine:
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
            LIN.reserve_lib_workspace(self.device)
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
        self.max_blocks_per_seq = (self.max_context + BS - 1) // BS + 1
        self.seqs: Dict[int, Sequence] = {}
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
        self._last_tok = None  # TP workers: device tokens of the last sampling (decode inputs of the next step)
        # TP: exact vocab-parallel sampling (B10) instead of all-gathering logits
        self._dist_sample = (self.pc.tp_size > 1 and not self._sim and hasattr(self.model, "vocab_local")
                             and self.model.vocab_local % 8 == 0)
        # TP: every rank needs the sampled tokens on its device to overlap steps
        self._async = cfg.async_steps and (self.pc.tp_size == 1 or self._dist_sample or self._sim)
        self._mask_sent = 0      # rank 0: mask-table rows already broadcast to the workers
        self._wmask = None       # TP ranks: device copy of the mask table (rows received so far)
        # knob shape_trace=path: append every step's attention shapes as JSON
        # lines (replayed by tools/bench_kernels.py --what replay)
        self._shape_trace = KNOBS.shape_trace
        # knob step_timing: per-path host-issue vs GPU time of the forward
        self._step_timing = KNOBS.step_timing
        self._pending_ev: list = []
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
                      "tiny_chunk_tokens": 0}
        self._cancels: List[int] = []
        self.error: Optional[BaseException] = None
        self._fault: Optional[str] = None  # a dead communicator: every later request fails at admission
        self._test_stall = False  # tests: a TP worker that receives steps but never executes them
        self._test_host_stall_s = 0.0  # tests: rank 0 sleeps between a step's message and its own launch
        self.comm_dead = False  # a TP worker whose own collective timed out: it stops executing steps

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
                    self.kv.release(s.blocks)
                    s.blocks = []
                    s.bh = []
            self._releases = keep + self._releases

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
                s.n_cached = 0
                self.kv.release(s.blocks)
                s.blocks = []
                s.bh = []
                if r.on_done:
                    r.on_done(None, {"error": err})

    def _has_work(self) -> bool:
        return any(s.req is not None for s in self.seqs.values())

    def run_until_idle(self, max_steps: int = 1_000_000) -> None:
        for _ in range(max_steps):
            if not self.step():
                return

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
            BS = self.kv.block_size
            del s.bh[lcp // BS:]
            keep = (lcp + BS - 1) // BS
            if lcp % BS and keep <= len(s.blocks) and not self.kv.make_private(s.blocks[keep - 1]):
                # the history diverges inside a page other threads share: recompute it privately
                keep -= 1
                s.n_cached = keep * BS
            if len(s.blocks) > keep:
                self.kv.release(s.blocks[keep:])
                s.blocks = s.blocks[:keep]
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

    def _ensure_blocks(self, s: Sequence, upto: int, protect: set) -> bool:
        need = (upto + self.kv.block_size - 1) // self.kv.block_size - len(s.blocks)
        if need <= 0:
            return True
        if need > self.kv.free_blocks:
            self._evict(need - self.kv.free_blocks, protect)
        if need > self.kv.free_blocks:
            return False
        s.blocks.extend(self.kv.alloc(need))
        return True

    def _evict(self, n_blocks: int, protect: set) -> None:
        idle = sorted((s for s in self._snapshot() if s.req is None and s.blocks and s.id not in protect),
                      key=lambda s: s.last_used)
        freed = 0
        for s in idle:
            freed += self.kv.release(s.blocks)  # pages other threads still share stay resident
            s.blocks = []
            s.bh = []
            s.n_cached = 0
            self.stats["evictions"] += 1
            if freed >= n_blocks:
                return

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
        t_host0 = time.perf_counter()
        if self._cancels or self.cfg.max_run_s is not None:
            ps0 = self._pending_sample
            self._apply_cancels(set(s.id for s in ps0[1]) if ps0 is not None else set())
        self._admit()
        self.stats["admit_s"] += time.perf_counter() - t_host0
        if self._releases:
            self._apply_releases()
        # The previous forward's sampling is launched only now, AFTER this
        # step is scheduled, so sample(k) and forward(k+1) reach the GPU back
        # to back while it is still busy with forward(k): the host's
        # scheduling never leaves the GPU idle.
        ps = self._pending_sample
        self._pending_sample = None
        if ps is not None:
            for s in ps[1]:
                s.tokens.append(SPEC)
        active = [s for s in self._snapshot() if s.req is not None and s.pending > 0]
        if not active:
            if ps is not None:  # nothing else to run: just finish the pending sample
                for s in ps[1]:
                    s.tokens.pop()
                self._process_tokens(self._launch_sample(*ps))
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
                if self._ensure_blocks(s, s.n_cached + 1, protect) or self._preempt_for(s, s.n_cached + 1, placed,
                                                                                        protect, active):
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
                self._attach_prefix(s)
                q = min(s.pending, budget)
            if not (self._ensure_blocks(s, s.n_cached + q, protect)
                    or self._preempt_for(s, s.n_cached + q, placed, protect, active)):
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
                self._register_blocks(s)
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
                    del s.bh[p // self.kv.block_size:]
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

    def _preempt_for(self, s: Sequence, upto: int, placed: set, protect: set, active: List[Sequence]) -> bool:
        """Free KV for ``s`` by preempting younger active requests (youngest
        first; not ones already placed in this step): a victim keeps its
        request and tokens, drops its pages and is re-prefilled when pages
        are free again (recompute preemption).  False if ``s`` still does not fit."""
        for v in reversed(active):
            if v is s or v.req is None or v.id in placed or not v.blocks:
                continue
            if v.req.t_submit <= s.req.t_submit:
                break  # only younger requests yield to older ones
            self.kv.release(v.blocks)  # pages other threads share stay resident
            v.blocks = []
            v.bh = []
            v.n_cached = 0
            self.stats["preemptions"] += 1
            if self._ensure_blocks(s, upto, protect):
                return True
        return False

    def _attach_prefix(self, s: Sequence) -> None:
        """Map the next full blocks of ``s``'s prompt onto published pages
        (at least one token is left to prefill: it produces the logits)."""
        BS = self.kv.block_size
        toks = s.tokens
        parent = s.bh[-1] if s.bh else 0
        if len(s.bh) != len(s.blocks):  # chain keys of this thread's own leading pages first
            for j in range(len(s.bh), len(s.blocks)):
                parent = chain_key(parent, toks[j * BS:(j + 1) * BS])
                s.bh.append(parent)
        n = s.n_cached
        hit = 0
        while n + BS < len(toks):
            k = chain_key(parent, toks[n:n + BS])
            b = self.kv.lookup(k)
            if b is None:
                break
            s.blocks.append(b)
            s.bh.append(k)
            parent = k
            n += BS
            hit += 1
        if hit:
            s.n_cached = n
            self.stats["prefix_hit_tokens"] += hit * BS

    def _register_blocks(self, s: Sequence) -> None:
        BS = self.kv.block_size
        toks = s.tokens
        parent = s.bh[-1] if s.bh else 0
        for j in range(len(s.bh), s.n_cached // BS):
            parent = chain_key(parent, toks[j * BS:(j + 1) * BS])
            s.bh.append(parent)
            self.kv.register(s.blocks[j], parent)

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
        timed = self._step_timing and self.device.type == "cuda"
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
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
        dt = time.perf_counter() - t0
        self.stats["forward_s"] += dt
        if timed:
            ev[1].record()
            self._pending_ev.append((kind, dt, ev))
        return out

    def _graphs_ok(self) -> bool:
        """Decode steps replay HIP graphs at TP=1, and under TP when every
        all-reduce of a decode step runs on the capturable xGMI kernel."""
        if self.pc.tp_size == 1:
            return True
        car = self.pc.custom_ar
        return car is not None and getattr(car, "max_bytes", 0) >= max(self.cfg.graph_batch_sizes) * self.mc.hidden * 2

    def _collect_timing(self) -> None:
        """Fold completed step events into stats (with overlapped steps the
        newest forward may still be running: its events stay pending)."""
        keep = []
        for kind, dt, (e0, e1) in self._pending_ev:
            if not e1.query():
                keep.append((kind, dt, (e0, e1)))
                continue
            self.stats[kind + "_issue_s"] += dt
            self.stats[kind + "_gpu_s"] += e0.elapsed_time(e1) / 1e3
        self._pending_ev = keep

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
            n_parts, part = A.plan_decode_split(self._plan_ctx(ctx_d, chain), self.model.nkv)
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

    def _tp_sample(self, logits, mask_id, list_off, list_len, lists, seeds, steps, temps, topk, topp,
                   rows=None) -> torch.Tensor:
        """Rank 0: broadcast this step's sampling inputs (plus mask rows the
        workers have not seen), then sample on every rank's vocab shard."""
        import numpy as np_
        table = self.grt.masks.array() if self.grt.masks.rows else np_.zeros((0, self.grt.masks.words), np_.int32)
        new = table[self._mask_sent:]
        self._mask_sent = table.shape[0]
        B = mask_id.shape[0]
        hdr = np_.array([B, len(lists), new.shape[0], self.grt.masks.words], dtype=np_.int64)
        flat = np_.concatenate([mask_id, list_off, list_len, lists, seeds, steps, temps.view(np_.int32),
                                topk, topp.view(np_.int32), new.reshape(-1).astype(np_.int32)])
        from ..parallel.channel import SAMPLE
        rows_a = np_.asarray(rows if rows is not None else [], np_.int32)
        self._chan.send(SAMPLE, [hdr, flat, rows_a])
        return self._sample_rows(logits, hdr, flat, rows_a)

    def _sample_rows(self, logits, hdr, flat, rows_a) -> torch.Tensor:
        """Every TP rank: the rows of this step's logits that sample (all when
        ``rows_a`` is empty), then the vocab-parallel sampling."""
        B, L = int(hdr[0]), int(hdr[1])
        o = 3 * B + L + 3 * B  # the payload's top_k / top_p columns (host copy: no device read)
        topk_h = flat[o:o + B]
        topp_h = flat[o + B:o + 2 * B].view(np.float32)
        if rows_a.size:
            dev, rows_d = self._to_dev([flat, rows_a])
            logits = logits.index_select(0, rows_d.long())
        else:
            dev = self._to_dev([flat])[0]
        return self._sample_shard(logits, hdr, dev, topk_h, topp_h)

    def _sample_shard(self, logits, hdr, dev, topk_h: np.ndarray, topp_h: np.ndarray) -> torch.Tensor:
        """Every TP rank: masked Gumbel-max over its vocab shard, then an
        all-gather of the [B, 2] winners (a few bytes per row instead of the
        [B, vocab] logits).  Which rows filter is read from the host copy of
        the step's payload, so no rank waits for its GPU here.

        Filtered rows: a top-k row with ``k <= CAND_K`` (any top-p) is exact
        from the ranks' candidate lists -- its whole top-k set, and so its
        nucleus and the nucleus mass, is inside them.  Any other filtered row
        (top-p without such a k, or k > CAND_K) all-gathers its logits row and
        samples it with the single-device kernel over the full vocabulary
        (same global-id noise): a nucleus of flat logits can hold thousands of
        tokens per shard, more than any candidate list."""
        import torch.distributed as dist
        B, L, nr, words = (int(x) for x in hdr)
        o = 0

        def take(n):
            nonlocal o
            t = dev[o:o + n]
            o += n
            return t

        mask_id, list_off, list_len, lists, seeds, steps = (take(B), take(B), take(B), take(L), take(B), take(B))
        temps = take(B).view(torch.float32)
        topk = take(B)
        topp = take(B).view(torch.float32)
        rows = take(nr * words).view(nr, words)
        if nr:
            self._wmask = rows.clone() if self._wmask is None else torch.cat([self._wmask, rows])
        table = self._wmask if self._wmask is not None else torch.zeros(1, words, dtype=torch.int32,
                                                                         device=self.device)
        off = self.pc.tp_rank * self.model.vocab_local
        filt_h = (topk_h > 0) | (topp_h < 1.0)
        cand_h = filt_h & (topk_h > 0) & (topk_h <= SMP.CAND_K)
        full_h = np.flatnonzero(filt_h & ~cand_h)
        cdev = self._gather_device()
        if cand_h.any():
            pairs, cand = SMP.sample(logits, temps, seeds, steps, mask_id, table, list_off, list_len, lists,
                                     self.vocab, vocab_off=off, pairs=True, top_k=topk, top_p=topp, candidates=True)
            # one all-gather of [B, 2 + 3 * CAND_K] per rank: the Gumbel-max winner and,
            # for top-k rows, the shard's highest-v candidates (B10 distributed top-k)
            comm = torch.cat([pairs, cand.view(B, -1)], 1).to(cdev)
        else:
            comm = SMP.sample(logits, temps, seeds, steps, mask_id, table, list_off, list_len, lists, self.vocab,
                              vocab_off=off, pairs=True).to(cdev)
        g = self._all_gather(comm)
        if cand_h.any():
            tok = SMP.combine_shards(g[:, :, :2].contiguous(), g[:, :, 2:].reshape(self.pc.tp_size, B, -1, 3),
                                     self._h2d(cand_h, g.device), topk.to(g.device), topp.to(g.device))
        else:
            tok = SMP.combine_pairs(g[:, :, :2].contiguous())
        tok = tok.to(self.device)
        if full_h.size:
            tok[self._h2d(full_h.astype(np.int64), self.device)] = self._sample_gathered(
                logits, full_h, temps, seeds, steps, mask_id, table, list_off, list_len, lists, topk, topp)
        return tok

    def _sample_gathered(self, logits, rows_h, temps, seeds, steps, mask_id, table, list_off, list_len, lists,
                         topk, topp) -> torch.Tensor:
        """Rows ``rows_h``: all-gather their logits shards and sample them over
        the whole vocabulary with the single-device kernel (every rank computes
        the same tokens)."""
        import torch.distributed as dist
        idx = self._h2d(rows_h.astype(np.int64), self.device)
        shard = logits.index_select(0, idx).float().contiguous().to(self._gather_device())
        g = self._all_gather(shard)                         # [tp, rows, vocab_local]
        full = torch.cat(list(g.unbind(0)), 1).to(self.device)  # rank r holds columns [r * vocab_local, ...)

        def pick(t):
            return t.index_select(0, idx)
        return SMP.sample(full, pick(temps), pick(seeds), pick(steps), pick(mask_id), table, pick(list_off),
                          pick(list_len), lists, self.vocab, top_k=pick(topk), top_p=pick(topp))

    def _h2d(self, a: np.ndarray, device) -> torch.Tensor:
        """Host array -> ``device`` without a host sync (pinned, non-blocking)."""
        t = torch.from_numpy(np.ascontiguousarray(a))
        if device.type == "cuda":
            return t.pin_memory().to(device, non_blocking=True)
        return t

    def _gather_device(self):
        """Where the sampler's per-rank winners are gathered: on the device
        through the xGMI all-to-all when the TP group has one (no host sync,
        HIP-graph capturable), else on the group's backend device."""
        car = self.pc.custom_ar
        if car is not None and self.device.type == "cuda":
            return self.device
        return self._comm_device()

    def _all_gather(self, comm: torch.Tensor) -> torch.Tensor:
        """[tp, *comm.shape]: every TP rank's ``comm``."""
        import torch.distributed as dist
        car = self.pc.custom_ar
        if car is not None and comm.is_cuda:  # device-side xGMI all-gather, any size (buffer-sized pieces)
            return car.all_gather(comm)
        parts = [torch.empty_like(comm) for _ in range(self.pc.tp_size)]
        dist.all_gather(parts, comm, group=self.pc.tp_group)
        return torch.stack(parts)

    def _comm_device(self):
        """Device of the sampling all-gather's tensors: RCCL takes device
        tensors; a gloo TP group (CPU tests, processes sharing one GPU) host ones."""
        if self.device.type != "cuda":
            return torch.device("cpu")
        import torch.distributed as dist
        return self.device if dist.get_backend(self.pc.tp_group) == "nccl" else torch.device("cpu")

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
        return self._exec_step(header, flat, dev, spec)

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
                self._last_tok = self._sample_rows(logits, hdr, flat, rows_a)
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
        _, part = A.plan_decode_split(self._plan_ctx(ctx[:B], chain), self.model.nkv)
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
        ev = st["host_ev"][hi] = st["host_ev"][hi] or torch.cuda.Event()
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

    # ------------------------------------------------------------ sampling
    def _mask_table(self) -> Optional[torch.Tensor]:
        if self._mask_ver != self.grt.masks.version:
            arr = self.grt.masks.array()
            host = torch.from_numpy(arr)
            if self.device.type == "cuda":  # pinned + non-blocking: a pageable copy would wait for the GPU
                host = host.pin_memory()
            self._mask_dev = host.to(self.device, non_blocking=True)
            self._mask_ver = self.grt.masks.version
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
            tok = self._tp_sample(logits, mask_id, list_off, list_len, np.asarray(lists, np.int32),
                                  seeds, steps, temps, topk, topp, rows)
        else:
            table = self._mask_table()
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
        if tok.is_cuda:
            host = torch.empty(B, dtype=torch.int32, pin_memory=True)
            host.copy_(tok, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = tok, None
        self.stats["sample_s"] += time.perf_counter() - t0
        return InFlight(seqs, tok, host, ev, t0, status, nf)

    def _process_tokens(self, fl: InFlight, placeholders: bool = False) -> List[int]:
        """Host side of a sampled step: wait for its tokens (not for later GPU
        work), append them, advance grammars, jump-forward, finish requests.
        ``placeholders``: the sequences carry a SPEC token that the sampled
        token replaces."""
        t1 = time.perf_counter()
        if fl.event is not None:
            fl.event.synchronize()
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
