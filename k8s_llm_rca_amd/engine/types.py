"""Engine data types: configuration, requests, per-thread sequences, and the
in-flight sampled step."""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch

from ..knobs import KNOBS
from ..ops import attention as A
from .structured import GrammarState

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
    __slots__ = ("seqs", "tok", "tok_host", "event", "t0", "status", "nf", "flag_seq")

    def __init__(self, seqs, tok, tok_host, event, t0, status=None, nf=None, flag_seq=0):
        self.seqs = seqs
        self.tok = tok            # [B] int32 on the device (feeds the next forward)
        self.tok_host = tok_host  # [B] int32 host copy (pinned on GPU), valid once `event` completes
        self.event = event
        self.t0 = t0
        self.status = status      # TP: pinned copy of the xGMI STATUS word, taken before the sampling
        self.nf = nf              # knob nonfinite_check: pinned copy of the per-layer non-finite flags
        self.flag_seq = flag_seq  # knob token_flag: the host flag reaches this value once tok_host is valid


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
    # sys.setswitchinterval while the engine thread runs (seconds; None keeps the
    # interpreter's 5 ms): the engine thread re-takes the GIL from the pipeline
    # threads after every device wait, and a step boundary it reaches late is GPU
    # idle.  0.5 ms, interleaved A/B at the 104-concurrency operating point
    # (profiles/r5/ab_gil104/): 4.703 / 4.655 -> 4.716 / 4.763 analyses/s, p50
    # 19.47 / 19.48 -> 19.15 / 19.19 s
    gil_switch_interval: Optional[float] = 0.0005
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
    # KV host tier (engine/kv_offload.py): GB of page-locked host memory that idle
    # threads' pages are swapped to instead of being dropped (0 = off; TP = 1)
    kv_host_gb: float = field(default_factory=lambda: _knob("kv_host_gb", 0.0))
    # swap idle threads out ahead of need while free + in-flight pool pages are
    # below this many (None: one max-size prefill step plus one full thread)
    kv_host_watermark: Optional[int] = None
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
    __slots__ = ("id", "tokens", "n_cached", "blocks", "req", "last_used", "bh", "host", "loading")

    def __init__(self, sid: int):
        self.id = sid
        self.tokens: List[int] = []
        self.n_cached = 0
        self.blocks: List[int] = []
        self.bh: List[int] = []  # chain keys of the leading full blocks (prefix table)
        self.req: Optional[Request] = None
        self.last_used = 0.0
        # KV host tier (engine/kv_offload.py): while swapped out, ``blocks`` is
        # empty and ``host`` holds the host slots of pages 0..len(host)-1 (the
        # first n_cached tokens); ``loading`` is the completion event of a
        # swap-in still on the copy stream (the sequence is not scheduled before)
        self.host: Optional[List[int]] = None
        self.loading = None

    @property
    def pending(self) -> int:
        return len(self.tokens) - self.n_cached
