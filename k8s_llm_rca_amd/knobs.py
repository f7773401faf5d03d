"""Every runtime switch of the framework, typed, in one place.

The engine's workload parameters live in :class:`engine.engine.EngineConfig`;
what is here are the implementation switches -- kernel choices kept for A/B,
debug and tracing hooks, the xGMI communicator's sizing -- that used to be
read from ~40 environment variables under three prefixes across ``ops/``,
``engine/``, ``parallel/`` and the HIP sources.  Now:

* one prefix, ``K8SRCA_``: the field ``pf_w8`` is ``K8SRCA_PF_W8``;
* the environment is read HERE only (the in-tree build's compiler and arch too:
  ``offload_arch``, ``hipcc``) (:func:`from_env`, once, at import);
  other modules read ``KNOBS.<field>`` or a module constant initialised from
  it;
* the switches the HIP launchers consult per launch (``NATIVE``) are pushed
  into the library through ``k8s_set_knob`` when it loads (``ops/_lib.py``)
  and whenever :func:`override` changes them, so an A/B in one process is
  ``with knobs.override(pf_w8=5): ...`` instead of editing ``os.environ``.

Names of the earlier prefixes (``K8S_RCA_*``, ``K8S_*``) are still honoured,
with a warning naming the new variable.  (Reference: the hard-coded settings
of ``/root/reference/test_all.py:21-22`` are what EngineConfig + this replace.)
"""
from __future__ import annotations

import contextlib
import dataclasses
import logging
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, Iterator, Optional

log = logging.getLogger(__name__)

PREFIX = "K8SRCA_"


def _f(default, doc: str, legacy: Optional[str] = None, native: Optional[int] = None, at_import: Optional[str] = None):
    """``at_import``: the module constant the knob is copied into when that
    module is imported (a per-call read would cost host time on the hot path);
    :func:`override` / :func:`set_knob` refuse such knobs -- changing
    ``KNOBS`` afterwards would silently do nothing."""
    return field(default=default, metadata={"doc": doc, "legacy": legacy, "native": native, "at_import": at_import})


@dataclass
class Knobs:
    # ---------------------------------------------------------------- GEMM dispatch (ops/linear.py)
    skinny: bool = _f(True, "skinny weight-streaming GEMM for M <= skinny_max_m decode projections",
                   at_import="ops.linear._enabled (ops.linear.set_skinny)")
    skinny_max_m: int = _f(16, "largest M the skinny GEMM takes without a dispatch-table entry",
                   at_import="ops.linear.SKINNY_MAX_M")
    skinny_rope: bool = _f(True, "RoPE + paged-KV-write epilogue on the skinny qkv GEMM",
                   at_import="ops.attention._skinny_rope")
    native_blaslt: bool = _f(True, "library GEMMs through the native hipBLASLt front end (not F.linear)",
                   at_import="ops.linear._native_lib_gemm")
    blaslt_algos: bool = _f(True, "pinned hipBLASLt solutions per M bucket (data/blaslt_algos_*.json)",
                            legacy="K8S_BLASLT_ALGOS")
    gemm_dispatch: bool = _f(True, "measured decode-GEMM dispatch table (data/gemm_dispatch_*.json)")
    gemm_dispatch_file: Optional[str] = _f(None, "alternate dispatch table (A/B of two measured tables)")
    gemm_tuning: bool = _f(False, "TunableOp table for torch GEMMs (ops/gemm_tuning.py)",
                           legacy="K8S_RCA_GEMM_TUNING")
    big_gemm: str = _f("1", "prefill GEMMs on gemm_big where measured faster; 0 off, 'all' everywhere it fits",
                   at_import="ops.linear._big_mode (ops.linear.set_big)")
    big_var: int = _f(1, "gemm_big schedule variant (1 ping-pong, 3 + setprio, 5/7 32x32 MFMA)",
                   at_import="ops.linear.BIG_PIPE")
    big_tail: bool = _f(True, "gemm_big split-tail (stream-K last wave) workspace",
                   at_import="ops.linear._big_tail (ops.linear.reserve_big_ws(dev, enable))")
    stream_silu: bool = _f(True, "SwiGLU epilogue on the decode stream GEMM's gate_up",
                   at_import="ops.linear._stream_silu")
    glds_hand: bool = _f(True, "hand-issued LDS reads in the LDS-DMA decode GEMM", native=0)
    # ---------------------------------------------------------------- attention (ops/attention.py)
    fuse_splitk: bool = _f(True, "split-K partials reduced inside the next RoPE/KV-write or add+RMSNorm",
                   at_import="ops.layer_exec._fuse_splitk / ops.attention._fuse_qkv")
    decode_group: bool = _f(True, "consecutive tokens of one sequence share multi-token decode items",
                            legacy="K8S_DECODE_GROUP",
                   at_import="ops.attention.DECODE_GROUP_TOKENS")
    decode_low_units: int = _f(512, "low-batch decode split: fewest keys per item keeping <= this many waves "
                                    "(ops/attention.py DECODE_LOW_UNITS; 0 = the makespan planner everywhere)",
                   at_import="ops.attention.DECODE_LOW_UNITS")
    decode_reduce_pre: bool = _f(True, "decode split-KV reduce: register-prefetch form for <= 16 partitions",
                                 native=1)
    decode_kv_nt: bool = _f(False, "non-temporal K/V loads in the decode attention stream (A/B: 5.6 % slower on "
                                   "the contract run's decode steps, profiles/r5/decode_nt/)", native=5)
    pf_w8: int = _f(6, "prefill attention kernel: 6 (default) / 5 / 4 / 2 8-wave variants, 0 the 4-wave pg64",
                    native=2)
    pf_merge16: bool = _f(True, "prefill split-KV merge at 16 B per lane for bf16 partials", native=3)
    pf_target_wgs: int = _f(512, "prefill split target (workgroups per launch)", legacy="K8S_PF_TARGET_WGS",
                   at_import="ops.attention.PF_TARGET_WGS")
    pf_overhead_pages: float = _f(8.0, "makespan split planner: fixed cost per work item in pages (0 = fixed target)",
                                  legacy="K8S_PF_OVERHEAD_PAGES",
                   at_import="ops.attention.PF_OVERHEAD_PAGES")
    pf_makespan_all: bool = _f(False, "makespan planner also for launches with enough tiles",
                               legacy="K8S_PF_MAKESPAN_ALL",
                   at_import="ops.attention.PF_MAKESPAN_ALL")
    # ---------------------------------------------------------------- native layer executor / TP
    layer_exec: bool = _f(True, "whole dense layer stack issued by one C call (ops/layer_exec.py)",
                   at_import="ops.layer_exec._enabled (ops.layer_exec.set_enabled)")
    nano_batch: bool = _f(False, "mixed steps as two layer stacks on two streams: decode rows (high-priority "
                                 "side stream) beside prefill rows (compute stream)",
                          at_import="ops.layer_exec._nano")
    norm_fuse: bool = _f(True, "steps of <= 4 rows: the RMSNorms ride in the qkv / gate_up GEMMs' prologues "
                               "(csrc/kernels/norm_prologue.h)",
                   at_import="ops.layer_exec._norm_fuse")
    tp_fused_norm: bool = _f(True, "TP all-reduce + residual add + RMSNorm in one launch",
                   at_import="ops.layer_exec._fuse_ar_norm")
    tp_push: bool = _f(False, "TP o/down GEMM epilogue stores into the all-reduce slots (push) wherever it fits "
                              "(default: where the init-time fabric tuning measured it faster)",
                   at_import="ops.layer_exec._tp_push")
    tp_autotune: bool = _f(True, "time one-/two-shot x staged/push per decode bucket at communicator init")
    tp_push_force: bool = _f(False, "test hook: route o/down through the stream GEMM wherever it fits",
                   at_import="ops.layer_exec._tp_push_force")
    custom_ar: bool = _f(True, "xGMI communicator for TP/EP collectives (0: RCCL)", legacy="K8S_RCA_CUSTOM_AR")
    ar_max_mb: int = _f(64, "xGMI buffer per rank in MiB (larger messages run in chunks of it)",
                        legacy="K8S_RCA_AR_MAX_MB")
    ar_fence_all: bool = _f(False, "all-reduce publish with a system fence in every wave (old form, A/B)",
                            native=4)
    # ---------------------------------------------------------------- MoE (models/moe.py)
    moe_glds_max_rows: int = _f(384, "MoE gate_up on the LDS-DMA strip kernel up to this many rows (0 off)",
                                legacy="K8S_MOE_GLDS_MAX_ROWS",
                   at_import="models.moe.MoE.GLDS_MAX_ROWS")
    moe_big: bool = _f(True, "MoE prefill experts on the grouped gemm_big (0: per-expert hipBLASLt)",
                   at_import="models.moe.MoE.BIG_PREFILL")
    # ---------------------------------------------------------------- engine hooks (engine/engine.py)
    prefill_min: Optional[int] = _f(None, "EngineConfig.prefill_min_tokens override")
    prefill_defer_rows: Optional[int] = _f(None, "EngineConfig.prefill_defer_min_rows override")
    prefill_defer_s: Optional[float] = _f(None, "EngineConfig.prefill_max_defer_s override")
    kv_host_gb: Optional[float] = _f(None, "EngineConfig.kv_host_gb override (KV host tier, GB pinned)")
    tiny_chunk_tokens: Optional[int] = _f(None, "EngineConfig.tiny_chunk_tokens override",
                                          legacy="K8S_TINY_CHUNK_TOKENS")
    shape_trace: Optional[str] = _f(None, "append every step's attention shapes to this JSONL file",
                                    legacy="K8S_RCA_SHAPE_TRACE")
    step_timing: bool = _f(False, "per-path host-issue vs GPU time of every forward", legacy="K8S_RCA_STEP_TIMING")
    step_trace: Optional[str] = _f(None, "JSONL of every forward: GPU start / end (timing events) and the host's "
                                         "enqueue time against its last token wait (step-boundary idle analysis)")
    switch_interval: Optional[float] = _f(None, "sys.setswitchinterval for the serving process (s)",
                                          legacy="K8S_RCA_SWITCH_INTERVAL")
    profile_engine: Optional[str] = _f(None, "cProfile of the engine thread dumped to this path",
                                       legacy="K8S_RCA_PROFILE_ENGINE")
    token_flag: bool = _f(True, "TP = 1: the engine waits for a step's sampled tokens by polling a pinned-host flag "
                                "a one-wave kernel sets after their copy (50 us sleeps), not spinning in "
                                "hipEventSynchronize: engine thread 66 -> 10 CPU-s per contract window, throughput "
                                "unchanged (profiles/r6/token_flag/)")
    blocking_sync: bool = _f(False, "host waits on the engine's token / staging / graph-mirror events block in the "
                                    "driver (hipEventBlockingSync) instead of spinning")
    nonfinite_check: bool = _f(False, "device-side non-finite flag on every layer's normed input (no host sync)")
    poison: bool = _f(False, "fill scratch / partial / KV buffers with NaN at allocation: a read of memory no "
                             "kernel wrote shows up as NaN (sampler NON_FINITE) instead of stale finite data")
    # ---------------------------------------------------------------- library / debug / process
    hip_lib: Optional[str] = _f(None, "alternate build of libk8srca_hip.so (compile-time A/Bs)")
    offload_arch: str = _f("gfx950", "hipcc --offload-arch of the in-tree build (_build.py); MI355X = gfx950")
    hipcc: str = _f("/opt/rocm/bin/hipcc", "HIP compiler driver of the in-tree build (_build.py)")
    autobuild: bool = _f(True, "build the HIP library on first use when it is missing")
    sync_debug: bool = _f(False, "synchronise + check after every native launch", legacy="K8S_RCA_SYNC_DEBUG",
                   at_import="ops._lib._SYNC_DEBUG")
    no_native: bool = _f(False, "do not load the C++ graph core (_graphcore)")
    roctx: bool = _f(False, "roctx ranges around tracing spans (rocprofv3 --marker-trace)")
    bind: bool = _f(True, "bind each rank to its GPU's NUMA-local CPU slice")
    torch_threads: Optional[int] = _f(None, "torch intra-op threads of a serving rank (default 1)")
    max_batch_tokens: int = _f(8192, "bench default for --max-batch-tokens")

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def env_name(name: str) -> str:
        return PREFIX + name.upper()

    @classmethod
    def from_env(cls, env: Optional[Dict[str, str]] = None) -> "Knobs":
        env = os.environ if env is None else env
        kw: Dict[str, Any] = {}
        for f in fields(cls):
            raw = env.get(cls.env_name(f.name))
            legacy = f.metadata.get("legacy")
            if raw is None and legacy and legacy in env:
                raw = env[legacy]
                log.warning("%s is deprecated: set %s", legacy, cls.env_name(f.name))
            if raw is not None:
                kw[f.name] = _parse(f, raw)
        return cls(**kw)

    def describe(self) -> Dict[str, Any]:
        """{env name: value} of every knob that differs from its default."""
        out = {}
        for f in fields(self):
            v = getattr(self, f.name)
            if v != f.default:
                out[self.env_name(f.name)] = v
        return out


def _parse(f: dataclasses.Field, raw: str):
    t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
    raw = raw.strip()
    if "bool" in t:
        return raw not in ("0", "", "false", "False", "no", "off")
    if "Optional" in t and raw == "":
        return None
    if "int" in t:
        return int(raw)
    if "float" in t:
        return float(raw)
    return raw


KNOBS = Knobs.from_env()

# knob -> slot of the native table (csrc/kernels/knobs.h)
NATIVE = {f.name: f.metadata["native"] for f in fields(Knobs) if f.metadata.get("native") is not None}


def push_native(L=None) -> None:
    """Copy the NATIVE knobs into the loaded HIP library (``k8s_set_knob``)."""
    if L is None:
        from .ops import _lib
        if _lib._lib is None:
            return  # pushed by lib() when it loads
        L = _lib._lib
    fn = getattr(L, "k8s_set_knob", None)
    if fn is None:
        return
    for name, slot in NATIVE.items():
        fn(slot, int(getattr(KNOBS, name)))


# knob -> the module constant it was copied into at import (changing
# such a knob in a running process has no effect, so it is refused)
AT_IMPORT = {f.name: f.metadata["at_import"] for f in fields(Knobs) if f.metadata.get("at_import")}


def _runtime_settable(name: str) -> None:
    if not hasattr(KNOBS, name):
        raise AttributeError(f"no knob {name!r}")
    if name in AT_IMPORT:
        raise ValueError(f"knob {name!r} is read once at import into {AT_IMPORT[name]}: set "
                         f"{Knobs.env_name(name)} before the process starts, or change that constant")


@contextlib.contextmanager
def override(**kw) -> Iterator[Knobs]:
    """Temporarily change knobs (tests, in-process A/B); native ones are pushed
    to the library on entry and restored on exit.  Knobs copied into a module
    constant at import (``AT_IMPORT``) raise ``ValueError``."""
    for k in kw:
        _runtime_settable(k)
    old = {k: getattr(KNOBS, k) for k in kw}
    for k, v in kw.items():
        setattr(KNOBS, k, v)
    if any(k in NATIVE for k in kw):
        push_native()
    try:
        yield KNOBS
    finally:
        for k, v in old.items():
            setattr(KNOBS, k, v)
        if any(k in NATIVE for k in kw):
            push_native()


def set_knob(name: str, value) -> None:
    """Set one knob for the rest of the process (a string is parsed like its
    environment variable); native knobs are pushed to the library.  Knobs
    copied into a module constant at import raise ``ValueError``."""
    _runtime_settable(name)
    f = {f.name: f for f in fields(Knobs)}[name]
    setattr(KNOBS, name, _parse(f, value) if isinstance(value, str) else value)
    if name in NATIVE:
        push_native()
