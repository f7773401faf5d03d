"""Projection GEMMs: hand-written skinny MFMA GEMM for decode shapes, hipBLASLt otherwise."""
from __future__ import annotations

import json
import os
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

from ..knobs import KNOBS
from ._lib import check, lib, ptr, scratch, stream_ptr

SKINNY_MAX_M = KNOBS.skinny_max_m
# measured on MI355X (tools/bench_kernels.py): the skinny kernel beats hipBLASLt
# ~2x on the small-N decode projections (o_proj / QKV) for M <= 16 and ties or
# loses on the wide ones; beyond M = 16 its L2-read X operand is the bottleneck.
SKINNY_MAX_NK = 8192 * 4096
_enabled = KNOBS.skinny


def set_skinny(enabled: bool) -> None:
    global _enabled
    _enabled = enabled


KIND_LIB, KIND_SKINNY, KIND_MID, KIND_GRP, KIND_STREAM, KIND_BIG = 0, 1, 2, 3, 4, 5


def select_gemm(M: int, N: int, K: int, x_ok_layout: bool = True, out_contig: bool = True) -> Tuple[int, int, int]:
    """(kind, cfg, splits) :func:`linear` runs for a contiguous bf16 ``x`` [M, K]
    and ``w`` [N, K] on the GPU -- the measured dispatch table first, then the
    skinny kernel's default range, else hipBLASLt.  Also used by the native
    layer executor (ops/layer_exec.py) so both paths pick the same kernel."""
    forced_skinny = False
    if _dispatch and M <= DISPATCH_MAX_M:
        ent = _lookup(N, K, M)
        if ent is not None:
            kind, cfg, splits = ent
            if kind == "mid" and x_ok_layout and _mid_shape_ok(M, N, K, cfg, splits):
                return KIND_MID, cfg, splits
            if kind == "grp" and x_ok_layout and out_contig and N % 128 == 0 and K % (64 * splits) == 0:
                return KIND_GRP, 0, splits
            if kind == "stream" and x_ok_layout and out_contig and stream_shape_ok(M, N, K, cfg, splits):
                return KIND_STREAM, cfg, splits
            if kind == "lib":
                return KIND_LIB, 0, 1
            forced_skinny = kind == "skinny" and M <= 128
    if M > DISPATCH_MAX_M and x_ok_layout:
        big_splits = _big_pick(M, N, K)
        if big_splits:
            return KIND_BIG, BIG_PIPE, big_splits
    if (_enabled and (M == 1 or forced_skinny or (M <= SKINNY_MAX_M and N * K <= SKINNY_MAX_NK))
            and x_ok_layout and K % 256 == 0 and N % 16 == 0):
        return KIND_SKINNY, 0, 1
    return KIND_LIB, 0, 1


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """``x @ w.T`` for ``x`` [M, K] and ``w`` [N, K] (bf16)."""
    M, K = x.shape
    N = w.shape[0]
    if not (x.is_cuda and x.dtype == torch.bfloat16):
        return lib_gemm(x, w, out)
    layout = x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous()
    kind, cfg, splits = select_gemm(M, N, K, layout, out is None or out.is_contiguous())
    if kind == KIND_MID:
        return gemm_mid(x, w, cfg, splits, out)
    if kind == KIND_GRP:
        return gemm_grp(x, w, splits, out)
    if kind == KIND_STREAM:
        return gemm_stream(x, w, cfg, splits, out)
    if kind == KIND_BIG:
        return gemm_big(x, w, out, pipe=cfg, splits=splits)
    if kind == KIND_SKINNY:
        if out is None:
            out = torch.empty((M, N), dtype=x.dtype, device=x.device)
        check(lib().k8s_gemm_skinny(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K,
                                    stream_ptr(x)), "gemm_skinny")
        return out
    return lib_gemm(x, w, out)


# ------------------------------------------------------------ library GEMM
# Native hipBLASLt front end (csrc/kernels/blaslt.hip): descriptors and the
# heuristic's algorithm cached per shape, so a call costs a hash lookup plus
# hipblasLtMatmul instead of F.linear's ~28 us of host time.
BLASLT_WS_BYTES = 64 << 20
_blaslt_ws = {}
_native_lib_gemm = KNOBS.native_blaslt


def lib_gemm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """``x @ w.T`` on hipBLASLt (bf16, fp32 accumulate)."""
    if (_native_lib_gemm and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.stride(1) == 1 and w.is_contiguous() and (out is None or out.stride(1) == 1)):
        M, K = x.shape
        N = w.shape[0]
        if out is None:
            out = torch.empty((M, N), dtype=x.dtype, device=x.device)
        if M == 0:
            return out
        ws = _blaslt_ws.get(x.device)
        if ws is None:
            ws = _blaslt_ws[x.device] = torch.empty(BLASLT_WS_BYTES, dtype=torch.uint8, device=x.device)
        check(lib().k8s_blaslt_gemm(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, ptr(ws),
                                    BLASLT_WS_BYTES, stream_ptr(x)), "blaslt_gemm")
        return out
    if out is None:
        return F.linear(x, w)
    return torch.matmul(x, w.t(), out=out)


def linear_f32out(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x @ w.T`` with fp32 output (bf16 operands, fp32 accumulate): the
    lm_head, whose logits the sampler reads in fp32."""
    if x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(1) == 1 \
            and w.is_contiguous():
        M, K = x.shape
        N = w.shape[0]
        out = torch.empty((M, N), dtype=torch.float32, device=x.device)
        if M == 0:  # a step whose chunks all end mid-prompt samples no row
            return out
        ws = _blaslt_ws.get(x.device)
        if ws is None:
            ws = _blaslt_ws[x.device] = torch.empty(BLASLT_WS_BYTES, dtype=torch.uint8, device=x.device)
        check(lib().k8s_blaslt_gemm2(ptr(x), x.stride(0), ptr(w), ptr(out), N, M, N, K, ptr(ws), BLASLT_WS_BYTES,
                                     stream_ptr(x), 1), "blaslt_gemm_f32out")
        return out
    return x.float() @ w.float().t()


def reserve_lib_workspace(dev: torch.device, claim_stream: int = None) -> None:
    """Allocate the hipBLASLt workspace (and gemm_big's split-tail workspace)
    before any HIP-graph capture.  ``claim_stream`` (a raw hipStream_t): the
    stream that owns the split tail (the engine's compute stream)."""
    if dev not in _blaslt_ws:
        _blaslt_ws[dev] = torch.empty(BLASLT_WS_BYTES, dtype=torch.uint8, device=dev)
    reserve_big_ws(dev)
    if claim_stream is not None and dev in _big_ws and _big_tail:
        with torch.cuda.device(dev):
            check(lib().k8s_gemm_big_claim_ws(claim_stream), "gemm_big_claim_ws")


def big_tail_foreign(dev: torch.device) -> int:
    """gemm_big launches on ``dev`` that ran without the split tail because
    another stream owns its workspace (reported in the bench line)."""
    if torch.device(dev).type != "cuda":
        return 0
    with torch.cuda.device(dev):
        return int(lib().k8s_gemm_big_tail_foreign())


_big_ws: Dict[torch.device, torch.Tensor] = {}
_big_tail = KNOBS.big_tail


def reserve_big_ws(dev: torch.device, enable: bool = None) -> None:
    """gemm_big's split-tail workspace on ``dev`` (csrc/kernels/gemm_big.hip:
    256 fp32 partial tiles + tickets, zeroed once): without it the kernel runs
    a partial last wave of whole tiles.  ``enable=False`` unregisters it (A/B).

    One workspace per device, so gemm_big launches must not overlap in time on
    that device: two in flight would mix their partial tiles and tickets.  The
    engine issues every projection on its one compute stream (the TP overlap's
    side stream carries only collectives, ``parallel/groups.py``); a second
    stream issuing gemm_big needs its own workspace or an event between them."""
    dev = torch.device(dev)
    if dev.type != "cuda":
        return
    on = _big_tail if enable is None else enable
    with torch.cuda.device(dev):
        if not on:
            check(lib().k8s_gemm_big_set_ws(None), "gemm_big_set_ws")
            return
        t = _big_ws.get(dev)
        if t is None:
            t = _big_ws[dev] = torch.zeros(lib().k8s_gemm_big_ws_bytes(), dtype=torch.uint8, device=dev)
        check(lib().k8s_gemm_big_set_ws(ptr(t)), "gemm_big_set_ws")


# ------------------------------------------------ hipBLASLt solution tables
# (Engine-init tuning of hipBLASLt solutions over an M ladder lost 4 % end to
# end -- profiles/r1_blaslt_tune_8b.txt -- and was retired in round 4; the
# bucketed table below, verified per bucket, stays.)


def projection_shapes(mc, tp: int = 1) -> List[Tuple[int, int]]:
    """(N, K) of the dense projections hipBLASLt runs at prefill M (per TP rank)."""
    H, I = mc.hidden, mc.intermediate
    qkv = (mc.n_heads + 2 * mc.n_kv_heads) * mc.head_dim // tp
    out = [(qkv, H), (H, mc.n_heads * mc.head_dim // tp)]
    if not getattr(mc, "n_experts", 0):
        out += [(2 * I // tp, H), (H, I // tp)]
    return out


def lib_algos_path(model: str, tp: int = 1) -> str:
    return os.path.join(DATA_DIR, f"blaslt_algos_{model}" + (f"-tp{tp}" if tp > 1 else "") + ".json")


def load_lib_algos(path: str) -> int:
    """Register the measured hipBLASLt solutions of ``path`` with the native
    front end; returns how many were accepted.  ON by default
    (K8S_BLASLT_ALGOS=0 disables it).

    The file's ``buckets`` (tools/blaslt_tune_buckets.py) hold, per (N, K),
    ``[lo, hi, solution]`` rows: a solution is used for M in [lo, hi] only,
    and was kept only where, registered and re-timed on this call path with
    cold weights, it was no slower than the heuristic's own choice at lo, mid
    and hi and >= 3 % faster over the three -- 14 of 76 buckets, mostly where
    the heuristic's pick misfires just above a tile boundary (down M = 1537:
    328 -> 177 us).  Replayed on 811 recorded prefill-size steps: 11.68 ->
    11.46 s (profiles/r2_blaslt_buckets/).  The older one-point ``algos``
    ladder (tools/blaslt_sweep.py) picked winners of noisy sweeps and applied
    them up to the next ladder point; it measured slower (profiles/r2_blaslt_ab/)
    and is still read for other models' files.  No-op without the native
    library GEMM."""
    if not _native_lib_gemm or not KNOBS.blaslt_algos or not os.path.exists(path):
        return 0
    with open(path) as f:
        d = json.load(f)
    n = 0
    for key, ladder in d.get("algos", {}).items():
        N, K = (int(v) for v in key.split(","))
        for M, idx in sorted(ladder.items(), key=lambda kv: int(kv[0])):
            if lib().k8s_blaslt_set_algo(int(M), N, K, int(idx)) == 0:
                n += 1
    # bucketed form (tools/blaslt_tune_buckets.py): [lo, hi, solution] per (N, K),
    # each verified on the engine's own call path at the bucket's ends and middle
    for key, rows in d.get("buckets", {}).items():
        N, K = (int(v) for v in key.split(","))
        for lo, hi, idx in rows:
            if lib().k8s_blaslt_set_algo_range(int(lo), int(hi), N, K, int(idx)) == 0:
                n += 1
    return n


def clear_lib_tuning() -> None:
    lib().k8s_blaslt_clear_tuning()


# ------------------------------------------------------- measured dispatch
# data/gemm_dispatch_<model>.json (tools/gemm_mid_sweep.py --emit): for each
# (N, K) projection, per M bucket, the fastest of hipBLASLt / skinny / a
# gemm_mid variant measured on MI355X with cold (per-layer) weights.  An M
# between buckets uses the next bucket up (every listed kernel handles any M
# up to its bucket).
DISPATCH_MAX_M = 256
_dispatch: Dict[Tuple[int, int], List[tuple]] = {}


DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def dispatch_path(model: str, tp: int = 1) -> str:
    override = KNOBS.gemm_dispatch_file  # A/B of two measured tables
    if override:
        return override
    return os.path.join(DATA_DIR, f"gemm_dispatch_{model}" + (f"-tp{tp}" if tp > 1 else "") + ".json")


def load_dispatch(path: str) -> bool:
    global _dispatch
    if not os.path.exists(path) or not KNOBS.gemm_dispatch:
        return False
    with open(path) as f:
        d = json.load(f)
    tab = {}
    for key, rows in d["shapes"].items():
        fused = key.startswith("silu:")
        n, k = (int(v) for v in key.split(":")[-1].split(","))
        tab[("silu", n, k) if fused else (n, k)] = sorted((int(r["m"]), r["kind"], int(r.get("cfg", -1)), int(r.get("splits", 1))) for r in rows)
    _dispatch = tab
    return True


def clear_dispatch() -> None:
    _dispatch.clear()


def dispatch_table() -> Dict[Tuple[int, int], List[tuple]]:
    return _dispatch


def _lookup(N: int, K: int, M: int, silu: bool = False):
    rows = _dispatch.get(("silu", N, K) if silu else (N, K))
    if not rows:
        return None
    for m, kind, cfg, splits in rows:
        if M <= m:
            return kind, cfg, splits
    return None


def _mid_shape_ok(M: int, N: int, K: int, cfg: int, splits: int) -> bool:
    mt, nt, nw, _, silu = mid_configs()[cfg]
    return not silu and M <= 16 * mt and N % (16 * nt * nw) == 0 and K % (64 * splits) == 0


def _mid_ok(x: torch.Tensor, w: torch.Tensor, cfg: int, splits: int) -> bool:
    mt, nt, nw, _, silu = mid_configs()[cfg]
    M = x.shape[0]
    N, K = w.shape
    return (x.dtype == torch.bfloat16 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous()
            and x.shape[1] == (2 * K if silu else K) and M <= 16 * mt and N % (16 * nt * nw) == 0
            and K % (64 * splits) == 0)


_offs_cache = {}


def _grp_ok(x: torch.Tensor, w: torch.Tensor, splits: int) -> bool:
    N, K = w.shape
    return (x.dtype == torch.bfloat16 and x.stride(1) == 1 and w.is_contiguous() and x.shape[1] == K
            and N % 128 == 0 and K % (64 * splits) == 0)


def grp_offsets(dev: torch.device, M: int) -> torch.Tensor:
    """Device [0, M] expert offsets of a single-expert grouped GEMM: a row of
    one table uploaded once per device (a per-M ``torch.tensor`` upload is a
    pageable copy that waits for every queued kernel -- a GPU bubble each
    time a new M shows up mid-run)."""
    tab = _offs_cache.get(dev)
    if tab is None:
        rows = torch.arange(DISPATCH_MAX_M + 1, dtype=torch.int32)
        tab = torch.stack([torch.zeros_like(rows), rows], 1)
        tab = _offs_cache[dev] = tab.to(dev)
    if M <= DISPATCH_MAX_M:
        return tab[M]
    key = (dev, M)
    offs = _offs_cache.get(key)
    if offs is None:
        offs = _offs_cache[key] = torch.tensor([0, M], dtype=torch.int32, device=dev)
    return offs


def gemm_grp(x: torch.Tensor, w: torch.Tensor, splits: int, out: torch.Tensor = None) -> torch.Tensor:
    """``x @ w.T`` on the grouped-GEMM kernel with a single expert (64 x 128
    tiles through swizzled LDS, split-K partials + reduce): the structure that
    streams the MoE down projection at 5.8 TB/s, applied to dense shapes."""
    from . import moe as MO
    M = x.shape[0]
    offs = grp_offsets(x.device, M)
    if out is None:
        out = torch.empty((M, w.shape[0]), dtype=x.dtype, device=x.device)
    return MO.grouped_gemm(x, w.view(1, *w.shape), offs, out=out, splits=splits)


def gemm_stream(x: torch.Tensor, w: torch.Tensor, cfg: int = 8, splits: int = 1,
                out: torch.Tensor = None) -> torch.Tensor:
    """``x @ w.T`` on the W-shared decode kernel (csrc/kernels/gemm_stream.hip):
    a workgroup's 4 waves split the rows of a 64-column strip, W is staged once
    through swizzled LDS, X goes L2 -> registers; ``cfg`` = W register ring
    depth (4 / 8), K split over ``splits`` workgroups (fp32 partials + reduce)."""
    M = x.shape[0]
    N, K = w.shape
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    part = _scratch(x.device, splits * M * N) if splits > 1 else None
    check(lib().k8s_gemm_stream(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, cfg, splits,
                                ptr(part), stream_ptr(x)), "gemm_stream")
    return out


BIG_PIPE = KNOBS.big_var  # schedule variant (gemm_big.hip: 1 = ping-pong)
# Prefill-size dispatch between gemm_big and hipBLASLt: per (N, K) the M ranges
# where the hand-written kernel measured faster, each with its K split count
# (data/gemm_big_<model>.json, tools/big_gemm_ab.py --emit), separately for the
# SwiGLU-fused gate_up form (against hipBLASLt + silu_mul).
# K8SRCA_BIG_GEMM=0 disables it; K8SRCA_BIG_GEMM=all uses gemm_big (no K split)
# for every shape it accepts above DISPATCH_MAX_M (A/B runs).
_big_mode = KNOBS.big_gemm
_big_ranges: Dict[Tuple, List[Tuple[int, int, int]]] = {}


def big_path(model: str, tp: int = 1) -> str:
    return os.path.join(DATA_DIR, f"gemm_big_{model}" + (f"-tp{tp}" if tp > 1 else "") + ".json")


def load_big(path: str) -> int:
    """Register the measured gemm_big M ranges of ``path``; returns how many."""
    _big_ranges.clear()
    if _big_mode == "0" or not os.path.exists(path):
        return 0
    with open(path) as f:
        d = json.load(f)
    n = 0
    for tag in ("ranges", "silu", "rope"):
        for key, rows in d.get(tag, {}).items():
            N, K = (int(v) for v in key.split(","))
            parsed = [(int(r[0]), int(r[1]), int(r[2]) if len(r) > 2 else 1) for r in rows]
            if tag != "ranges" and any(s != 1 for _, _, s in parsed):
                # the SwiGLU / RoPE epilogue forms have no split-K variant
                raise ValueError(f"{path}: {tag} row for {key} carries splits > 1")
            _big_ranges[(tag, N, K) if tag != "ranges" else (N, K)] = parsed
            n += len(rows)
    return n


def rope_choice(M: int, N: int, K: int) -> bool:
    """The qkv projection of M rows on gemm_big with its RoPE + paged KV-write
    epilogue (data file table ``rope``: measured against hipBLASLt +
    k8s_rope_kv)?  ``K8SRCA_BIG_GEMM=all`` takes it wherever the shape fits."""
    if _big_mode == "0" or M <= DISPATCH_MAX_M or not big_shape_ok(M, N, K):
        return False
    if _big_mode == "all":
        return True
    return any(lo <= M <= hi for lo, hi, _ in _big_ranges.get(("rope", N, K), ()))


def gemm_big_rope(x: torch.Tensor, w: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                  slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, nq: int, nkv: int,
                  out: torch.Tensor = None, pipe: int = None) -> torch.Tensor:
    """``qkv = x @ w.T`` with q, k rotated and k, v written to their pages in
    the GEMM's epilogue (csrc/kernels/gemm_big.hip MODE 2): bit-identical to
    :func:`gemm_big` + ``ops.attention.rope_kv_write``, one launch and one
    pass over qkv fewer."""
    M, K = x.shape
    N = w.shape[0]
    assert N == (nq + 2 * nkv) * 128 and big_shape_ok(M, N, K) and x.stride(1) == 1 and w.is_contiguous()
    assert positions.dtype == torch.int32 and cos_sin.dtype == torch.float32
    assert slots is None or slots.dtype == torch.int32
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    if M == 0:
        return out
    if x.device not in _big_ws and _big_tail:
        reserve_big_ws(x.device)
    BS = k_cache.shape[2]
    check(lib().k8s_gemm_big_rope(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, ptr(positions),
                                  ptr(cos_sin), ptr(slots), ptr(k_cache), ptr(v_cache), nq, nkv, BS,
                                  BIG_PIPE if pipe is None else pipe, stream_ptr(x)), "gemm_big_rope")
    return out


def big_scratch_elems() -> int:
    """fp32 elements of split-K partials the loaded gemm_big ranges can need
    (the gemm_mid scratch, reserved before any capture)."""
    need = 0
    for key, rows in _big_ranges.items():
        if isinstance(key[0], str):  # ("silu" / "rope", N, K): no split-K form (load_big rejects splits > 1)
            continue
        for lo, hi, splits in rows:
            if splits > 1:
                need = max(need, min(hi, 8192) * key[0] * splits)
    return need


def set_big(mode: str) -> None:
    global _big_mode
    _big_mode = mode


def _big_pick(M: int, N: int, K: int, silu: bool = False) -> int:
    """K splits of gemm_big for this (M, N, K), 0 = not gemm_big.  ``N`` is
    the weight's row count (2I for the SwiGLU form)."""
    if _big_mode == "0" or M <= DISPATCH_MAX_M:
        return 0
    if not big_shape_ok(M, N // 2 if silu else N, K, silu):
        return 0
    if _big_mode == "all":
        return 1
    for lo, hi, splits in _big_ranges.get(("silu", N, K) if silu else (N, K), ()):
        if lo <= M <= hi and big_shape_ok(M, N // 2 if silu else N, K, silu, splits):
            return splits
    return 0


# SwiGLU epilogue on the decode stream kernel: where the dispatch table picks
# gemm_stream with one K split for gate_up, the SwiGLU form of the same strip
# kernel (64-row W strips = 32 gate + 32 up rows) replaces gate_up + silu_mul --
# the same weight bytes, no [M, 2I] write and re-read, one launch fewer.
_stream_silu = KNOBS.stream_silu


def swiglu_choice(M: int, N2: int, K: int):
    """(kind, cfg, splits) of the SwiGLU-epilogue gate_up GEMM for ``M`` rows of
    a [N2 = 2I, K] gate_up weight, or ``None`` (gate_up GEMM + silu_mul)."""
    if _big_pick(M, N2, K, silu=True):
        return KIND_BIG, BIG_PIPE, 1
    if _stream_silu and _dispatch and M <= DISPATCH_MAX_M and (N2 // 2) % 64 == 0:
        kind, cfg, splits = select_gemm(M, N2, K)
        if kind == KIND_STREAM and splits == 1:
            return KIND_STREAM, cfg, 1
    return None


def gemm_stream_silu(x: torch.Tensor, w: torch.Tensor, cfg: int, out: torch.Tensor = None) -> torch.Tensor:
    """``silu(x @ Wg.T) * (x @ Wu.T)`` on the decode stream kernel (w = [Wg; Wu])."""
    M, K = x.shape
    N = w.shape[0] // 2
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    check(lib().k8s_gemm_stream_silu(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, cfg,
                                     stream_ptr(x)), "gemm_stream_silu")
    return out


def swiglu_gemm(y: torch.Tensor, w_gu: torch.Tensor):
    """``silu_mul(y @ w_gu.T)`` in one launch (gemm_big's or the stream kernel's
    SwiGLU epilogue) where :func:`swiglu_choice` picks one; ``None`` otherwise
    (the caller runs the gate_up GEMM + silu_mul)."""
    M, K = y.shape
    if not (y.is_cuda and y.dtype == torch.bfloat16 and y.stride(1) == 1 and y.stride(0) % 8 == 0
            and w_gu.is_contiguous()):
        return None
    ch = swiglu_choice(M, w_gu.shape[0], K)
    if ch is None:
        return None
    if ch[0] == KIND_BIG:
        return gemm_big(y, w_gu, silu=True, pipe=ch[1])
    return gemm_stream_silu(y, w_gu, ch[1])


def big_shape_ok(M: int, N: int, K: int, silu: bool = False, splits: int = 1) -> bool:
    """What csrc/kernels/gemm_big.hip accepts: 256-column tiles (128 act
    columns for the SwiGLU form), K in pairs of 64-deep tiles per K split
    (split-K only for the plain form)."""
    return (M > 0 and splits >= 1 and K % (128 * splits) == 0 and N % (128 if silu else 256) == 0
            and not (silu and splits > 1))


def gemm_big(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None, silu: bool = False,
             pipe: int = None, splits: int = 1) -> torch.Tensor:
    """``x @ w.T`` on the prefill-size MFMA kernel (csrc/kernels/gemm_big.hip:
    256 x 256 x 64 tiles, eight-phase ping-pong schedule, LDS-DMA staging;
    ``pipe`` = the VAR bits (1 = the ping-pong stagger, the default ``BIG_PIPE``;
    +2 static priority, +4 the 32x32x16-MFMA form)).  ``silu=True``: ``w`` is the gate_up weight
    [2I, K] and the result is ``silu(x @ Wg.T) * (x @ Wu.T)`` [M, I] -- the
    SwiGLU epilogue, with the unfused path's bf16 rounding of gate and up.
    ``splits`` > 1: K split over that many workgroups per tile (fp32 partials
    in the gemm_mid scratch, then a reduce launch)."""
    M, K = x.shape
    N = w.shape[0] // 2 if silu else w.shape[0]
    if not (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and w.is_contiguous() and w.shape[1] == K and big_shape_ok(M, N, K, silu, splits)):
        raise ValueError(f"gemm_big: unsupported operands x {tuple(x.shape)} w {tuple(w.shape)} silu={silu} "
                         f"splits={splits}")
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    if M == 0:
        return out
    var = BIG_PIPE if pipe is None else pipe
    if x.device not in _big_ws and _big_tail:
        reserve_big_ws(x.device)
    if splits > 1:
        part = _scratch(x.device, splits * M * N)
        check(lib().k8s_gemm_big_split(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, var, splits,
                                       ptr(part), stream_ptr(x)), "gemm_big_split")
        return out
    check(lib().k8s_gemm_big(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, int(silu), var,
                             stream_ptr(x)), "gemm_big")
    return out


def stream_shape_ok(M: int, N: int, K: int, cfg: int, splits: int) -> bool:
    """What csrc/kernels/gemm_stream.hip's launcher accepts: 64-column strips,
    64-deep chunks, a slice of whole cfg-chunk loop trips, the 8-deep ring only
    up to two 16-row fragments per wave (M <= 128)."""
    # cfg 13..16: the LDS-DMA kernel with 3..6 stages (any chunk count); 23 / 24:
    # the same on 128-column strips with 3 / 4 stages; 4 / 8: the register ring,
    # whose loop has no partial trip
    ok_cfg = (cfg == 4 or (cfg == 8 and M <= 128) or cfg == 13 or (cfg == 14 and M <= 192)
              or (cfg in (15, 16) and M <= 64) or cfg == 23 or (cfg == 24 and M <= 192))
    bn = 128 if cfg > 20 else 64
    return (ok_cfg and 0 < M <= 256 and N % bn == 0 and splits >= 1 and K % (64 * splits) == 0
            and (cfg > 10 or (K // splits // 64) % cfg == 0))


def stream_candidates(M: int, N: int, K: int):
    """(cfg, splits) of the stream kernel for (M, N, K): 128..2048 workgroups."""
    out = []
    if not (0 < M <= 256 and N % 64 == 0):
        return out
    for cfg in (4, 8, 13, 14, 15, 16, 23, 24):
        for s in (1, 2, 4, 7, 8, 14, 16):
            if not stream_shape_ok(M, N, K, cfg, s):
                continue
            if 128 <= (N // (128 if cfg > 20 else 64)) * s <= 2048:
                out.append((cfg, s))
    return out


def linear_silu(gu: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``silu_mul(gu) @ w.T`` (the SwiGLU down projection): one SwiGLU-fused
    gemm_mid launch where the dispatch table measured it fastest, else the
    activation kernel followed by :func:`linear`."""
    M = gu.shape[0]
    N, K = w.shape
    if _dispatch and gu.is_cuda and M <= DISPATCH_MAX_M:
        ent = _lookup(N, K, M, silu=True)
        if ent is not None and ent[0] == "mid" and _mid_ok(gu, w, ent[1], ent[2]):
            return gemm_mid(gu, w, ent[1], ent[2])
    from .norm import silu_mul
    return linear(silu_mul(gu), w)

# ------------------------------------------------------------ mid-M GEMM
_mid_cfgs = None
_mid_scratch = {}


def mid_configs():
    """[(mt, nt, nw, u, silu)] of the compiled gemm_mid variants (index = cfg id)."""
    global _mid_cfgs
    if _mid_cfgs is None:
        import ctypes
        L = lib()
        out = []
        buf = (ctypes.c_int * 5)()
        for i in range(L.k8s_gemm_mid_num_cfgs()):
            check(L.k8s_gemm_mid_cfg(i, buf), "gemm_mid_cfg")
            out.append(tuple(buf))
        _mid_cfgs = out
    return _mid_cfgs


# Split-K partial buffers that were replaced by a larger one.  They are never
# freed: a HIP graph captured before the growth still writes (and reads back)
# its partials at the old address on every replay.  Freed, that memory would go
# back to the caching allocator and be handed to some later tensor -- the
# grammar mask table, an activation, a sampling input -- which each replay would
# then overwrite with fp32 partials: silent corruption of every request that
# tensor serves, for the rest of the run.  Growth after the engine's up-front
# reservation is rare (reserve_dispatch_scratch sizes it for the whole table);
# keeping the old buffer costs its bytes once.
_retired_scratch: List[torch.Tensor] = []
scratch_growths = 0


def _scratch(dev: torch.device, n: int) -> torch.Tensor:
    global scratch_growths
    t = _mid_scratch.get(dev)
    if t is None or t.numel() < n:
        if t is not None:
            _retired_scratch.append(t)
            scratch_growths += 1
        t = scratch(max(n, 1 << 20), torch.float32, dev)
        _mid_scratch[dev] = t
    return t


def reserve_mid_scratch(dev: torch.device, max_m: int, max_n: int, max_splits: int = 8) -> None:
    """Allocate the split-K partial buffer up front (before HIP-graph capture)."""
    _scratch(dev, max_m * max_n * max_splits)


def reserve_dispatch_scratch(dev: torch.device) -> None:
    """Size both split-K partial buffers (gemm_mid's and the grouped kernel's)
    for the largest split entry of the loaded dispatch table."""
    from . import moe as MO
    need_mid = need_grp = 0
    for key, rows in _dispatch.items():
        n = key[-2]
        for m, kind, _, splits in rows:
            if kind in ("mid", "stream") and splits > 1:  # both use the gemm_mid partial buffer
                need_mid = max(need_mid, m * n * splits)
            elif kind == "grp" and splits > 1:
                need_grp = max(need_grp, m * n * splits)
    need_mid = max(need_mid, big_scratch_elems())
    if need_mid:
        _scratch(dev, need_mid)
    if need_grp:
        MO.reserve_split_scratch(dev, need_grp, 1, 1)
    if dev.type == "cuda":
        grp_offsets(dev, 0)  # the offsets table, before any timed step or capture


def gemm_mid(x: torch.Tensor, w: torch.Tensor, cfg: int, splits: int, out: torch.Tensor = None) -> torch.Tensor:
    """``x @ w.T`` on the mid-M kernel (csrc/kernels/gemm_mid.hip), variant
    ``cfg``, K split over ``splits`` workgroups (fp32 partials + reduce).  For
    a SwiGLU variant ``x`` is the gate_up activation [M, 2K] and the product
    is ``silu_mul(x) @ w.T``."""
    M = x.shape[0]
    N, K = w.shape
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    part = _scratch(x.device, splits * M * N) if splits > 1 else None
    check(lib().k8s_gemm_mid(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K, cfg, splits,
                             ptr(part), stream_ptr(x)), "gemm_mid")
    return out


def mid_candidates(M: int, N: int, K: int, silu: bool = False):
    """Every (cfg, splits) that applies to (M, N, K): grid of 128..1024 workgroups."""
    out = []
    for i, (mt, nt, nw, u, fused) in enumerate(mid_configs()):
        bn = 16 * nt * nw
        if bool(fused) != silu or M > 16 * mt or M <= 16 * mt // 2 and mt > 2 or N % bn:
            continue
        for s in (1, 2, 4, 7, 8):
            if K % (64 * s) or K // s < 64 * u:
                continue
            if 128 <= (N // bn) * s <= 1024:
                out.append((i, s))
    return out


def candidate_kernels(M: int, N: int, K: int):
    """Hand-written kernels applicable to an (M, N, K) bf16 projection, as
    ``(name, fn(x, w) -> y)`` pairs (used by tools/gemm_mid_sweep.py)."""
    out = []
    if M <= 128 and N % 16 == 0 and K % 256 == 0:
        def skinny(x, w):
            y = torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
            check(lib().k8s_gemm_skinny(ptr(x), x.stride(0), ptr(w), ptr(y), y.stride(0), x.shape[0], w.shape[0],
                                        x.shape[1], stream_ptr(x)), "gemm_skinny")
            return y
        out.append(("skinny", skinny))
    if 16 < M <= 256 and x_ok(K):
        for cfg, s in mid_candidates(M, N, K):
            out.append((f"mid{cfg}:{mid_configs()[cfg][:4]}x{s}", lambda x, w, cfg=cfg, s=s: gemm_mid(x, w, cfg, s)))
    if M <= 256 and N % 128 == 0:
        for s in (1, 2, 4, 8):
            if K % (64 * s) == 0 and (N // 128) * ((M + 63) // 64) * s <= 2048:
                out.append((f"grp:x{s}", lambda x, w, s=s: gemm_grp(x, w, s)))
    for cfg, s in stream_candidates(M, N, K):
        out.append((f"stream{cfg}:x{s}", lambda x, w, cfg=cfg, s=s: gemm_stream(x, w, cfg, s)))
    return out


def silu_candidates(M: int, N: int, K: int):
    """SwiGLU-fused gemm_mid variants for ``silu_mul(gu) @ w.T`` (w [N, K], gu [M, 2K])."""
    out = []
    if 16 < M <= 256 and x_ok(K):
        for cfg, s in mid_candidates(M, N, K, silu=True):
            out.append((f"mid{cfg}:{mid_configs()[cfg][:4]}x{s}", lambda g, w, cfg=cfg, s=s: gemm_mid(g, w, cfg, s)))
    return out


def x_ok(K: int) -> bool:
    return K % 64 == 0
