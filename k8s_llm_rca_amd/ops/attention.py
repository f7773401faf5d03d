"""RoPE + paged-KV write (B3+B5) and paged GQA attention (B6/B7).

KV cache layout per layer (page = ``block_size`` tokens):
``k_cache[num_blocks, n_kv, block_size, 128]`` and
``v_cache[num_blocks, n_kv, 128, block_size]`` (V pages transposed so the PV
MFMA operand is a contiguous load; see ``csrc/kernels/attention.hip``).
"""
from __future__ import annotations

from ..knobs import KNOBS
import math
import os
from dataclasses import dataclass
from typing import List, Optional

import torch

from ._lib import check, lib, ptr, scratch, stream_ptr, use_hip

HEAD_DIM = 128


def rope_cos_sin(max_pos: int, theta: float = 500000.0, head_dim: int = HEAD_DIM, scaling: Optional[dict] = None,
                 device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: cos(f_i p) for i < d/2, then sin(f_i p)."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) / half))
    # ModelConfig keeps only the numeric scaling fields (config_from_hf): a
    # `factor` without another rope_type is Llama-3.1's "llama3" scaling
    if scaling and "factor" in scaling and scaling.get("type", scaling.get("rope_type", "llama3")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * math.pi / inv
        lo_w, hi_w = old / lo, old / hi
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_w, inv / factor, inv)
        mid = (wavelen <= lo_w) & (wavelen >= hi_w)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    p = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([p.cos(), p.sin()], dim=1).to(torch.float32).to(device)


def kv_write(k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor,
             v_cache: torch.Tensor) -> None:
    """Scatter un-rotated k,v [T, nkv, D] into pages (learned-position models, e.g. OPT)."""
    BS = k_cache.shape[2]
    s = slots.long()
    ok = s >= 0
    blk, off = (s // BS)[ok], (s % BS)[ok]
    k_cache[blk, :, off, :] = k[ok].to(k_cache.dtype)
    v_cache[blk, :, :, off] = v[ok].to(v_cache.dtype)


def rope_kv_write(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor, slots: Optional[torch.Tensor],
                  k_cache: torch.Tensor, v_cache: torch.Tensor, nq: int, nkv: int) -> None:
    """Rotate q,k in place inside ``qkv`` and scatter k,v into their pages."""
    T, ld = qkv.shape
    BS = k_cache.shape[2]
    assert ld >= (nq + 2 * nkv) * HEAD_DIM
    if use_hip(qkv):
        assert qkv.stride(1) == 1 and positions.dtype == torch.int32 and cos_sin.dtype == torch.float32
        assert slots is None or slots.dtype == torch.int32
        assert k_cache.shape[1] == nkv and v_cache.shape[2] == HEAD_DIM and v_cache.shape[3] == BS
        check(lib().k8s_rope_kv(ptr(qkv), qkv.stride(0), ptr(positions), ptr(cos_sin), ptr(slots), ptr(k_cache),
                                ptr(v_cache), T, nq, nkv, BS, stream_ptr(qkv)), "rope_kv")
        return
    half = HEAD_DIM // 2
    cs = cos_sin[positions.long()]
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    nh = nq + nkv
    x = qkv[:, : nh * HEAD_DIM].float().view(T, nh, HEAD_DIM)
    a, b = x[..., :half], x[..., half:]
    rot = torch.cat([a * cos - b * sin, b * cos + a * sin], dim=-1)
    qkv[:, : nh * HEAD_DIM] = rot.reshape(T, -1).to(qkv.dtype)
    if slots is None:
        return
    k = qkv[:, nq * HEAD_DIM: nh * HEAD_DIM].view(T, nkv, HEAD_DIM)
    v = qkv[:, nh * HEAD_DIM: (nh + nkv) * HEAD_DIM].view(T, nkv, HEAD_DIM)
    s = slots.long()
    ok = s >= 0
    blk, off = (s // BS)[ok], (s % BS)[ok]
    k_cache[blk, :, off, :] = k[ok]
    v_cache[blk, :, :, off] = v[ok]


_fuse_qkv = KNOBS.fuse_splitk


# RoPE / KV-write epilogue on the skinny qkv GEMM (decode at M <= 16 where the
# dispatch picks the skinny kernel): one launch instead of GEMM + rope_kv.
_skinny_rope = KNOBS.skinny_rope


def skinny_rope_ok(M: int, N: int, K: int, nq: int, nkv: int) -> bool:
    return _skinny_rope and 0 < M <= 16 and K % 256 == 0 and N == (nq + 2 * nkv) * HEAD_DIM


def linear_rope_kv(y: torch.Tensor, w: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                   slots: Optional[torch.Tensor], k_cache: torch.Tensor, v_cache: torch.Tensor, nq: int,
                   nkv: int) -> torch.Tensor:
    """``qkv = y @ w.T`` followed by :func:`rope_kv_write`.  When the measured
    dispatch picks a split-K kernel for this M, its fp32 partials go straight
    to ``k8s_splitk_rope_kv``, which reduces them in the reduce kernel's order
    before rotating: bit-identical to ``linear`` + ``rope_kv_write`` with one
    launch fewer (csrc/kernels/norm_act.hip, PART form of rope_kv_kernel)."""
    from . import linear as LIN
    M, K = y.shape
    N = w.shape[0]
    if _fuse_qkv and use_hip(y) and y.dtype == torch.bfloat16 and slots is not None:
        layout = y.stride(1) == 1 and y.stride(0) % 8 == 0 and w.is_contiguous()
        kind, cfg, splits = LIN.select_gemm(M, N, K, layout, True)
        if kind == LIN.KIND_SKINNY and layout and skinny_rope_ok(M, N, K, nq, nkv):
            qkv = torch.empty((M, N), dtype=y.dtype, device=y.device)
            BS = k_cache.shape[2]
            check(lib().k8s_gemm_skinny_rope(ptr(y), y.stride(0), ptr(w), ptr(qkv), N, M, N, K, ptr(positions),
                                             ptr(cos_sin), ptr(slots), ptr(k_cache), ptr(v_cache), nq, nkv, BS,
                                             stream_ptr(y)), "gemm_skinny_rope")
            return qkv
        if layout and N == (nq + 2 * nkv) * HEAD_DIM and LIN.rope_choice(M, N, K):
            # the prefill-size qkv GEMM with RoPE + the paged KV write in its epilogue
            return LIN.gemm_big_rope(y, w, positions, cos_sin, slots, k_cache, v_cache, nq, nkv)
        if kind in (LIN.KIND_STREAM, LIN.KIND_MID, LIN.KIND_BIG) and splits > 1:
            qkv = torch.empty((M, N), dtype=y.dtype, device=y.device)
            part = LIN._scratch(y.device, splits * M * N)
            fn = {LIN.KIND_STREAM: lib().k8s_gemm_stream_part, LIN.KIND_MID: lib().k8s_gemm_mid_part,
                  LIN.KIND_BIG: lib().k8s_gemm_big_part}[kind]
            check(fn(ptr(y), y.stride(0), ptr(w), ptr(qkv), N, M, N, K, cfg, splits, ptr(part), stream_ptr(y)),
                  "qkv gemm (split-K partials)")
            BS = k_cache.shape[2]
            assert positions.dtype == torch.int32 and cos_sin.dtype == torch.float32 and slots.dtype == torch.int32
            assert k_cache.shape[1] == nkv and v_cache.shape[2] == HEAD_DIM and v_cache.shape[3] == BS
            assert N >= (nq + 2 * nkv) * HEAD_DIM
            check(lib().k8s_splitk_rope_kv(ptr(part), splits, ptr(qkv), N, ptr(positions), ptr(cos_sin), ptr(slots),
                                           ptr(k_cache), ptr(v_cache), M, nq, nkv, BS, stream_ptr(y)),
                  "splitk_rope_kv")
            return qkv
    qkv = LIN.linear(y, w)
    rope_kv_write(qkv, positions, cos_sin, slots, k_cache, v_cache, nq, nkv)
    return qkv


@dataclass
class AttnMeta:
    """Per-step attention metadata (device tensors, int32)."""
    block_tables: torch.Tensor   # [S, max_blocks]
    ctx_lens: torch.Tensor       # [S]
    q_start: torch.Tensor        # [S+1]
    num_seqs: int
    decode: bool                 # every sequence has exactly one query token
    # prefill tiling
    tile_seq: Optional[torch.Tensor] = None
    tile_tok0: Optional[torch.Tensor] = None
    tile_len: Optional[torch.Tensor] = None
    n_tiles: int = 0
    # prefill split-KV (paged-64 kernel): see :func:`plan_prefill`
    tile_kv0: Optional[torch.Tensor] = None
    tile_kv1: Optional[torch.Tensor] = None
    tile_slot: Optional[torch.Tensor] = None
    m_tok0: Optional[torch.Tensor] = None
    m_len: Optional[torch.Tensor] = None
    m_slot0: Optional[torch.Tensor] = None
    m_np: Optional[torch.Tensor] = None
    n_merge: int = 0
    pf_o: Optional[torch.Tensor] = None
    pf_ml: Optional[torch.Tensor] = None
    # decode split-KV
    n_parts: int = 1
    part_size: int = 512
    part_o: Optional[torch.Tensor] = None
    part_ml: Optional[torch.Tensor] = None
    # decode work list (persistent kernel, BS % 64 == 0): see build_decode_items
    items: Optional[torch.Tensor] = None      # [n_items, 4] int32
    n_items: int = 0
    d_n_items: Optional[torch.Tensor] = None  # [2] int32 device {item count, part_size} (HIP graphs)
    grid_waves: int = 0
    # host copies for the reference path
    ctx_lens_host: Optional[list] = None
    q_start_host: Optional[list] = None

    def m_slot0_end(self) -> int:
        """Slots used by the merge list (workspace size when allocated lazily)."""
        if not self.n_merge:
            return 0
        s0, npp = self.m_slot0.tolist(), self.m_np.tolist()
        return max(a + b for a, b in zip(s0, npp))


DECODE_PARTS = tuple(range(256, 1537, 64))  # candidate keys per decode work item (64-key aligned)
DECODE_PARTS_V1 = (512, 768, 1024)
# consecutive tokens of one sequence in a decode step share multi-token work items
DECODE_GROUP_TOKENS = KNOBS.decode_group
DECODE_WAVE_SLOTS = 2048                 # resident decode waves: 256 CUs x 4 SIMDs x 2 (<= 256 VGPRs)
DECODE_ITEM_OVERHEAD = 256               # per-item start cost in key-equivalents (replay-calibrated)
_DECODE_PLANNER = "makespan"
# Low batch (the whole step is one round of waves at 256 keys per item): the
# fewest keys per item that keep the launch at <= this many (item, kv head)
# waves, from 64 keys up.  Measured over cold K/V, 1-8 rows x 2k-8k keys
# (tools/decode_part_sweep.py, profiles/r5/decode_parts/): the best part size
# puts ~256-512 waves on the 256 CUs -- fewer, longer items at 4-8 rows (512
# keys: 30.7 vs 34.4 us at 4 x 8k), shorter ones at one row (192: 13.7 vs
# 15.4 us at 5k) -- where the makespan model's fixed item cost took 256 keys
# everywhere.  0 = off.
DECODE_LOW_UNITS = KNOBS.decode_low_units
DECODE_LOW_PARTS = tuple(range(64, 1537, 64))
DECODE_LOW_ROWS = 8  # the measured range of the rule (1-8 rows); larger steps keep the makespan planner


def plan_decode_split(ctx_lens, nkv: int, slots: int = DECODE_WAVE_SLOTS, candidates=None,
                      max_parts: Optional[int] = None) -> tuple:
    """Keys per decode work item for one step -> (max items per sequence, part_size).

    The persistent decode kernel runs ``slots`` waves over a longest-first
    work list (unit u = item * nkv + kv head goes to wave u mod slots), so the
    step takes as long as wave 0's share: the first unit of every round.
    Sorted longest-first, the items are the full ``P``-key items followed by
    each sequence's remainder, so that makespan is exact and cheap to compute
    for every candidate ``P`` (one sort of S remainders each):
    ``sum over rounds r of (size of unit r*slots + start overhead)``.
    A coarse candidate set with a "total/slots + P" bound (round-1 planner,
    ``DECODE_PARTS_V1``) left up to a whole item of LPT tail: e.g. 96
    sequences x 3.4k keys ran 3 rounds of 512 keys (1536) where 448-key items
    give 3 rounds of 448 (ideal 1275)."""
    import numpy as np
    c = np.asarray(ctx_lens, dtype=np.int64)
    mx = int(c.max()) if c.size else 1
    if DECODE_LOW_UNITS and candidates is None and 0 < c.size <= DECODE_LOW_ROWS:
        P0 = min(DECODE_PARTS)
        if nkv * int(((c + P0 - 1) // P0).sum()) <= slots:  # one round: the low-batch rule
            for P in DECODE_LOW_PARTS:
                n = -(-mx // P)
                if (max_parts is None or n <= max_parts) and nkv * int(((c + P - 1) // P).sum()) <= DECODE_LOW_UNITS:
                    return max(1, n), P
    if _DECODE_PLANNER == "v1":
        return _plan_decode_split_v1(c, nkv, slots, candidates or DECODE_PARTS_V1)
    Ps = np.asarray(candidates or DECODE_PARTS, dtype=np.int64)[:, None]      # [nc, 1]
    n = (c[None, :] + Ps - 1) // Ps                                            # [nc, S]
    rem = c[None, :] - (n - 1) * Ps                                            # 1..P keys
    n_full = (n - 1).sum(1) + (rem == Ps).sum(1)                               # [nc]
    rems = np.sort(np.where(rem < Ps, rem, 0), axis=1)[:, ::-1]                 # partial items, longest first
    n_items = n.sum(1)
    rounds = -(-(n_items * nkv) // slots)
    R = int(rounds.max())
    first = np.arange(R, dtype=np.int64)[None, :] * slots // nkv               # [1, R] item index per round
    live = np.arange(R)[None, :] < rounds[:, None]
    ridx = np.clip(first - n_full[:, None], 0, c.size - 1)
    sizes = np.where(first < n_full[:, None], Ps, np.take_along_axis(rems, ridx, axis=1))
    cost = (np.where(live, sizes + DECODE_ITEM_OVERHEAD, 0)).sum(1)
    P = int(Ps[int(np.argmin(cost)), 0])
    return max(1, -(-mx // P)), P


def _plan_decode_split_v1(c, nkv, slots, candidates):
    mx = int(c.max()) if c.size else 1
    total = nkv * int(c.sum())
    best = None
    for P in candidates:
        items = nkv * int(((c + P - 1) // P).sum())
        cost = (total + items * DECODE_ITEM_OVERHEAD) / slots + min(P, mx)
        if best is None or cost < best[0] - 1e-9:
            best = (cost, P)
    P = best[1]
    return max(1, -(-mx // P)), P


def set_decode_planner(name: str) -> None:
    """``"makespan"`` (default) or ``"v1"`` (A/B in tools/bench_kernels.py --what replay)."""
    global _DECODE_PLANNER
    assert name in ("makespan", "v1")
    _DECODE_PLANNER = name


def attach_decode_plan(meta: "AttnMeta", ctx_host, nq: int, nkv: int, block_size: int, device,
                       q_rows=None, part: Optional[int] = None, chain=None) -> "AttnMeta":
    """Plan + upload the decode split for ``meta`` (tests / tools; the engine
    ships the same arrays in its step buffer).  Paged-64 caches use the
    persistent work-list kernel; other page sizes the (seq, part) grid."""
    import numpy as np
    ctx_host = [int(c) for c in ctx_host]
    S = len(ctx_host)
    if block_size % 64 == 0:
        n_parts, P = plan_decode_split(ctx_host, nkv)
        if part is not None:
            P = part
            n_parts = max(1, -(-max(ctx_host) // P))
        G = nq // nkv
        items = build_decode_items(ctx_host, q_rows if q_rows is not None else np.arange(S), P, chain,
                                   max(1, 16 // G) if G <= 16 else 1)
        meta.items = torch.from_numpy(items).to(device)
        meta.n_items = items.shape[0]
    else:
        P = part or 512
        n = max(1, -(-max(ctx_host) // P))
        n_parts = 1 << (n - 1).bit_length()
    meta.n_parts, meta.part_size = n_parts, P
    if n_parts > 1:
        meta.part_o = scratch(S * nq * n_parts * HEAD_DIM, torch.float32, device)
        meta.part_ml = scratch(S * nq * n_parts * 2, torch.float32, device)
    return meta


def decode_groups(ctx_lens, q_rows, chain, gmax: int, part: Optional[int] = None):
    """Multi-token decode items: ``chain[i]`` = row i is the next token of row
    i-1's sequence (a short prefill chunk run as decode rows).  Runs of chained
    rows are cut into groups of at most ``gmax`` (= 16 // G: the decode MFMA's
    16 rows hold G q heads per token) consecutive q rows; with ``part`` a group
    also never mixes rows of different partition counts (each row's split-KV
    reduce reads its own count).  Returns (first row, tokens) per group."""
    import numpy as np
    c = np.asarray(ctx_lens, dtype=np.int64)
    S = c.size
    idx = np.arange(S)
    ok = np.zeros(S, dtype=bool)
    if chain is not None and gmax > 1 and S > 1:
        qr = np.asarray(q_rows, dtype=np.int64)
        ok[1:] = np.asarray(chain[1:], dtype=bool) & (qr[1:] == qr[:-1] + 1)
        if part is not None:
            n = (c + part - 1) // part
            ok[1:] &= n[1:] == n[:-1]
    brk = ~ok
    start = np.maximum.accumulate(np.where(brk, idx, 0))
    lead = np.nonzero(brk | ((idx - start) % max(gmax, 1) == 0))[0]
    nt = np.diff(np.append(lead, S))
    return lead, nt


def build_decode_items(ctx_lens, q_rows, part: int, chain=None, gmax: int = 1):
    """Work list [n_items, 4] int32 = (seq, part | -1 for a one-item row, end
    key, q row | (tokens - 1) << 24), longest first.  With ``chain`` rows of
    one sequence's consecutive tokens share items (``decode_groups``): the
    item's seq / q row are its first token's, its key range its last token's."""
    import numpy as np
    c = np.asarray(ctx_lens, dtype=np.int64)
    qr = np.asarray(q_rows, dtype=np.int64)
    if chain is not None and gmax > 1:
        lead, nt = decode_groups(c, qr, chain, gmax, part)
    else:
        lead, nt = np.arange(c.size), np.ones(c.size, dtype=np.int64)
    cl = c[lead + nt - 1]
    n = (cl + part - 1) // part
    g = np.repeat(np.arange(lead.size), n)
    first = np.repeat(np.cumsum(n) - n, n)
    pidx = np.arange(g.size) - first
    k0 = pidx * part
    k1 = np.minimum(cl[g], k0 + part)
    out = np.empty((g.size, 4), dtype=np.int32)
    out[:, 0] = lead[g]
    out[:, 1] = np.where(n[g] == 1, -1, pidx)
    out[:, 2] = k1
    out[:, 3] = qr[lead[g]] | ((nt[g] - 1) << 24)
    order = np.argsort(-(k1 - k0), kind="stable")
    return out[order]


def pf_wg_rows(G: int) -> int:
    """(token, q-head) rows per paged-64 prefill workgroup: 256 for the 8-wave
    LDS-DMA kernel (knob ``pf_w8``, default on; the C launcher reads the
    same switch per launch), 128 for the 4-wave pg64 kernel."""
    if KNOBS.pf_w8 != 0 and PF8_ROWS % G == 0:
        return PF8_ROWS
    return PF_ROWS


def prefill_tile_tokens(G: int, block_size: int) -> int:
    """Tokens per prefill tile: the paged-64 kernels cover 256 (8 waves) or
    128 (4 waves) (token, q-head) rows per workgroup, the generic one 64."""
    if block_size == 64 and PF_ROWS % G == 0:
        return max(1, pf_wg_rows(G) // G)
    return max(1, 64 // G)


PF_ROWS = 128               # (token, q-head) rows per pg64 prefill workgroup
PF8_ROWS = 256              # rows per 8-wave (w8) prefill workgroup
PF8_MAXP = 1024             # key pages per w8 work item (page ids staged in LDS; attention.hip)
PF_MAX_SLOTS = 512          # partial-result slots of the prefill split-KV workspace
# split long key ranges until a prefill launch has about this many workgroups
PF_TARGET_WGS = KNOBS.pf_target_wgs
# makespan planner (PF_OVERHEAD_PAGES > 0): where the fixed-target rule would split
# (too few tiles to fill the chip), pick instead the split length that minimises
# the launch's estimated makespan on the CU slots, pricing every work item at its
# pages + this many pages of fixed cost (Q load, first DMAs, epilogue, merge share).
# Replayed steady-state mix (profiles/r4/planner/): fixed target 635.5 -> 725.5
# TFLOP/s at 8 pages (200-700-token extends -24 %, longer ones -7 %); applying it
# to launches with enough tiles too (PF_MAKESPAN_ALL) 675-715; 0 = the fixed target.
PF_OVERHEAD_PAGES = KNOBS.pf_overhead_pages
PF_CU_SLOTS = 256           # concurrent prefill workgroups: one 8-wave w8 workgroup per CU
PF_MAKESPAN_ALL = KNOBS.pf_makespan_all
_NO_END = 1 << 30


@dataclass
class PrefillPlan:
    """Work list of one prefill/extend attention launch.

    Item i covers query tokens ``tok0[i] .. tok0[i]+length[i]`` of sequence
    ``seq[i]`` against key pages ``kv0[i] .. kv1[i]``; ``slot[i] == -1`` means
    the item owns the whole key range and writes final rows, otherwise it
    writes an fp32 partial into ``slot`` and the merge list combines the
    ``np`` consecutive slots of each split tile (flash-decoding for extend).

    Dispatch order = list order, and the kernel maps kv head -> XCD, so items
    are grouped by sequence and key range: every query tile of a sequence
    streams the same pages at about the same time and the pages are read
    from HBM once per XCD instead of once per tile (the L2 is 4 MB per XCD; a
    3k-token context is 1.5 MB per kv head)."""
    seq: List[int]
    tok0: List[int]
    length: List[int]
    kv0: List[int]
    kv1: List[int]
    slot: List[int]
    m_tok0: List[int]
    m_len: List[int]
    m_slot0: List[int]
    m_np: List[int]

    @property
    def n_tiles(self) -> int:
        return len(self.seq)

    @property
    def n_merge(self) -> int:
        return len(self.m_tok0)

    def arrays(self) -> List[list]:
        return [self.seq, self.tok0, self.length, self.kv0, self.kv1, self.slot,
                self.m_tok0, self.m_len, self.m_slot0, self.m_np]


def plan_prefill(q_start_host: list, G: int, block_size: int = 64, ctx_lens_host: Optional[list] = None,
                 nkv: int = 8, max_slots: int = PF_MAX_SLOTS, target_wgs: Optional[int] = None) -> PrefillPlan:
    """Tile every prefill chunk (``prefill_tile_tokens`` tokens per tile) and,
    for the paged-64 kernel, split long key ranges so the launch has about
    ``target_wgs`` workgroups: extend steps in an RCA batch are small (a few
    hundred new tokens over ~3k cached ones), so without splitting a handful
    of workgroups walk 50+ pages each while most CUs idle.  Items are ordered
    most-pages first so the longest ones start first."""
    target_wgs = target_wgs or PF_TARGET_WGS
    per = prefill_tile_tokens(G, block_size)
    # the 8-wave kernel stages a tile's page ids in LDS: at most PF8_MAXP pages
    # per item (ctx > 64k tokens: the key range is split, never truncated)
    max_part = PF8_MAXP if block_size == 64 and pf_wg_rows(G) == PF8_ROWS else None
    tiles = []
    for s in range(len(q_start_host) - 1):
        a, b = q_start_host[s], q_start_host[s + 1]
        base = (ctx_lens_host[s] - (b - a)) if ctx_lens_host is not None else 0
        for t in range(a, b, per):
            n = min(per, b - t)
            tiles.append((base + (t - a) + n, s, t, n))
    plan = PrefillPlan(*[[] for _ in range(10)])
    too_long = max_part is not None and any((end + 63) // 64 > max_part for end, _, _, _ in tiles)
    split = block_size == 64 and PF_ROWS % G == 0 and (ctx_lens_host is not None or too_long)
    # sequences with the most work first; inside a sequence, longest tile first
    work = {}
    for end, s, _, n in tiles:
        work[s] = work.get(s, 0) + end * n
    rank = {s: i for i, s in enumerate(sorted(work, key=lambda s: -work[s]))}
    if not split:
        if ctx_lens_host is not None:
            tiles.sort(key=lambda x: (rank[x[1]], -x[0]))
        for _, s, t, n in tiles:
            for lst, v in zip(plan.arrays()[:6], (s, t, n, 0, _NO_END, -1)):
                lst.append(v)
        return plan
    pages = [(end + 63) // 64 for end, _, _, _ in tiles]
    total = sum(pages)
    enough = len(tiles) * nkv >= target_wgs // 2
    if PF_OVERHEAD_PAGES > 0 and pages and (PF_MAKESPAN_ALL or not enough):
        part = _makespan_part(pages, nkv, PF_OVERHEAD_PAGES, max_part, max_slots,
                              PF_CU_SLOTS if max_part is not None else 2 * PF_CU_SLOTS)
    else:
        # enough tiles to fill the chip (two 4-wave workgroups per CU): no split
        part = max(pages) if pages and enough else max(4, -(-total * nkv // target_wgs))
    part = _fit_slots(pages, part, max_part, max_slots)
    items = []
    slot = 0
    for (end, s, t, n), p in zip(tiles, pages):
        k = -(-p // part)
        if k == 1:
            items.append((p, s, t, n, 0, p, -1))
            continue
        bounds = [(i * p) // k for i in range(k + 1)]
        for i in range(k):
            items.append((bounds[i + 1] - bounds[i], s, t, n, bounds[i], bounds[i + 1], slot + i))
        plan.m_tok0.append(t)
        plan.m_len.append(n)
        plan.m_slot0.append(slot)
        plan.m_np.append(k)
        slot += k
    items.sort(key=lambda x: (rank[x[1]], x[4], -x[0]))
    for _, s, t, n, k0, k1, sl in items:
        for lst, v in zip(plan.arrays()[:6], (s, t, n, k0, k1, sl)):
            lst.append(v)
    return plan


_PART_CANDIDATES = (4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40, 48, 56, 64, 80, 96, 128, 160, 192, 256, 384,
                    512, 768, 1024)


def _fit_slots(pages: List[int], part: int, max_part: Optional[int], max_slots: int) -> int:
    """Grow ``part`` (pages per split item) until the split tiles need at most
    ``max_slots`` partial-result slots.  ``part`` need not be a power of two
    (makespan candidates such as 384 / 768), so the doubling is clamped at
    ``max_part``; only ``max_part`` itself overflowing is an error."""
    if max_part is not None:
        part = min(part, max_part)
    while sum(-(-p // part) for p in pages if p > part) > max_slots:
        if max_part is not None and part >= max_part:
            raise ValueError(f"prefill plan needs more than {max_slots} split-KV slots at "
                             f"{max_part} pages per item (context too long for the workspace)")
        part = part * 2 if max_part is None else min(part * 2, max_part)
    return part


def _makespan_part(pages: List[int], nkv: int, overhead: float, max_part: Optional[int], max_slots: int,
                   slots: int) -> int:
    """Split length (pages per item) minimising the estimated makespan of a
    prefill launch: items (every tile cut into ceil(p / part) near-equal
    pieces, times nkv heads) sorted longest first run in rounds of ``slots``
    workgroups, each round as long as its longest item plus ``overhead``
    pages.  The no-split choice (part = the longest tile) is a candidate."""
    import numpy as np
    pg = np.asarray(pages, dtype=np.int64)
    longest = int(pg.max())
    best, best_t = longest, None
    for part in [c for c in _PART_CANDIDATES if c < longest] + [longest]:
        if max_part is not None and part > max_part:
            continue
        k = -(-pg // part)
        if int(k[k > 1].sum()) > max_slots:
            continue
        # piece lengths of tile i: floor / ceil of p_i / k_i (the planner's bounds split)
        lo = pg // k
        n_hi = pg - lo * k
        lens = np.sort(np.concatenate([np.repeat(lo + 1, n_hi), np.repeat(lo, k - n_hi)]))[::-1]
        # every piece runs once per kv head: round r of the nkv-fold list starts at
        # its element r * slots, i.e. element (r * slots) // nkv of the piece list
        rounds = -(-lens.size * nkv // slots)
        t = float(lens[(np.arange(rounds) * slots) // nkv].sum()) + overhead * rounds
        if best_t is None or t < best_t:
            best, best_t = part, t
    return best


def attach_plan(meta: "AttnMeta", plan: PrefillPlan, device, workspace: Optional[tuple] = None) -> "AttnMeta":
    """Upload ``plan`` into ``meta`` (tests / tools; the engine ships the same
    arrays inside its one-copy step buffer)."""
    t = [torch.tensor(x if x else [0], dtype=torch.int32, device=device) for x in plan.arrays()]
    (meta.tile_seq, meta.tile_tok0, meta.tile_len, meta.tile_kv0, meta.tile_kv1, meta.tile_slot,
     meta.m_tok0, meta.m_len, meta.m_slot0, meta.m_np) = t
    meta.n_tiles, meta.n_merge = plan.n_tiles, plan.n_merge
    if workspace is not None:
        meta.pf_o, meta.pf_ml = workspace
    return meta


def prefill_workspace(nkv: int, device, slots: int = PF_MAX_SLOTS, D: int = HEAD_DIM) -> tuple:
    """fp32 partial-O / (max, sum) buffers for ``slots`` split-tile parts
    (sized for the larger, 256-row workgroup)."""
    return (scratch(slots * nkv * PF8_ROWS * D, torch.float32, device),
            scratch(slots * nkv * PF8_ROWS * 2, torch.float32, device))


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, meta: AttnMeta, nq: int,
                    nkv: int, scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q: [T, >= nq*D] (row stride free) -> out [T, nq*D]."""
    T = q.shape[0]
    BS = k_cache.shape[2]
    D = k_cache.shape[3]
    if out is None:
        out = torch.empty((T, nq * D), dtype=q.dtype, device=q.device)
    if use_hip(q) and D == HEAD_DIM:
        assert q.stride(1) == 1 and out.stride(1) == 1 and q.dtype == torch.bfloat16
        assert meta.block_tables.dtype == torch.int32 and meta.block_tables.is_contiguous()
        L = lib()
        if meta.decode:
            assert T == meta.num_seqs
            grid = meta.grid_waves or min(DECODE_WAVE_SLOTS, meta.n_items * nkv)
            check(L.k8s_attn_decode(ptr(q), q.stride(0), ptr(k_cache), ptr(v_cache), ptr(meta.block_tables),
                                    meta.block_tables.stride(0), ptr(meta.ctx_lens), ptr(meta.q_start),
                                    meta.num_seqs, nq, nkv, BS, float(scale), ptr(out), out.stride(0),
                                    ptr(meta.part_o), ptr(meta.part_ml), meta.n_parts, meta.part_size,
                                    ptr(meta.items), meta.n_items, ptr(meta.d_n_items), grid,
                                    stream_ptr(q)), "attn_decode")
        else:
            if meta.n_merge and meta.pf_o is None:
                meta.pf_o, meta.pf_ml = prefill_workspace(nkv, q.device, max(meta.m_slot0_end(), 1))
            check(L.k8s_attn_prefill(ptr(q), q.stride(0), ptr(k_cache), ptr(v_cache), ptr(meta.block_tables),
                                     meta.block_tables.stride(0), ptr(meta.ctx_lens), ptr(meta.q_start),
                                     ptr(meta.tile_seq), ptr(meta.tile_tok0), ptr(meta.tile_len),
                                     ptr(meta.tile_kv0), ptr(meta.tile_kv1), ptr(meta.tile_slot), meta.n_tiles,
                                     ptr(meta.m_tok0), ptr(meta.m_len), ptr(meta.m_slot0), ptr(meta.m_np),
                                     meta.n_merge, ptr(meta.pf_o), ptr(meta.pf_ml), nq, nkv, BS, float(scale),
                                     ptr(out), out.stride(0), stream_ptr(q)),
                  "attn_prefill")
        return out
    return _attention_ref(q, k_cache, v_cache, meta, nq, nkv, scale, out)


def _attention_ref(q, k_cache, v_cache, meta: AttnMeta, nq, nkv, scale, out):
    BS = k_cache.shape[2]
    HEAD_DIM = k_cache.shape[3]
    G = nq // nkv
    qs = meta.q_start_host if meta.q_start_host is not None else meta.q_start.tolist()
    cl = meta.ctx_lens_host if meta.ctx_lens_host is not None else meta.ctx_lens.tolist()
    bt = meta.block_tables
    for s in range(meta.num_seqs):
        a, b = qs[s], qs[s + 1]
        qlen, ctx = b - a, cl[s]
        nb = (ctx + BS - 1) // BS
        blocks = bt[s, :nb].long()
        if qlen == 1:
            # decode row (the CPU preset's common case): score page by page on the
            # gathered pages, no head-major K/V copies (1.3-2.4x faster at 0.5-4k keys)
            Kg = k_cache[blocks].float()                                  # [nb, nkv, BS, D]
            Q = q[a, : nq * HEAD_DIM].float().view(1, nkv, G, HEAD_DIM).transpose(2, 3)
            S = torch.matmul(Kg, Q).permute(1, 3, 0, 2).reshape(nkv, G, nb * BS)
            if ctx < nb * BS:
                S[:, :, ctx:] = float("-inf")
            P = torch.softmax(S * scale, dim=-1).view(nkv, G, nb, BS).permute(2, 0, 3, 1)   # [nb, nkv, BS, G]
            Vg = v_cache[blocks].float()                                  # [nb, nkv, D, BS]
            O = torch.matmul(Vg, P).sum(0)                                # [nkv, D, G]
            out[a] = O.transpose(1, 2).reshape(nq * HEAD_DIM).to(out.dtype)
            continue
        K = k_cache[blocks].permute(1, 0, 2, 3).reshape(nkv, nb * BS, HEAD_DIM)[:, :ctx].float()
        V = v_cache[blocks].permute(1, 0, 3, 2).reshape(nkv, nb * BS, HEAD_DIM)[:, :ctx].float()
        Q = q[a:b, : nq * HEAD_DIM].float().view(qlen, nkv, G, HEAD_DIM)
        S = torch.einsum("tkgd,knd->kgtn", Q, K) * scale
        pos = torch.arange(ctx - qlen, ctx)[:, None]
        mask = torch.arange(ctx)[None, :] <= pos
        S = S.masked_fill(~mask, float("-inf"))
        P = torch.softmax(S, dim=-1)
        O = torch.einsum("kgtn,knd->tkgd", P, V)
        out[a:b] = O.reshape(qlen, nq * HEAD_DIM).to(out.dtype)
    return out
