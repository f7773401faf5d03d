"""Mixtral sparse MoE block (B11-B13, B15).

``router -> top-k -> permute -> per-expert SwiGLU -> weighted combine``.
Routing (softmax + top-2 + renormalise), the token permutation (expert
histogram + prefix scan) and the weighted combine are HIP kernels
(``csrc/kernels/moe.hip``); the expert GEMMs are one grouped-GEMM launch per
projection (``csrc/kernels/grouped_gemm.hip``) driven by the device-side
expert offsets -- no host sync, so MoE decode steps are graph-capturable --
with the down projection split over K for decode-sized batches.  Under expert parallelism (EP) the whole experts live
on ``E / ep`` ranks and tokens travel by all-to-all (:mod:`..parallel.ep`).
"""
from __future__ import annotations

from ..knobs import KNOBS
import os

from typing import List, Optional

import torch

from ..ops import moe as M
from ..ops import norm as N
from ..ops.linear import lib_gemm
from ..parallel.groups import ParallelContext
from .config import ModelConfig


class MoELayerSet:
    def __init__(self, cfg: ModelConfig, device, dtype, pc: ParallelContext, g: torch.Generator, out_std: float,
                 full_slice: bool = False):
        self.cfg = cfg
        self.pc = pc
        self.E = cfg.n_experts
        self.k = cfg.top_k
        ep = pc.ep_size
        if self.E % ep:
            raise ValueError(f"{self.E} experts not divisible by ep={ep}")
        self.E_local = self.E // ep
        self.e0 = pc.ep_rank * self.E_local
        H, I = cfg.hidden, cfg.intermediate
        self.router: List[torch.Tensor] = []
        self.w13: List[torch.Tensor] = []
        self.w2: List[torch.Tensor] = []
        ne = self.E if full_slice else self.E_local
        sl = slice(self.e0, self.e0 + self.E_local) if full_slice else slice(0, self.E_local)
        for _ in range(cfg.n_layers):
            r = torch.empty(self.E, H, dtype=dtype, device=device)
            r.normal_(0.0, cfg.init_std, generator=g)
            self.router.append(r)
            w13 = torch.empty(ne, 2 * I, H, dtype=dtype, device=device)
            w13.normal_(0.0, cfg.init_std, generator=g)
            w2 = torch.empty(ne, H, I, dtype=dtype, device=device)
            w2.normal_(0.0, out_std, generator=g)
            self.w13.append(w13[sl].contiguous())
            self.w2.append(w2[sl].contiguous())
        if torch.device(device).type == "cuda":  # split-K partials exist before any HIP-graph capture
            M.reserve_split_scratch(torch.device(device), self.SPLIT_MAX_ROWS, H, self.DOWN_SPLITS)

    def weight_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for lst in (self.router, self.w13, self.w2) for t in lst)

    def forward(self, li: int, y: torch.Tensor) -> torch.Tensor:
        T, H = y.shape
        logits = lib_gemm(y, self.router[li])                          # [T, E]
        topk_w, topk_ids = M.route_topk(logits, self.k)                # [T,k] fp32, int32
        if self.pc.ep_size > 1:
            from ..parallel.ep import ep_moe_forward
            return ep_moe_forward(self, li, y, topk_w, topk_ids)
        order, inv, offsets = M.align(topk_ids, self.E)                # (token,k) slots sorted by expert
        x_perm = y.index_select(0, (order // self.k).long())           # [T*k, H]
        out_perm = self.experts(li, x_perm, offsets)
        return M.combine(out_perm, inv, topk_w, T, self.k)

    GROUPED_MAX_ROWS = 2048  # above: the grouped 8-phase GEMM (gemm_big.hip) -- SwiGLU fused, no host sync
    # split-K of the grouped down projection (tools/bench_kernels.py --what
    # moe_split, Mixtral shapes): 237 -> 161-185 us (5.8 TB/s) at <= 512 rows,
    # 264 -> 305 / 485 -> 442 us at 1024 / 2048 rows with 2 slices
    DOWN_SPLITS = 2
    SPLIT_MAX_ROWS = 2048
    # gate_up on the LDS-DMA strip kernel (ops/moe.py grouped_gemm(glds=...))
    # for decode-sized batches, (cfg, splits): 343-365 vs 383-391 us per layer
    # at 64-250 rows (5.2-5.5 TB/s); the down projection measured equal to the
    # split-K grouped kernel and stays there; at 512 rows the grouped kernel wins
    # (tools/bench_kernels.py --what moe_glds, profiles/r2_moe_glds.txt)
    GLDS_MAX_ROWS = KNOBS.moe_glds_max_rows  # 0 disables (A/B)
    BIG_PREFILL = KNOBS.moe_big  # 0: per-expert hipBLASLt (A/B)
    GLDS_UP = (13, 1)

    def experts(self, li: int, x_perm: torch.Tensor, offsets: torch.Tensor,
                device_offsets: bool = False) -> torch.Tensor:
        """Grouped SwiGLU over contiguous expert slices offsets[e]..offsets[e+1]
        (``offsets`` int32 [E_local+1], on the rows' device).  Decode-sized
        batches use the grouped weight-streaming kernel, prefill-sized ones the
        grouped form of gemm_big (below); neither syncs with the host.  The
        per-expert library loop (one offsets sync) is the fallback for shapes
        gemm_big does not take (K8SRCA_MOE_BIG=0 forces it for A/B).  ``device_offsets``: the
        grouped kernels whatever the row count (the EP dispatch buffer holds
        ``ep``-fold capacity rows, most of them the never-computed null
        expert: a host read of the offsets would stall every prefill layer).

        Prefill-sized batches run the grouped form of the 8-phase prefill GEMM
        (``ops/moe.py grouped_big``): gate_up with its SwiGLU epilogue, then
        down, two launches over every expert with the offsets read on the
        device -- no ``offsets.tolist()`` host sync per layer, no
        silu_mul launch.  The per-expert hipBLASLt loop remains only for shapes
        that kernel does not take."""
        H = x_perm.shape[1]
        I = self.w2[li].shape[2]
        if (x_perm.is_cuda and x_perm.shape[0] > self.GROUPED_MAX_ROWS and self.BIG_PREFILL
                and M.grouped_big_ok(x_perm.shape[0], I, H, True) and M.grouped_big_ok(x_perm.shape[0], H, I, False)):
            act = M.grouped_big(x_perm, self.w13[li], offsets, silu=True)
            return M.grouped_big(act, self.w2[li], offsets)
        if x_perm.is_cuda and x_perm.shape[0] > self.GROUPED_MAX_ROWS and not device_offsets:
            offs = offsets.tolist()
            out = torch.empty_like(x_perm)
            for e in range(self.E_local):
                a, b = offs[e], offs[e + 1]
                if b > a:
                    gu = lib_gemm(x_perm[a:b], self.w13[li][e])
                    lib_gemm(N.silu_mul(gu), self.w2[li][e], out=out[a:b])
            return out
        rows = x_perm.shape[0]
        if x_perm.is_cuda and rows <= self.GLDS_MAX_ROWS:
            gu = M.grouped_gemm(x_perm, self.w13[li], offsets, glds=self.GLDS_UP[0], splits=self.GLDS_UP[1])
        else:
            gu = M.grouped_gemm(x_perm, self.w13[li], offsets)
        # measured (tools/bench_kernels.py --what moe_split): silu_mul + the
        # un-fused down GEMM beats the SwiGLU-fused operand load (244 vs 287-305
        # us per layer at decode sizes), and splitting K (only 32 column tiles
        # per expert) fills the chip: 168-192 us
        splits = self.DOWN_SPLITS if rows <= self.SPLIT_MAX_ROWS and not device_offsets else 1
        return M.grouped_gemm(N.silu_mul(gu), self.w2[li], offsets, splits=splits)
