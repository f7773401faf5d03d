"""Llama-3 / Mixtral decoder (the in-process replacement for GPT-4).

Per layer (bf16, fp32 accumulation inside every kernel)::

    y      = rmsnorm(prev + residual)            # HIP fused add+norm, residual updated in place
    qkv    = y @ Wqkv^T                          # hipBLASLt (column-parallel under TP)
    rope_kv_write(qkv)                           # HIP: rotate q,k in place, scatter k,v to pages
    a      = paged_attention(qkv)                # HIP MFMA kernels (decode split-KV / varlen prefill)
    o      = a @ Wo^T ; all_reduce(o)            # row-parallel + RCCL
    y      = rmsnorm(o + residual)
    d      = silu_mul(y @ Wgu^T) @ Wdown^T ; all_reduce(d)     (dense)
           = moe(y)                                             (Mixtral: router + grouped experts)

Logits are computed only for the rows that sample (last token of each
sequence); the lm_head is vocab-parallel under TP and all-gathered.
Weights are random-init (seeded, std ``init_std``) in the real shapes;
``load_safetensors`` accepts real checkpoints when present.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from ..ops import attention as A
from ..ops import layer_exec as LX
from ..ops import norm as N
from ..ops.norm import nonfinite_flag
from ..ops.linear import linear, linear_f32out, linear_silu, swiglu_gemm
from ..parallel.groups import ParallelContext, single
from .config import ModelConfig
from . import moe as MOE


@dataclass
class StepInputs:
    input_ids: torch.Tensor        # [T] int32
    positions: torch.Tensor        # [T] int32
    slots: torch.Tensor            # [T] int32 (-1: no KV write)
    n_decode: int                  # rows [0, n_decode) are single-token decode rows
    meta_decode: Optional[A.AttnMeta]
    meta_prefill: Optional[A.AttnMeta]
    logits_idx: torch.Tensor       # [n] int64 rows whose logits are needed


class LlamaModel:
    def __init__(self, cfg: ModelConfig, device, dtype=torch.bfloat16, pc: Optional[ParallelContext] = None,
                 seed: int = 0, init: bool = True, init_mode: str = "shard"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.pc = pc or single()
        tp = self.pc.tp_size
        if cfg.n_heads % tp:
            raise ValueError(f"{cfg.n_heads} heads not divisible by tp={tp}")
        self.nq = cfg.n_heads // tp
        self.nkv = max(1, cfg.n_kv_heads // tp)   # kv heads replicated when n_kv < tp
        self.D = cfg.head_dim
        self.inter = cfg.intermediate // tp if cfg.n_experts == 0 else cfg.intermediate
        self.vocab_local = (cfg.vocab_size + tp - 1) // tp
        self.scale = 1.0 / math.sqrt(self.D)
        self._exec = None  # native layer executor (ops/layer_exec.py), bound on first GPU forward
        # debug (knob nonfinite_check): int32 [n_layers + 1] device flags, set by
        # ops.norm.nonfinite_flag when a layer's normed input holds NaN / inf
        self.nf_flags: Optional[torch.Tensor] = None
        self.cos_sin = A.rope_cos_sin(cfg.max_position, cfg.rope_theta, self.D, cfg.scaling_dict(), device=self.device)
        self.layers: List[Dict[str, torch.Tensor]] = []
        self.moe: Optional[MOE.MoELayerSet] = None
        self.init_mode = init_mode
        self.logits_f32 = True  # the sampler reads fp32 logits (EngineConfig.logits_fp32)
        if init:
            self._random_init(seed)

    # --------------------------------------------------------------- weights
    def _randn(self, g, *shape, std=None):
        std = self.cfg.init_std if std is None else std
        t = torch.empty(*shape, dtype=self.dtype, device=self.device)
        t.normal_(0.0, std, generator=g)
        return t

    def _random_init(self, seed: int) -> None:
        """Seeded random weights in the real shapes.

        ``init_mode='shard'``: each TP rank draws only its own shard (fast: a
        70B/TP8 rank never materialises the full model).  ``'full_slice'``:
        every rank draws the FULL tensors from the same seed and keeps its slice,
        so a TP=k model equals the TP=1 model exactly (used by the parity tests).
        """
        cfg = self.cfg
        tp, r = self.pc.tp_size, self.pc.tp_rank
        full = self.init_mode == "full_slice"
        g = torch.Generator(device=self.device)
        g.manual_seed(seed * 1000 + (0 if full else r))
        H, D = cfg.hidden, self.D
        out_std = cfg.init_std / math.sqrt(2 * cfg.n_layers)
        nq, nkv = self.nq, self.nkv
        kv_rep = cfg.n_kv_heads < tp  # kv heads replicated across ranks

        def qkv_shard():
            if not full:
                return self._randn(g, (nq + 2 * nkv) * D, H)
            w = self._randn(g, (cfg.n_heads + 2 * cfg.n_kv_heads) * D, H)
            q = w[: cfg.n_heads * D].view(cfg.n_heads, D, H)[r * nq:(r + 1) * nq]
            kh = (r * cfg.n_kv_heads) // tp if kv_rep else r * nkv
            k = w[cfg.n_heads * D:(cfg.n_heads + cfg.n_kv_heads) * D].view(cfg.n_kv_heads, D, H)[kh:kh + nkv]
            v = w[(cfg.n_heads + cfg.n_kv_heads) * D:].view(cfg.n_kv_heads, D, H)[kh:kh + nkv]
            return torch.cat([q.reshape(-1, H), k.reshape(-1, H), v.reshape(-1, H)]).contiguous()

        def cols(n_out, n_in_full, lo, hi, std):
            if not full:
                return self._randn(g, n_out, hi - lo, std=std)
            return self._randn(g, n_out, n_in_full, std=std)[:, lo:hi].contiguous()

        for _ in range(cfg.n_layers):
            L = {
                "in_norm": torch.ones(H, dtype=self.dtype, device=self.device),
                "post_norm": torch.ones(H, dtype=self.dtype, device=self.device),
                "wqkv": qkv_shard(),
                "wo": cols(H, cfg.n_heads * D, r * nq * D, (r + 1) * nq * D, out_std),
            }
            if cfg.n_experts == 0:
                I, Il = cfg.intermediate, self.inter
                if full:
                    gu = self._randn(g, 2 * I, H)
                    L["w_gu"] = torch.cat([gu[r * Il:(r + 1) * Il], gu[I + r * Il: I + (r + 1) * Il]]).contiguous()
                else:
                    L["w_gu"] = self._randn(g, 2 * Il, H)
                L["w_down"] = cols(H, I, r * Il, (r + 1) * Il, out_std)
            self.layers.append(L)
        if cfg.n_experts:
            self.moe = MOE.MoELayerSet(cfg, self.device, self.dtype, self.pc, g, out_std, full_slice=full)
        self.embed = self._randn(g, cfg.vocab_size, H)
        self.final_norm = torch.ones(H, dtype=self.dtype, device=self.device)
        if full:
            lm = self._randn(g, cfg.vocab_size, H)
            pad = self.vocab_local * tp - cfg.vocab_size
            if pad:
                lm = torch.cat([lm, torch.zeros(pad, H, dtype=self.dtype, device=self.device)])
            self.lm_head = lm[r * self.vocab_local:(r + 1) * self.vocab_local].contiguous()
        else:
            self.lm_head = self._randn(g, self.vocab_local, H)

    def weight_bytes(self) -> int:
        n = sum(t.numel() * t.element_size() for L in self.layers for t in L.values())
        n += self.embed.numel() * 2 + self.lm_head.numel() * 2
        if self.moe is not None:
            n += self.moe.weight_bytes()
        return n

    # -------------------------------------------------------------- forward
    def _lm_head(self, y: torch.Tensor) -> torch.Tensor:
        return linear_f32out(y, self.lm_head) if self.logits_f32 else linear(y, self.lm_head)

    def forward(self, inp: StepInputs, k_cache: torch.Tensor, v_cache: torch.Tensor,
                gather_logits: bool = True) -> torch.Tensor:
        """k_cache/v_cache: [n_layers, NB, nkv, BS, D] / [n_layers, NB, nkv, D, BS].
        ``gather_logits=False`` under TP returns this rank's vocab shard
        (columns ``tp_rank * vocab_local ..``) for distributed sampling."""
        cfg = self.cfg
        T = inp.input_ids.shape[0]
        H = cfg.hidden
        residual = F.embedding(inp.input_ids.long(), self.embed)     # [T, H]
        if self._exec is None and LX.LlamaExecutor.eligible(self):
            self._exec = LX.LlamaExecutor(self)
        if self._exec is not None and LX.LlamaExecutor.eligible(self) and self._exec.fits(T):
            # the dense layer stack in one native call (ops/layer_exec.py): same kernels, same order
            prev, residual = self._exec.run(inp, residual, k_cache, v_cache)
            y = torch.empty_like(residual)
            N.rmsnorm(prev, self.final_norm, cfg.rms_eps, residual=residual, out=y)
            sel = y.index_select(0, inp.logits_idx) if inp.logits_idx.numel() != T else y
            logits = self._lm_head(sel)
            return self.pc.all_gather_last(logits) if gather_logits else logits
        prev: Optional[torch.Tensor] = None
        y = torch.empty_like(residual)
        attn = torch.empty((T, self.nq * self.D), dtype=self.dtype, device=self.device)
        nd = inp.n_decode
        for li, L in enumerate(self.layers):
            if prev is None:
                N.rmsnorm(residual, L["in_norm"], cfg.rms_eps, out=y)
            else:
                N.rmsnorm(prev, L["in_norm"], cfg.rms_eps, residual=residual, out=y)
            if self.nf_flags is not None:
                nonfinite_flag(y, self.nf_flags[li:li + 1])
            qkv = A.linear_rope_kv(y, L["wqkv"], inp.positions, self.cos_sin, inp.slots, k_cache[li], v_cache[li],
                                   self.nq, self.nkv)
            if inp.meta_decode is not None and nd > 0:
                A.paged_attention(qkv[:nd], k_cache[li], v_cache[li], inp.meta_decode, self.nq, self.nkv, self.scale,
                                  out=attn[:nd])
            if inp.meta_prefill is not None and nd < T:
                A.paged_attention(qkv[nd:], k_cache[li], v_cache[li], inp.meta_prefill, self.nq, self.nkv,
                                  self.scale, out=attn[nd:])
            o = self.pc.linear_all_reduce(attn, L["wo"], linear_fn=linear)
            N.rmsnorm(o, L["post_norm"], cfg.rms_eps, residual=residual, out=y)
            if self.moe is not None:
                prev = self.moe.forward(li, y)
            else:
                act = swiglu_gemm(y, L["w_gu"])  # gate_up + SwiGLU in one launch where measured faster
                if act is not None:
                    prev = self.pc.linear_all_reduce(act, L["w_down"], linear_fn=linear)
                    continue
                gu = linear(y, L["w_gu"])
                if self.pc.tp_size == 1:
                    prev = linear_silu(gu, L["w_down"])  # SwiGLU fused into the down GEMM's operand staging
                else:
                    prev = self.pc.linear_all_reduce(N.silu_mul(gu), L["w_down"], linear_fn=linear)
        if self.nf_flags is not None:
            nonfinite_flag(prev, self.nf_flags[len(self.layers):])
        N.rmsnorm(prev, self.final_norm, cfg.rms_eps, residual=residual, out=y)
        sel = y.index_select(0, inp.logits_idx) if inp.logits_idx.numel() != T else y
        logits = self._lm_head(sel)
        return self.pc.all_gather_last(logits) if gather_logits else logits
