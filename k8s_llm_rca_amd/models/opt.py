"""OPT-125m decoder -- the CPU plumbing backend (BASELINE.json config 1, B16).

Pre-LayerNorm blocks, learned positions (offset 2), ReLU FFN, MHA with
biases, lm_head tied to the token embedding.  Uses the same paged KV pool and
``StepInputs`` contract as :class:`~.llama.LlamaModel`, so the engine,
scheduler and assistant semantics are exercised identically on CPU.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from ..ops import attention as A
from .config import ModelConfig


class OPTModel:
    POS_OFFSET = 2

    def __init__(self, cfg: ModelConfig, device, dtype=torch.float32, seed: int = 0, init: bool = True):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.nq = self.nkv = cfg.n_heads
        self.D = cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.layers = []
        if init:
            g = torch.Generator(device=self.device)
            g.manual_seed(seed)
            H, I = cfg.hidden, cfg.intermediate

            def rnd(*s):
                t = torch.empty(*s, dtype=dtype, device=self.device)
                return t.normal_(0.0, cfg.init_std, generator=g)

            def z(*s):
                return torch.zeros(*s, dtype=dtype, device=self.device)

            def o(*s):
                return torch.ones(*s, dtype=dtype, device=self.device)

            for _ in range(cfg.n_layers):
                self.layers.append({"ln1_w": o(H), "ln1_b": z(H), "wqkv": rnd(3 * H, H), "bqkv": z(3 * H),
                                    "wo": rnd(H, H), "bo": z(H), "ln2_w": o(H), "ln2_b": z(H),
                                    "fc1": rnd(I, H), "b1": z(I), "fc2": rnd(H, I), "b2": z(H)})
            self.embed = rnd(cfg.vocab_size, H)
            self.pos = rnd(cfg.max_position + self.POS_OFFSET, H)
            self.lnf_w, self.lnf_b = o(H), z(H)

    def forward(self, inp, k_cache: torch.Tensor, v_cache: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        T = inp.input_ids.shape[0]
        H = cfg.hidden
        x = F.embedding(inp.input_ids.long(), self.embed) + F.embedding(inp.positions.long() + self.POS_OFFSET,
                                                                         self.pos)
        nd = inp.n_decode
        for li, L in enumerate(self.layers):
            h = F.layer_norm(x, (H,), L["ln1_w"], L["ln1_b"])
            qkv = F.linear(h, L["wqkv"], L["bqkv"])
            q, k, v = qkv.split(H, dim=-1)
            A.kv_write(k.view(T, self.nkv, self.D), v.view(T, self.nkv, self.D), inp.slots, k_cache[li], v_cache[li])
            attn = torch.empty(T, H, dtype=x.dtype, device=x.device)
            if inp.meta_decode is not None and nd > 0:
                A.paged_attention(q[:nd], k_cache[li], v_cache[li], inp.meta_decode, self.nq, self.nkv, self.scale,
                                  out=attn[:nd])
            if inp.meta_prefill is not None and nd < T:
                A.paged_attention(q[nd:], k_cache[li], v_cache[li], inp.meta_prefill, self.nq, self.nkv, self.scale,
                                  out=attn[nd:])
            x = x + F.linear(attn, L["wo"], L["bo"])
            h = F.layer_norm(x, (H,), L["ln2_w"], L["ln2_b"])
            x = x + F.linear(F.relu(F.linear(h, L["fc1"], L["b1"])), L["fc2"], L["b2"])
        x = F.layer_norm(x, (H,), self.lnf_w, self.lnf_b)
        sel = x.index_select(0, inp.logits_idx)
        return F.linear(sel, self.embed)
