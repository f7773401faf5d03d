"""Checkpoint IO: Hugging-Face-format safetensors <-> the engine's sharded layout.

SURVEY.md §5.4: benchmarks use seeded random weights, but a user switching
from the reference (GPT-4 behind an API) wants real open weights.  This loads
a HF Llama-3 / Mixtral checkpoint directory (``config.json`` + ``*.safetensors``
+ ``tokenizer.json``) straight into this rank's tensor-parallel shards:

  q/k/v_proj        -> ``wqkv`` rows [q heads of this rank | kv heads | kv heads]
  gate/up_proj      -> ``w_gu`` [gate shard | up shard]          (dense MLP)
  o_proj, down_proj -> column shards (row-parallel)
  block_sparse_moe  -> router, ``w13[e] = [w1 | w3]``, ``w2[e]`` for this rank's experts
  lm_head           -> vocab shard (padded to tp * vocab_local); tied to the
                       embedding when the checkpoint has none

Only the shards a rank needs are read (``safe_open`` slices lazily).  RoPE uses
the rotate-half convention of HF checkpoints (``ops/attention.py``), so no q/k
permutation is needed.  ``save_safetensors`` writes the same names back (TP=1).
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch

from .config import ModelConfig


def config_from_hf(path: str, name: Optional[str] = None) -> ModelConfig:
    d = json.load(open(os.path.join(path, "config.json") if os.path.isdir(path) else path))
    arch = "mixtral" if d.get("num_local_experts") else "llama"
    rs = d.get("rope_scaling")
    kw = dict(rope_theta=float(d.get("rope_theta", 10000.0)), max_position=int(d.get("max_position_embeddings", 8192)),
              rms_eps=float(d.get("rms_norm_eps", 1e-5)), tie_embeddings=bool(d.get("tie_word_embeddings", False)))
    if d.get("head_dim"):
        kw["head_dim"] = int(d["head_dim"])
    if arch == "mixtral":
        kw.update(n_experts=int(d["num_local_experts"]), top_k=int(d.get("num_experts_per_tok", 2)))
    if rs and rs.get("rope_type", rs.get("type")) == "llama3":
        kw["rope_scaling"] = tuple(sorted((k, v) for k, v in rs.items() if isinstance(v, (int, float))))
    return ModelConfig(name or os.path.basename(os.path.normpath(path)), arch, int(d["vocab_size"]),
                       int(d["hidden_size"]), int(d["num_hidden_layers"]), int(d["num_attention_heads"]),
                       int(d.get("num_key_value_heads", d["num_attention_heads"])), int(d["intermediate_size"]),
                       **kw)


class _Reader:
    def __init__(self, path: str):
        from safetensors import safe_open
        files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
        if not files:
            raise FileNotFoundError(f"no *.safetensors under {path}")
        self._h = [safe_open(f, framework="pt", device="cpu") for f in files]
        self._where: Dict[str, int] = {}
        for i, h in enumerate(self._h):
            for k in h.keys():
                self._where[k] = i

    def has(self, name: str) -> bool:
        return name in self._where

    def get(self, name: str, rows: Optional[slice] = None, cols: Optional[slice] = None) -> torch.Tensor:
        sl = self._h[self._where[name]].get_slice(name)
        if rows is not None and cols is not None:
            return sl[rows, cols]
        if rows is not None:
            return sl[rows]
        if cols is not None:
            return sl[:, cols]
        return sl[:]


def load_safetensors(model, path: str) -> None:
    """Fill ``model`` (a LlamaModel built with ``init=False``) from a HF checkpoint."""
    from . import moe as MOE
    cfg = model.cfg
    pc = model.pc
    tp, r = pc.tp_size, pc.tp_rank
    H, D = cfg.hidden, model.D
    nq, nkv = model.nq, model.nkv
    kh = (r * cfg.n_kv_heads) // tp if cfg.n_kv_heads < tp else r * nkv
    dev, dt = model.device, model.dtype
    R = _Reader(path)

    def put(t: torch.Tensor) -> torch.Tensor:
        return t.to(device=dev, dtype=dt).contiguous()

    model.layers = []
    for i in range(cfg.n_layers):
        p = f"model.layers.{i}."
        q = R.get(p + "self_attn.q_proj.weight", rows=slice(r * nq * D, (r + 1) * nq * D))
        k = R.get(p + "self_attn.k_proj.weight", rows=slice(kh * D, (kh + nkv) * D))
        v = R.get(p + "self_attn.v_proj.weight", rows=slice(kh * D, (kh + nkv) * D))
        L = {"in_norm": put(R.get(p + "input_layernorm.weight")),
             "post_norm": put(R.get(p + "post_attention_layernorm.weight")),
             "wqkv": put(torch.cat([q, k, v])),
             "wo": put(R.get(p + "self_attn.o_proj.weight", cols=slice(r * nq * D, (r + 1) * nq * D)))}
        if cfg.n_experts == 0:
            Il = model.inter
            g = R.get(p + "mlp.gate_proj.weight", rows=slice(r * Il, (r + 1) * Il))
            u = R.get(p + "mlp.up_proj.weight", rows=slice(r * Il, (r + 1) * Il))
            L["w_gu"] = put(torch.cat([g, u]))
            L["w_down"] = put(R.get(p + "mlp.down_proj.weight", cols=slice(r * Il, (r + 1) * Il)))
        model.layers.append(L)
    if cfg.n_experts:
        ms = MOE.MoELayerSet.__new__(MOE.MoELayerSet)
        ms.cfg, ms.pc, ms.E, ms.k = cfg, pc, cfg.n_experts, cfg.top_k
        ms.E_local = cfg.n_experts // pc.ep_size
        ms.e0 = pc.ep_rank * ms.E_local
        ms.router, ms.w13, ms.w2 = [], [], []
        for i in range(cfg.n_layers):
            p = f"model.layers.{i}.block_sparse_moe."
            ms.router.append(put(R.get(p + "gate.weight")))
            w13, w2 = [], []
            for e in range(ms.e0, ms.e0 + ms.E_local):
                w13.append(torch.cat([R.get(p + f"experts.{e}.w1.weight"), R.get(p + f"experts.{e}.w3.weight")]))
                w2.append(R.get(p + f"experts.{e}.w2.weight"))
            ms.w13.append(put(torch.stack(w13)))
            ms.w2.append(put(torch.stack(w2)))
        model.moe = ms
    model.embed = put(R.get("model.embed_tokens.weight"))
    model.final_norm = put(R.get("model.norm.weight"))
    V, vl = cfg.vocab_size, model.vocab_local
    lo, hi = r * vl, min(V, (r + 1) * vl)
    lm_name = "lm_head.weight" if R.has("lm_head.weight") else "model.embed_tokens.weight"
    lm = R.get(lm_name, rows=slice(lo, hi)) if hi > lo else torch.zeros(0, H)
    if lm.shape[0] < vl:
        lm = torch.cat([lm, torch.zeros(vl - lm.shape[0], H, dtype=lm.dtype)])
    model.lm_head = put(lm)


def save_safetensors(model, path: str, config_json: bool = True) -> None:
    """Write a TP=1 model in HF naming (checkpointing a seeded model, tests)."""
    from safetensors.torch import save_file
    cfg = model.cfg
    if model.pc.tp_size != 1 or (model.moe is not None and model.pc.ep_size != 1):
        raise ValueError("save_safetensors needs the unsharded (TP=1, EP=1) model")
    H, D = cfg.hidden, model.D
    out: Dict[str, torch.Tensor] = {}
    for i, L in enumerate(model.layers):
        p = f"model.layers.{i}."
        q, k, v = torch.split(L["wqkv"], [cfg.n_heads * D, cfg.n_kv_heads * D, cfg.n_kv_heads * D])
        out[p + "self_attn.q_proj.weight"] = q
        out[p + "self_attn.k_proj.weight"] = k
        out[p + "self_attn.v_proj.weight"] = v
        out[p + "self_attn.o_proj.weight"] = L["wo"]
        out[p + "input_layernorm.weight"] = L["in_norm"]
        out[p + "post_attention_layernorm.weight"] = L["post_norm"]
        if "w_gu" in L:
            g, u = torch.split(L["w_gu"], [cfg.intermediate, cfg.intermediate])
            out[p + "mlp.gate_proj.weight"] = g
            out[p + "mlp.up_proj.weight"] = u
            out[p + "mlp.down_proj.weight"] = L["w_down"]
    if model.moe is not None:
        for i in range(cfg.n_layers):
            p = f"model.layers.{i}.block_sparse_moe."
            out[p + "gate.weight"] = model.moe.router[i]
            for e in range(cfg.n_experts):
                w1, w3 = torch.split(model.moe.w13[i][e], [cfg.intermediate, cfg.intermediate])
                out[p + f"experts.{e}.w1.weight"] = w1
                out[p + f"experts.{e}.w3.weight"] = w3
                out[p + f"experts.{e}.w2.weight"] = model.moe.w2[i][e]
    out["model.embed_tokens.weight"] = model.embed
    out["model.norm.weight"] = model.final_norm
    out["lm_head.weight"] = model.lm_head[: cfg.vocab_size]
    os.makedirs(path, exist_ok=True)
    save_file({k: v.detach().contiguous().cpu() for k, v in out.items()}, os.path.join(path, "model.safetensors"))
    if config_json:
        d = {"vocab_size": cfg.vocab_size, "hidden_size": H, "num_hidden_layers": cfg.n_layers,
             "num_attention_heads": cfg.n_heads, "num_key_value_heads": cfg.n_kv_heads,
             "intermediate_size": cfg.intermediate, "rope_theta": cfg.rope_theta,
             "max_position_embeddings": cfg.max_position, "rms_norm_eps": cfg.rms_eps, "head_dim": D,
             "tie_word_embeddings": False}
        # HF loaders (transformers' LlamaForCausalLM / MixtralForCausalLM) read these too
        d.update(model_type="mixtral" if cfg.n_experts else "llama", hidden_act="silu", attention_bias=False,
                 mlp_bias=False, architectures=["MixtralForCausalLM" if cfg.n_experts else "LlamaForCausalLM"])
        if cfg.n_experts:
            d.update(num_local_experts=cfg.n_experts, num_experts_per_tok=cfg.top_k, router_jitter_noise=0.0)
        if cfg.rope_scaling:
            d["rope_scaling"] = dict(cfg.rope_scaling, rope_type="llama3")
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(d, f, indent=1)
