"""Model presets for every backend named in BASELINE.json.

Shapes are the public architectures (SURVEY.md §2 Part B):
Llama-3-8B / 70B (GQA, RoPE theta 5e5), Mixtral-8x7B (8 experts top-2, theta
1e6, vocab 32000) and OPT-125m (LayerNorm, ReLU, learned positions; the CPU
plumbing backend).  ``tiny-*`` presets keep the same structure at test size.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str                 # 'llama' | 'mixtral' | 'opt'
    vocab_size: int
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    intermediate: int
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: Optional[tuple] = None  # tuple(sorted(dict.items())) to stay hashable
    rms_eps: float = 1e-5
    max_position: int = 8192
    n_experts: int = 0
    top_k: int = 0
    tie_embeddings: bool = False
    init_std: float = 0.02

    @property
    def q_size(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.n_kv_heads * self.head_dim

    def param_count(self) -> int:
        h, i, L = self.hidden, self.intermediate, self.n_layers
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        mlp = 3 * h * i * max(1, self.n_experts) + (h * self.n_experts if self.n_experts else 0)
        emb = self.vocab_size * h * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * h) + emb + h

    def scaling_dict(self) -> Optional[dict]:
        return dict(self.rope_scaling) if self.rope_scaling else None


PRESETS: Dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig("llama3-8b", "llama", 128256, 4096, 32, 32, 8, 14336),
    "llama3-70b": ModelConfig("llama3-70b", "llama", 128256, 8192, 80, 64, 8, 28672),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", "mixtral", 32000, 4096, 32, 32, 8, 14336, rope_theta=1e6,
                                max_position=32768, n_experts=8, top_k=2),
    "opt-125m": ModelConfig("opt-125m", "opt", 50272, 768, 12, 12, 12, 3072, head_dim=64, max_position=2048,
                            tie_embeddings=True),
    # test-size models with the same structure
    "tiny-llama": ModelConfig("tiny-llama", "llama", 8192, 512, 2, 8, 2, 1024, max_position=8192),
    "tiny-llama-g8": ModelConfig("tiny-llama-g8", "llama", 8192, 1024, 2, 8, 1, 1024, max_position=8192),
    "tiny-mixtral": ModelConfig("tiny-mixtral", "mixtral", 8192, 512, 2, 8, 2, 512, rope_theta=1e6,
                                max_position=8192, n_experts=4, top_k=2),
    "tiny-opt": ModelConfig("tiny-opt", "opt", 8192, 256, 2, 4, 4, 512, head_dim=64, max_position=4096,
                            tie_embeddings=True),
}


def get_config(name: str, **overrides) -> ModelConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    c = PRESETS[name]
    return replace(c, **overrides) if overrides else c
