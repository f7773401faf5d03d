"""Paged KV pool (B5 storage) sized for 288 GB of HBM.

One allocation per layer stack:
``k[L, NB, n_kv, BS, D]`` and ``v[L, NB, n_kv, D, BS]`` (V pages transposed,
see ``csrc/kernels/attention.hip``).  Blocks are handed out from a free list;
a conversation thread keeps its blocks across runs (prefix reuse) until the
scheduler evicts it under memory pressure.
"""
from __future__ import annotations

import threading
from typing import List

import torch


class KVPool:
    def __init__(self, n_layers: int, n_kv: int, head_dim: int, num_blocks: int, block_size: int, device,
                 dtype=torch.bfloat16):
        if block_size % 32:
            raise ValueError("block_size must be a multiple of 32")
        self.L, self.nkv, self.D = n_layers, n_kv, head_dim
        self.num_blocks = num_blocks
        self.block_size = block_size
        # zero-filled: stale pages never hold NaN (masked keys multiply V by 0)
        self.k = torch.zeros(n_layers, num_blocks, n_kv, block_size, head_dim, dtype=dtype, device=device)
        self.v = torch.zeros(n_layers, num_blocks, n_kv, head_dim, block_size, dtype=dtype, device=device)
        self._free: List[int] = list(range(num_blocks - 1, -1, -1))
        self.peak_used = 0
        self._lock = threading.Lock()

    @staticmethod
    def bytes_per_block(n_layers: int, n_kv: int, head_dim: int, block_size: int, elem: int = 2) -> int:
        return 2 * n_layers * n_kv * head_dim * block_size * elem

    @property
    def free_blocks(self) -> int:
        return len(self._free)

    def alloc(self, n: int) -> List[int]:
        with self._lock:
            if n > len(self._free):
                raise MemoryError(f"KV pool exhausted: need {n}, have {len(self._free)}")
            out = [self._free.pop() for _ in range(n)]
            self.peak_used = max(self.peak_used, self.num_blocks - len(self._free))
        return out

    def release(self, blocks: List[int]) -> None:
        if not blocks:
            return
        with self._lock:
            self._free.extend(reversed(blocks))

    def reset_peak(self) -> None:
        self.peak_used = self.num_blocks - len(self._free)

    def utilization(self) -> float:
        return 1.0 - len(self._free) / max(1, self.num_blocks)
