"""Paged KV pool (B5 storage) sized for 288 GB of HBM.

One allocation per layer stack:
``k[L, NB, n_kv, BS, D]`` and ``v[L, NB, n_kv, D, BS]`` (V pages transposed,
see ``csrc/kernels/attention.hip``).  Blocks are handed out from a free list;
a conversation thread keeps its blocks across runs (prefix reuse) until the
scheduler evicts it under memory pressure.

Cross-thread prefix sharing: a *full* block whose tokens were written by a
prefill is registered under a chain key ``(key of the previous block, its
token ids)``, so every thread whose token list starts with the same blocks
(the assistants' system prompts and seeding messages: ~0.5-1.2k tokens each,
identical across all concurrent RCA pipelines) maps them to the same physical
pages instead of prefilling and storing its own copy.  Blocks are
reference-counted; a registered block is never written again (writers only
touch positions >= their ``n_cached``, and a thread whose history diverges
inside a shared block drops it and recomputes that block privately), and it
is unregistered when its last holder releases it.  Decode then reads the
shared pages of many sequences from the same addresses, which HBM traffic
pays for once per step (L2 / MALL hits) instead of once per sequence.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch


def chain_key(parent: int, tokens) -> int:
    """Key of a full block given its predecessor's key (0 for block 0)."""
    return hash((parent, tuple(tokens)))


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
        self._ref = np.zeros(num_blocks, dtype=np.int32)
        self._key_of: Dict[int, int] = {}   # registered block -> chain key
        self._by_key: Dict[int, int] = {}   # chain key -> block
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
            self._ref[out] = 1
            self.peak_used = max(self.peak_used, self.num_blocks - len(self._free))
        return out

    def release(self, blocks: List[int]) -> int:
        """Drop one reference to each block; returns how many went back to the free list."""
        if not blocks:
            return 0
        freed = 0
        with self._lock:
            for b in reversed(blocks):
                r = self._ref[b] - 1
                self._ref[b] = r
                if r == 0:
                    k = self._key_of.pop(b, None)
                    if k is not None and self._by_key.get(k) == b:
                        del self._by_key[k]
                    self._free.append(b)
                    freed += 1
                elif r < 0:
                    raise RuntimeError(f"KV block {b} released more often than it was taken")
        return freed

    # ------------------------------------------------------ prefix sharing
    def lookup(self, key: int) -> Optional[int]:
        """Take a reference on the registered block with chain key ``key``."""
        with self._lock:
            b = self._by_key.get(key)
            if b is not None:
                self._ref[b] += 1
            return b

    def register(self, block: int, key: int) -> None:
        """Publish a fully written block (first writer wins for a given key)."""
        with self._lock:
            if key not in self._by_key and block not in self._key_of:
                self._by_key[key] = block
                self._key_of[block] = key

    def is_shared(self, block: int) -> bool:
        return int(self._ref[block]) > 1

    def make_private(self, block: int) -> bool:
        """Before its owner overwrites part of ``block``: unregister it.  False
        if other sequences hold it (the owner must drop it instead)."""
        with self._lock:
            if self._ref[block] > 1:
                return False
            k = self._key_of.pop(block, None)
            if k is not None and self._by_key.get(k) == block:
                del self._by_key[k]
            return True

    @property
    def shared_blocks(self) -> int:
        return int((self._ref > 1).sum())

    def reset_peak(self) -> None:
        self.peak_used = self.num_blocks - len(self._free)

    def utilization(self) -> float:
        return 1.0 - len(self._free) / max(1, self.num_blocks)
