"""Process groups for tensor / expert parallelism (one process per GPU).

``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm; intra-node
traffic rides xGMI.  TP shards attention heads and the MLP intermediate
(column-parallel QKV / gate_up, row-parallel O / down: two all-reduces per
layer) and the vocabulary (lm_head); EP places whole experts on ranks and
moves tokens with all-to-all.  ``gloo`` runs the same code on CPU for tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelContext:
    tp_size: int = 1
    tp_rank: int = 0
    tp_group: Optional[object] = None
    ep_size: int = 1
    ep_rank: int = 0
    ep_group: Optional[object] = None
    comm_stream: Optional[object] = None  # HIP stream for overlapped collectives

    @property
    def is_tp(self) -> bool:
        return self.tp_size > 1

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            dist.all_reduce(t, group=self.tp_group)
        return t

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        """[n, v_local] on every rank -> [n, v_local * tp] (rank-major)."""
        if self.tp_size == 1:
            return t
        parts = [torch.empty_like(t) for _ in range(self.tp_size)]
        dist.all_gather(parts, t.contiguous(), group=self.tp_group)
        return torch.cat(parts, dim=-1)


def init_distributed(backend: Optional[str] = None) -> ParallelContext:
    """Initialise from torchrun env vars; returns a TP context spanning the world."""
    if not dist.is_available():
        return ParallelContext()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return ParallelContext()
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend)
    r = dist.get_rank()
    return ParallelContext(tp_size=world, tp_rank=r, tp_group=dist.group.WORLD, ep_size=world, ep_rank=r,
                           ep_group=dist.group.WORLD)


def single() -> ParallelContext:
    return ParallelContext()
