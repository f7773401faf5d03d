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
    custom_ar: Optional[object] = None    # parallel.xgmi.XgmiAllReduce for small TP messages

    @property
    def is_tp(self) -> bool:
        return self.tp_size > 1

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            car = self.custom_ar
            if car is not None and car.mode_for(t):
                return car(t)
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
    pc = ParallelContext(tp_size=world, tp_rank=r, tp_group=dist.group.WORLD, ep_size=world, ep_rank=r,
                         ep_group=dist.group.WORLD)
    attach_custom_allreduce(pc)
    return pc


def attach_custom_allreduce(pc: ParallelContext) -> ParallelContext:
    """Give a GPU TP context the xGMI one/two-shot all-reduce for small
    messages (``K8S_RCA_CUSTOM_AR=0`` keeps every all-reduce on RCCL)."""
    if (pc.tp_size > 1 and torch.cuda.is_available() and os.environ.get("K8S_RCA_CUSTOM_AR", "1") != "0"
            and dist.get_backend(pc.tp_group) == "nccl"):
        try:
            from .xgmi import XgmiAllReduce
            pc.custom_ar = XgmiAllReduce(pc.tp_group)
        except Exception as e:  # noqa: BLE001 - RCCL remains correct, only slower for small messages
            import logging
            logging.getLogger(__name__).warning("xGMI all-reduce unavailable (%s); using RCCL", e)
    return pc


def single() -> ParallelContext:
    return ParallelContext()
