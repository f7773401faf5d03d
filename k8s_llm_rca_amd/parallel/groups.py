"""Process groups for tensor / expert parallelism (one process per GPU).

``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm; intra-node
traffic rides xGMI.  TP shards attention heads and the MLP intermediate
(column-parallel QKV / gate_up, row-parallel O / down: two all-reduces per
layer) and the vocabulary (lm_head); EP places whole experts on ranks and
moves tokens with all-to-all.  ``gloo`` runs the same code on CPU for tests.
"""
from __future__ import annotations

from ..knobs import KNOBS
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
    ar_chunks: int = 4                    # GEMM / all-reduce pipeline depth (linear_all_reduce)
    overlap_min_bytes: int = 256 << 10    # below this an all-reduce is latency-bound: no chunking
    # every TP / EP data collective on the xGMI kernels (larger-than-buffer
    # messages in buffer-sized chunks): no RCCL call on the data path.  Required
    # when ranks share one GPU (RCCL refuses duplicate devices), and the mode a
    # TP group runs in whenever its communicator is up (attach_custom_allreduce)
    xgmi_only: bool = False
    # pipeline depth per row-count bucket, timed on this fabric at init
    # (tune_overlap): the bucket at or above M, else ar_chunks
    chunk_plan: Optional[dict] = None
    # transport per row-count bucket (tune_overlap, same lookup): True = RCCL
    # (torch.distributed "nccl") for that step's all-reduces, False = the xGMI
    # kernels.  None: xGMI whenever the communicator takes the message.
    rccl_plan: Optional[dict] = None

    @staticmethod
    def _bucket(plan: Optional[dict], M: int, default):
        if plan:
            for b in sorted(plan):
                if b >= M:
                    return plan[b]
        return default

    def chunks_for(self, M: int) -> int:
        return self._bucket(self.chunk_plan, M, self.ar_chunks)

    def rccl_for(self, M: int) -> bool:
        """This M-row step's all-reduces go to RCCL (the tuned plan's pick)."""
        return bool(self._bucket(self.rccl_plan, M, False))

    def rccl_ok(self) -> bool:
        """RCCL can carry this group's data: a "nccl" group (one device per rank;
        RCCL refuses ranks that share a GPU, so a loopback rehearsal is gloo)."""
        return self.tp_size > 1 and self.tp_group is not None and dist.get_backend(self.tp_group) == "nccl"

    def _time_candidate(self, shapes, x, k: int, rccl: bool, iters: int) -> float:
        """us per (o, down) pair of :meth:`linear_all_reduce` with depth ``k``
        on one transport (every rank runs the same calls in lockstep)."""
        import time
        dev = shapes[0][1].device
        cuda = dev.type == "cuda"
        self.chunk_plan, self.rccl_plan = {1 << 30: k}, {1 << 30: rccl}
        for name, w in shapes:  # warm, and every rank enters this candidate together
            self.linear_all_reduce(x[name], w)
        if cuda:
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            for name, w in shapes:
                self.linear_all_reduce(x[name], w)
        if cuda:
            torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e6 / iters

    def tune_overlap(self, shapes, buckets, depths=(1, 2, 4), iters: int = 4, rounds: int = 3,
                     transports=None) -> dict:
        """Per row-count bucket T, the GEMM / all-reduce pipeline depth of
        :meth:`linear_all_reduce` (1 = no overlap: GEMM, then one all-reduce;
        k = k row chunks, chunk i's all-reduce on the comm stream beside chunk
        i+1's GEMM) AND its transport -- the xGMI kernels (two-shot over the
        hipIpc buffers, buffer-sized chunks past it) or RCCL's multi-channel
        rings (the north star's RCCL path is measured against
        the custom kernels per bucket, not assumed away) -- timed ON THIS
        FABRIC with the real row-parallel weights [(name, w [H, K_local])].
        ``transports``: subset of ("xgmi", "rccl"); default every one this
        group can run (RCCL needs a "nccl" group, xGMI the communicator).
        Every rank runs the same collectives in lockstep and each timing is
        max-reduced over the TP group, so all ranks hold the same plan
        (``chunk_plan``, ``rccl_plan``); the report goes into the bench line."""
        if self.tp_size == 1:
            return {}
        dev = shapes[0][1].device
        cuda = dev.type == "cuda"
        if transports is None:
            transports = tuple(t for t, ok in (("xgmi", self.custom_ar is not None and cuda),
                                                ("rccl", self.rccl_ok() or not cuda)) if ok)
        cands = [(tr, k) for tr in transports for k in depths]
        report, plan, rplan = {}, {}, {}
        saved = (self.chunk_plan, self.rccl_plan)
        for T in sorted(set(int(b) for b in buckets)):
            x = {name: torch.randn(T, int(w.shape[1]), device=dev).to(w.dtype) for name, w in shapes}
            us = {c: [] for c in cands}
            try:
                for _ in range(rounds):
                    for tr, k in cands:
                        us[(tr, k)].append(self._time_candidate(shapes, x, k, tr == "rccl", iters))
            finally:
                self.chunk_plan, self.rccl_plan = saved
            med = torch.tensor([sorted(v)[len(v) // 2] for v in us.values()], dtype=torch.float64)
            on_dev = cuda and dist.get_backend(self.tp_group) == "nccl"
            t = med.to(dev) if on_dev else med
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.tp_group)  # the slowest rank's view
            med = t.cpu().tolist()
            best = min(range(len(cands)), key=lambda i: (med[i], i))
            tr, k = cands[best]
            plan[T], rplan[T] = k, tr == "rccl"
            report[T] = {(f"k{k_}" if tr_ == "xgmi" else f"{tr_}_k{k_}"): round(v, 1)
                         for (tr_, k_), v in zip(cands, med)}
            report[T]["pick"] = k
            report[T]["transport"] = tr
        self.chunk_plan, self.rccl_plan = plan, rplan
        return report

    @property
    def is_tp(self) -> bool:
        return self.tp_size > 1

    def _xgmi(self, t: torch.Tensor, rccl: bool = False) -> bool:
        car = self.custom_ar
        return (not rccl and car is not None and t.is_cuda
                and (car.mode_for(t) != 0 or (self.xgmi_only and car.eligible(t))))

    def all_reduce(self, t: torch.Tensor, rccl: Optional[bool] = None) -> torch.Tensor:
        """Sum ``t`` over the TP group in place.  ``rccl``: the transport the
        tuned plan picked for this step (default: by ``t``'s row count)."""
        if self.tp_size > 1:
            if rccl is None:
                rccl = bool(self.rccl_plan) and t.dim() > 0 and self.rccl_for(t.shape[0])
            if self._xgmi(t, rccl):
                return self.custom_ar(t)
            if self.xgmi_only and t.is_cuda and not rccl:
                raise ValueError(f"xgmi_only: a {t.dtype} all-reduce of shape {tuple(t.shape)} has no xGMI path")
            dist.all_reduce(t, group=self.tp_group)
        return t

    def _all_reduce_async(self, t: torch.Tensor, rccl: bool = False):
        """Start an all-reduce of ``t`` that overlaps later work on the compute
        stream; returns a handle whose ``wait()`` orders the compute stream
        after it."""
        car = self.custom_ar
        if self._xgmi(t, rccl):
            cur = torch.cuda.current_stream(t.device)
            if self.comm_stream is None:
                self.comm_stream = torch.cuda.Stream(t.device)
            s = self.comm_stream
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                car(t)
            ev = torch.cuda.Event()
            ev.record(s)
            t.record_stream(s)

            class _W:
                def wait(self_inner):
                    cur.wait_event(ev)
            return _W()
        return dist.all_reduce(t, group=self.tp_group, async_op=True)

    def linear_all_reduce(self, x: torch.Tensor, w: torch.Tensor, linear_fn=None) -> torch.Tensor:
        """Row-parallel projection ``all_reduce(x @ w^T)`` with the reduction of
        chunk i overlapped with the GEMM of chunk i+1 (RCCL / the xGMI kernel
        run on their own streams).  Decode-sized M splits the OUTPUT COLUMNS
        (each chunk streams a disjoint weight slice: no weight byte is read
        twice); prefill-sized M splits the rows (contiguous, no copies)."""
        import torch.nn.functional as F
        lin = linear_fn or F.linear
        if self.tp_size == 1:
            return lin(x, w)
        M, N = x.shape[0], w.shape[0]
        k = self.chunks_for(M)
        rccl = bool(self.rccl_plan) and self.rccl_for(M)
        if k <= 1 or M * N * x.element_size() < self.overlap_min_bytes * k:
            return self.all_reduce(lin(x, w), rccl=rccl)
        works, parts = [], []
        if M <= 256:
            step = -(-N // k)
            step = -(-step // 8) * 8
            for a in range(0, N, step):
                y = lin(x, w[a:a + step]).contiguous()
                works.append(self._all_reduce_async(y, rccl))
                parts.append(y)
            for h in works:
                h.wait()
            return torch.cat(parts, dim=1)
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        step = -(-M // k)
        for a in range(0, M, step):
            y = out[a:a + step]
            torch.matmul(x[a:a + step], w.t(), out=y)  # prefill-sized: library GEMM straight into the slice
            works.append(self._all_reduce_async(y, rccl))
        for h in works:
            h.wait()
        return out

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        """[n, v_local] on every rank -> [n, v_local * tp] (rank-major)."""
        if self.tp_size == 1:
            return t
        car = self.custom_ar
        if car is not None and t.is_cuda:  # device-side, any size (buffer-sized pieces)
            g = car.all_gather(t)                                   # [tp, n, v_local]
            return g.permute(1, 0, *range(2, g.dim())).reshape(*t.shape[:-1], -1)
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


# grid cap of the xGMI collectives when the TP ranks share one GPU
SHARED_GPU_AR_BLOCKS = 32


def attach_custom_allreduce(pc: ParallelContext, same_gpu: bool = False) -> ParallelContext:
    """Give a GPU TP context the xGMI communicator (``parallel/xgmi.py``):
    one-/two-shot all-reduce, fused all-reduce + add + RMSNorm, all-to-all and
    all-gather over hipIpc-mapped peer buffers, every data collective on it
    (``xgmi_only``).  Knob ``custom_ar=0`` (``K8SRCA_CUSTOM_AR``) keeps every collective on RCCL.
    ``same_gpu``: the ranks share one device over a gloo group (the one-GPU
    rehearsal of a TP deployment: RCCL refuses duplicate devices, so the xGMI
    kernels are the only data path and a failure to map them is fatal)."""
    if pc.tp_size > 1 and torch.cuda.is_available() and KNOBS.custom_ar:
        from .xgmi import XgmiAllReduce
        # 64 MiB: every TP all-reduce up to 4,096 tokens of 70B (8,192 x bf16) in one xGMI
        # two-shot, which reads the N-1 peers over N-1 links at once; larger ones in
        # 64 MiB chunks (640 MiB of uncached HBM a rank)
        mb = KNOBS.ar_max_mb
        nccl = dist.get_backend(pc.tp_group) == "nccl"
        if not nccl and not same_gpu:
            return pc  # a gloo group on separate devices (CPU-side tests): the dist.* collectives
        try:
            # ranks sharing one GPU: cap the collectives' grids so a rank's blocks spinning for
            # its peer never hold every CU its peer's next kernel needs (XgmiAllReduce max_blocks)
            pc.custom_ar = XgmiAllReduce(pc.tp_group, max_bytes=mb << 20, timeout_s=60.0 if same_gpu else 10.0,
                                         max_blocks=SHARED_GPU_AR_BLOCKS if same_gpu else None)
            pc.xgmi_only = True
        except Exception as e:  # noqa: BLE001
            if same_gpu:
                raise  # RCCL cannot run two ranks on one device: nothing to fall back to
            import logging
            logging.getLogger(__name__).warning("xGMI all-reduce unavailable (%s); using RCCL", e)
    return pc


def single() -> ParallelContext:
    return ParallelContext()
