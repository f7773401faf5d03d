"""Custom one-shot / two-shot all-reduce over xGMI peer memory (B14).

``csrc/kernels/allreduce.hip`` does the work; this module sets up the IPC
buffers: every rank allocates one uncached buffer, exports it with
``hipIpcGetMemHandle``, the 64-byte handles are exchanged with
``all_gather_object`` on the TP group, and every rank maps every peer's buffer.

Selection (``XgmiAllReduce.mode_for``): one-shot up to 512 KiB (each rank reads
all peers: latency-optimal), two-shot up to ``max_bytes`` (reduce-scatter +
all-gather through the same buffers: 2(N-1)/N of the bytes), RCCL beyond.
The TP decode all-reduces of the 70B config (16 KiB .. 4 MiB) land in the
custom path; prefill-sized messages stay on RCCL's multi-channel rings.
"""
from __future__ import annotations

import ctypes
import logging
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops._lib import lib, stream_ptr

log = logging.getLogger(__name__)

ONE_SHOT_MAX = 512 << 10


class CommFault(RuntimeError):
    """A TP / EP collective timed out on this rank (a peer never arrived):
    every run in flight on the engine fails, and so does every later one."""


def _bind(L) -> None:
    if getattr(L, "_ar_bound", False):
        return
    c_long, c_int, P = ctypes.c_long, ctypes.c_int, ctypes.c_void_p
    sigs = {
        "k8s_ar_buffer_bytes": ([c_long], c_long),
        "k8s_ar_alloc": ([c_long, ctypes.POINTER(P)], c_int),
        "k8s_ar_free": ([P], c_int),
        "k8s_ar_get_handle": ([P, ctypes.c_char_p], c_int),
        "k8s_ar_open_handle": ([ctypes.c_char_p, ctypes.POINTER(P)], c_int),
        "k8s_ar_close_handle": ([P], c_int),
        "k8s_ar_handle_size": ([], c_int),
        "k8s_ar_register": ([c_int, c_int, ctypes.POINTER(P), c_long, ctypes.c_double], c_int),
        "k8s_ar_unregister": ([c_int], c_int),
        "k8s_ar_set_max_blocks": ([c_int, c_int], c_int),
        "k8s_ar_allreduce_bf16": ([c_int, P, P, c_long, c_int, P], c_int),
        "k8s_ar_alltoall_bf16": ([c_int, P, P, c_long, P], c_int),
        "k8s_ar_status": ([c_int, ctypes.POINTER(c_int)], c_int),
        "k8s_ar_status_async": ([c_int, P, P], c_int),
        "k8s_ar_addnorm_bf16": ([c_int, P, P, P, P, c_int, c_int, ctypes.c_float, c_int, P], c_int),
        "k8s_ar_push_ok": ([c_int, c_int, c_int, c_int], c_int),
        "k8s_ar_push_addnorm_bf16": ([c_int, P, P, P, c_int, c_int, ctypes.c_float, c_int, c_int, P], c_int),
        "k8s_gemm_stream_push": ([P, c_int, P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P], c_int),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    L._ar_bound = True


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (hip error {rc})")


class XgmiAllReduce:
    """In-place bf16 sum over a process group whose ranks share an xGMI mesh
    (one process per GPU, all in one node)."""

    def __init__(self, group=None, max_bytes: int = 8 << 20, timeout_s: float = 10.0,
                 max_blocks: Optional[int] = None):
        """``max_blocks`` caps every collective's grid (the same on every rank):
        needed only when ranks SHARE one GPU -- a full grid of blocks spinning
        for their peers can starve the peer process of the CUs its next kernel
        needs (csrc/kernels/allreduce.hip k8s_ar_set_max_blocks)."""
        L = lib()
        _bind(L)
        self.L = L
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("xGMI all-reduce supports up to 8 ranks (one node)")
        self.max_bytes = int(max_bytes)
        self._own = ctypes.c_void_p()
        _check(L.k8s_ar_alloc(L.k8s_ar_buffer_bytes(self.max_bytes), ctypes.byref(self._own)), "k8s_ar_alloc")
        hs = L.k8s_ar_handle_size()
        h = ctypes.create_string_buffer(hs)
        _check(L.k8s_ar_get_handle(self._own, h), "hipIpcGetMemHandle")
        handles: List[Optional[bytes]] = [None] * self.world
        dist.all_gather_object(handles, h.raw, group=group)
        self._bases = (ctypes.c_void_p * self.world)()
        self._opened = []
        for r in range(self.world):
            if r == self.rank:
                self._bases[r] = self._own.value
                continue
            q = ctypes.c_void_p()
            _check(L.k8s_ar_open_handle(handles[r], ctypes.byref(q)), "hipIpcOpenMemHandle")
            self._opened.append(q)
            self._bases[r] = q.value
        self.id = L.k8s_ar_register(self.world, self.rank, self._bases, self.max_bytes, float(timeout_s))
        if self.id < 0:
            raise RuntimeError("k8s_ar_register failed")
        if max_blocks is not None:
            _check(L.k8s_ar_set_max_blocks(self.id, int(max_blocks)), "k8s_ar_set_max_blocks")
        torch.cuda.synchronize()
        dist.barrier(group=group)

    def mode_for(self, t: torch.Tensor) -> int:
        """1 one-shot, 2 two-shot, 0 = not applicable in one call (RCCL, or
        :meth:`__call__`'s chunked form when :meth:`eligible`)."""
        nb = t.numel() * t.element_size()
        if not self.eligible(t) or nb > self.max_bytes:
            return 0
        return 1 if nb <= ONE_SHOT_MAX else 2

    @staticmethod
    def eligible(t: torch.Tensor) -> bool:
        """Any size: a larger tensor is reduced in buffer-sized chunks."""
        return t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0

    def chunk_elems(self) -> int:
        """Elements per chunk of a larger-than-buffer all-reduce: the buffer's
        capacity, whole 8 x world-element units (the two-shot's slice unit)."""
        unit = 8 * self.world
        return (self.max_bytes // 2) // unit * unit

    def __call__(self, t: torch.Tensor, mode: Optional[int] = None) -> torch.Tensor:
        """In-place sum over the group.  Tensors larger than the buffer (the
        prefill-size TP all-reduces: 70B at 8,192 tokens is 128 MiB) run as
        consecutive two-shot calls over buffer-sized chunks on the same stream
        -- each chunk reads the N-1 peers over N-1 links at once, so the whole
        TP data path stays on the xGMI kernels (no RCCL call)."""
        nb = t.numel() * t.element_size()
        if nb > self.max_bytes and mode is None and self.eligible(t):
            flat = t.view(-1)
            step = self.chunk_elems()
            for a in range(0, flat.numel(), step):
                c = flat[a:a + step]
                _check(self.L.k8s_ar_allreduce_bf16(self.id, c.data_ptr(), c.data_ptr(), c.numel(),
                                                    1 if c.numel() * 2 <= ONE_SHOT_MAX else 2, stream_ptr(t)),
                       "k8s_ar_allreduce_bf16")
            return t
        m = self.mode_for(t) if mode is None else mode
        if m == 0:
            raise ValueError("tensor not eligible for the xGMI all-reduce")
        _check(self.L.k8s_ar_allreduce_bf16(self.id, t.data_ptr(), t.data_ptr(), t.numel(), m, stream_ptr(t)),
               "k8s_ar_allreduce_bf16")
        return t

    def addnorm(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, y: torch.Tensor, eps: float,
                mode: Optional[int] = None) -> torch.Tensor:
        """The TP row-parallel epilogue in one launch: ``residual += all_reduce(x)``
        (bf16-rounded sum, then the add rounded to bf16), ``y = rmsnorm(residual) * w``.
        One-shot is bit-identical to ``self(x)`` + the rmsnorm kernel; two-shot
        computes the row's sum of squares from per-rank slice sums (the same
        value on every rank)."""
        T, H = x.shape
        m = mode or (1 if T * H * 2 <= ONE_SHOT_MAX else 2)
        _check(self.L.k8s_ar_addnorm_bf16(self.id, x.data_ptr(), residual.data_ptr(), w.data_ptr(), y.data_ptr(), T,
                                          H, float(eps), m, stream_ptr(x)), "k8s_ar_addnorm_bf16")
        return y

    def push_ok(self, H: int, T: int, mode: int) -> bool:
        """A [T, H] row-parallel output can take the push epilogue in ``mode``."""
        return push_ok(self, H, T, mode)

    def linear_push_addnorm(self, x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, nw: torch.Tensor,
                            y: torch.Tensor, eps: float, cfg: int, splits: int = 1,
                            mode: Optional[int] = None) -> torch.Tensor:
        """``residual += all_reduce(x @ w.T)``, ``y = rmsnorm(residual) * nw`` with
        the push epilogue: see :func:`linear_push_addnorm`."""
        return linear_push_addnorm(self, x, w, residual, nw, y, eps, cfg, splits, mode)

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        """Equal-split all-to-all: ``send`` [world, chunk...] bf16 -> ``recv`` (same
        shape), ``recv[r]`` = rank r's ``send[this rank]``.  Device-side epoch:
        no host sync, HIP-graph capturable (EP dispatch / combine, parallel/ep.py)."""
        assert send.dtype == torch.bfloat16 and send.is_contiguous() and recv.is_contiguous()
        assert send.shape[0] == self.world and send.shape == recv.shape
        chunk = send.numel() // self.world
        _check(self.L.k8s_ar_alltoall_bf16(self.id, send.data_ptr(), recv.data_ptr(), chunk, stream_ptr(send)),
               "k8s_ar_alltoall_bf16")
        return recv

    def all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """[world, *x.shape] = every rank's ``x`` (any dtype: the bytes are
        moved as bf16 pairs through :meth:`all_to_all` with the row replicated
        for every destination).  Device-side, no host sync: the TP sampler's
        winners / candidates travel this way (``VocabParallelSampler._sample_shard``).
        Larger than the buffer: consecutive buffer-sized pieces."""
        flat = x.contiguous().view(-1).view(torch.uint8)
        nb = flat.numel()
        pad = (-nb) % (16 * self.world)
        if pad:
            flat = torch.cat([flat, flat.new_zeros(pad)])
        row = flat.view(torch.bfloat16)
        n = row.numel()
        # bf16 elements per piece: the a2a moves world x piece, within 2 x max_bytes
        step = max(8, (self.max_bytes // self.world) // 8 * 8)
        out = torch.empty(self.world, n, dtype=torch.bfloat16, device=x.device)
        for a in range(0, n, step):
            piece = row[a:a + step]
            send = piece.unsqueeze(0).expand(self.world, -1).contiguous()
            recv = torch.empty_like(send)
            self.all_to_all(send, recv)
            out[:, a:a + piece.numel()] = recv
        out = out.view(torch.uint8)[:, :nb].contiguous()
        return out.view(x.dtype).view(self.world, *x.shape)

    # ------------------------------------------------------------ fabric tuning
    plan: Optional[dict] = None  # {T bucket: (mode, push)} from :meth:`tune`; None = the size rule

    def tune(self, shapes, nw: torch.Tensor, eps: float, buckets, iters: int = 10, rounds: int = 3) -> dict:
        """Pick, per decode row-count bucket T, the collective form of the TP
        row-parallel epilogue (GEMM + all-reduce + residual add + RMSNorm) by
        timing every candidate ON THIS FABRIC at communicator init: one-shot
        vs two-shot, staged (the GEMM writes y, the fused epilogue stages it)
        vs push (the stream GEMM stores into the peers' slots,
        csrc/kernels/allreduce.hip "push epilogue").  ``shapes``: the real
        row-parallel weights [(name, w [H, K_local])] (o and down).  Every
        rank runs the same sequence of collectives, and each timing is
        max-reduced over the group, so every rank gets the same plan.  The
        round-4 defaults (one-shot <= 512 KiB, push off) came from a
        loopback on one GPU, which cannot show xGMI behaviour; this replaces
        them with what the deployment's own links measure."""
        from ..ops import linear as LIN
        H = int(shapes[0][1].shape[0])
        dev = shapes[0][1].device
        report = {}
        plan = {}
        for T in sorted(set(int(b) for b in buckets)):
            if T * H * 2 + 4 * T > self.max_bytes:
                continue
            cands = [(1, False)]
            if (H // 8) % self.world == 0:
                cands.append((2, False))
            for m in (1, 2):
                if (m, False) not in cands:
                    continue
                ok = True
                for _, w in shapes:
                    kind, cfg, splits = LIN.select_gemm(T, H, int(w.shape[1]))
                    ok &= kind == LIN.KIND_STREAM and (cfg >= 13 or splits > 1) and self.push_ok(H, T, m)
                if ok:
                    cands.append((m, True))
            x = {name: torch.randn(T, int(w.shape[1]), device=dev).bfloat16() for name, w in shapes}
            res = torch.zeros(T, H, device=dev, dtype=torch.bfloat16)
            y = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
            out = torch.empty(T, H, device=dev, dtype=torch.bfloat16)

            def pair(m, push):
                for name, w in shapes:
                    if push:
                        kind, cfg, splits = LIN.select_gemm(T, H, int(w.shape[1]))
                        self.linear_push_addnorm(x[name], w, res, nw, y, eps, cfg, splits, m)
                    else:
                        LIN.linear(x[name], w, out)
                        self.addnorm(out, res, nw, y, eps, m)
                    res.zero_()

            us = {c: [] for c in cands}
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(rounds):
                for c in cands:
                    pair(*c)  # warm (also aligns the ranks on this candidate)
                    e0.record()
                    for _ in range(iters):
                        pair(*c)
                    e1.record()
                    e1.synchronize()
                    us[c].append(e0.elapsed_time(e1) * 1e3 / iters)
            med = torch.tensor([sorted(v)[len(v) // 2] for v in us.values()], dtype=torch.float64)
            on_dev = dist.get_backend(self.group) == "nccl"
            t = med.to(dev) if on_dev else med
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)  # the slowest rank's view
            med = t.cpu().tolist()
            best = min(range(len(cands)), key=lambda i: med[i])
            plan[T] = cands[best]
            report[T] = {f"{'two' if m == 2 else 'one'}_shot{'_push' if p else ''}": round(v, 2)
                         for (m, p), v in zip(cands, med)}
            report[T]["pick"] = list(cands[best])
        torch.cuda.synchronize()
        self.plan = plan
        self.tune_report = report
        return report

    def plan_for(self, T: int, H: int):
        """(mode, push) of a [T, H] row-parallel epilogue: the tuned bucket at or
        above T, else the size rule (one-shot <= 512 KiB, no push)."""
        if self.plan:
            for b in sorted(self.plan):
                if b >= T:
                    return self.plan[b]
        return (1 if T * H * 2 <= ONE_SHOT_MAX else 2), False

    def status_async(self, host: torch.Tensor) -> None:
        """Copy this rank's STATUS word into ``host`` (pinned int32[1]) on the
        current stream, ordered after the collectives issued before it."""
        _check(self.L.k8s_ar_status_async(self.id, host.data_ptr(), stream_ptr()), "k8s_ar_status_async")

    def a2a_fits(self, nbytes: int) -> bool:
        return nbytes <= 2 * self.max_bytes and (nbytes // 2) % (8 * self.world) == 0

    def status(self) -> int:
        v = ctypes.c_int(0)
        _check(self.L.k8s_ar_status(self.id, ctypes.byref(v)), "k8s_ar_status")
        return v.value

    def close(self) -> None:
        if self.id < 0:
            return
        torch.cuda.synchronize()
        self.L.k8s_ar_unregister(self.id)
        for q in self._opened:
            self.L.k8s_ar_close_handle(q)
        self.L.k8s_ar_free(self._own)
        self.id = -1


def push_ok(car, H: int, T: int, mode: int) -> bool:
    return bool(car.L.k8s_ar_push_ok(car.id, int(H), int(T), int(mode)))


def linear_push_addnorm(car, x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, nw: torch.Tensor,
                        y: torch.Tensor, eps: float, cfg: int, splits: int = 1, mode: Optional[int] = None):
    """The TP row-parallel projection + all-reduce + residual add + RMSNorm with
    the push epilogue (csrc/kernels/allreduce.hip "push epilogue"): the stream
    GEMM (``cfg``: LDS-DMA 13-16 / 23 / 24, or any cfg with ``splits`` > 1)
    stores ``x @ w.T`` straight into the communicator's slots -- the whole tile
    to every rank (one-shot) or each strip to the owner of its columns
    (two-shot) -- with one flag per strip, and the fused epilogue sums the
    local slots.  Bit-identical to ``linear`` + :meth:`XgmiAllReduce.addnorm`."""
    from ..ops import linear as LIN
    T, K = x.shape
    H = w.shape[0]
    m = mode or (1 if T * H * 2 <= ONE_SHOT_MAX else 2)
    if not car.push_ok(H, T, m):
        raise ValueError("output not eligible for the push epilogue")
    part = LIN._scratch(x.device, splits * T * H).data_ptr() if splits > 1 else None
    L = car.L
    _check(L.k8s_gemm_stream_push(x.data_ptr(), x.stride(0), w.data_ptr(), T, H, K, int(cfg), int(splits), part,
                                  car.id, m, stream_ptr(x)), "k8s_gemm_stream_push")
    S = H // (128 if (splits == 1 and cfg > 20) else 64)  # common.h k8s_push_strips
    _check(L.k8s_ar_push_addnorm_bf16(car.id, residual.data_ptr(), nw.data_ptr(), y.data_ptr(), T, H, float(eps), m,
                                      S, stream_ptr(x)), "k8s_ar_push_addnorm_bf16")
    return y
