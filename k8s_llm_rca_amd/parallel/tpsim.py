"""Per-rank projection of a TP / EP deployment on ONE GPU (``bench --tp-sim N``).

The 8-GPU configs of BASELINE.json (Llama-3-70B TP=8, Mixtral EP=8) cannot be
run on a one-GPU box, but what one rank of them computes can: this context
builds **rank 0's shard at the real shapes** (70B: 8 q / 1 kv heads,
intermediate 3,584, vocab shard 16,032 per rank) and runs the real engine on
it -- HIP-graph decode steps, the native layer executor, the sampler -- with
every collective replaced by a **local stand-in that moves the same bytes**:

* the xGMI one-shot / two-shot all-reduce and the all-to-all run the REAL
  kernels (``csrc/kernels/allreduce.hip``) on a loopback communicator whose
  ``world`` buffers all live on this GPU (``k8s_ar_register_loopback``): the
  same staging, flag stores and peer-slot reads, over local HBM instead of
  xGMI, waits skipped;
* messages above the xGMI buffer (prefill chunks, RCCL's ring on a real
  node) are stood in for by a local copy of the ring's per-rank traffic,
  2 (N - 1) / N of the message;
* the vocab-parallel logits all-gather tiles this rank's shard N times (the
  same [rows, vocab] bytes), so the sampler sees a full-vocabulary row.

Outputs are NOT the TP model's (peer partial sums are zeros): this is a
timing model of one rank, labelled as such in every result line.  The
projection adds modelled xGMI time for each collective
(:func:`xgmi_model_us`) in place of the stand-in's measured time.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from ..ops._lib import lib, stream_ptr
from .groups import ParallelContext
from .xgmi import ONE_SHOT_MAX, _bind, _check, linear_push_addnorm, push_ok

XGMI_LINK_GBPS = 153.0   # one xGMI link, per direction (7 links per GPU)
XGMI_HOP_US = 2.5        # one flag hand-off across the fabric (signal -> visible on the peer)
HOP_SENSITIVITY_US = (2.5, 5.0, 10.0)  # the projection is also reported at these hop latencies
RCCL_BUS_GBPS = 300.0    # assumed RCCL all-reduce bus bandwidth on an 8-GPU xGMI node (not measured here)


def xgmi_model_us(nbytes: int, world: int, mode: int, hop_us: float = XGMI_HOP_US) -> float:
    """Modelled time of one bf16 all-reduce of ``nbytes`` over a full xGMI
    mesh: one-shot reads (N-1) peer slices in parallel over N-1 links (one
    hop), two-shot moves 2 (N-1)/N of the message in two hops, and RCCL
    (mode 0, messages past the xGMI buffer) 2 (N-1)/N of it at
    ``RCCL_BUS_GBPS`` with 2 (N-1) ring hops."""
    bw = XGMI_LINK_GBPS * 1e3  # bytes per us
    if mode == 1:
        return hop_us + nbytes / bw
    if mode == 2:
        return 2 * hop_us + 2 * nbytes / (world * bw)
    return 2 * (world - 1) * hop_us + 2 * (world - 1) / world * nbytes / (RCCL_BUS_GBPS * 1e3)


class LoopbackAR:
    """The xGMI communicator interface (``parallel.xgmi.XgmiAllReduce``) over a
    loopback registration: same kernels, same bytes, no peers."""

    def __init__(self, world: int, max_bytes: int = 8 << 20):
        L = lib()
        _bind(L)
        if not getattr(L, "_loop_bound", False):
            L.k8s_ar_register_loopback.argtypes = [ctypes.c_int, ctypes.c_long]
            L.k8s_ar_register_loopback.restype = ctypes.c_int
            L._loop_bound = True
        self.L = L
        self.world = world
        self.rank = 0
        self.max_bytes = int(max_bytes)
        self.id = L.k8s_ar_register_loopback(world, self.max_bytes)
        if self.id < 0:
            raise RuntimeError("k8s_ar_register_loopback failed")

    def mode_for(self, t: torch.Tensor) -> int:
        nb = t.numel() * t.element_size()
        if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.numel() % 8 or nb > self.max_bytes:
            return 0
        return 1 if nb <= ONE_SHOT_MAX else 2

    def __call__(self, t: torch.Tensor, mode: Optional[int] = None) -> torch.Tensor:
        m = self.mode_for(t) if mode is None else mode
        if m == 0:
            raise ValueError("tensor not eligible for the xGMI all-reduce")
        _check(self.L.k8s_ar_allreduce_bf16(self.id, t.data_ptr(), t.data_ptr(), t.numel(), m, stream_ptr(t)),
               "k8s_ar_allreduce_bf16 (loopback)")
        return t

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        chunk = send.numel() // self.world
        _check(self.L.k8s_ar_alltoall_bf16(self.id, send.data_ptr(), recv.data_ptr(), chunk, stream_ptr(send)),
               "k8s_ar_alltoall_bf16 (loopback)")
        return recv

    def all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """The a2a stand-in moves the bytes; the result is this rank's ``x``
        replicated (the "peers" never wrote theirs)."""
        flat = x.contiguous().view(-1).view(torch.uint8)
        nb = flat.numel()
        pad = (-nb) % 16
        if pad:
            flat = torch.cat([flat, flat.new_zeros(pad)])
        send = flat.view(torch.bfloat16).unsqueeze(0).expand(self.world, -1).contiguous()
        self.all_to_all(send, torch.empty_like(send))
        return x.unsqueeze(0).expand(self.world, *x.shape).contiguous()

    def a2a_fits(self, nbytes: int) -> bool:
        return nbytes <= 2 * self.max_bytes and (nbytes // 2) % (8 * self.world) == 0

    def push_ok(self, H: int, T: int, mode: int) -> bool:
        return push_ok(self, H, T, mode)

    def addnorm(self, x, residual, w, y, eps, mode=None):
        T, H = x.shape
        m = mode or (1 if T * H * 2 <= ONE_SHOT_MAX else 2)
        _check(self.L.k8s_ar_addnorm_bf16(self.id, x.data_ptr(), residual.data_ptr(), w.data_ptr(), y.data_ptr(), T,
                                          H, float(eps), m, stream_ptr(x)), "k8s_ar_addnorm_bf16 (loopback)")
        return y

    def linear_push_addnorm(self, x, w, residual, nw, y, eps, cfg, splits=1, mode=None):
        """The push epilogue's stand-in: the GEMM stores into the loopback slots
        (the bytes of the real push), the consumer's waits are skipped."""
        return linear_push_addnorm(self, x, w, residual, nw, y, eps, cfg, splits, mode)

    def status_async(self, host: torch.Tensor) -> None:
        _check(self.L.k8s_ar_status_async(self.id, host.data_ptr(), stream_ptr()), "k8s_ar_status_async")

    def status(self) -> int:
        v = ctypes.c_int(0)
        _check(self.L.k8s_ar_status(self.id, ctypes.byref(v)), "k8s_ar_status")
        return v.value

    def close(self) -> None:
        if self.id >= 0:
            torch.cuda.synchronize()
            self.L.k8s_ar_unregister(self.id)
            self.id = -1


@dataclass
class SimParallelContext(ParallelContext):
    """Rank 0 of a ``tp_size``-way TP group, simulated on one GPU (see module
    docstring).  ``sim`` tells the engine not to open a step channel to
    workers that do not exist."""
    sim: bool = True

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        car = self.custom_ar
        if car is not None and car.mode_for(t):
            return car(t)
        # RCCL ring stand-in: this rank's 2 (N-1)/N share of the message, over local HBM
        n = t.numel()
        k = max(8, int(2 * (self.tp_size - 1) / self.tp_size * n))
        buf = _scratch(t.device, k, t.dtype)
        src = t.view(-1)
        done = 0
        while done < k:
            m = min(n, k - done)
            buf[done:done + m].copy_(src[:m])
            done += m
        return t

    def linear_all_reduce(self, x: torch.Tensor, w: torch.Tensor, linear_fn=None) -> torch.Tensor:
        import torch.nn.functional as F
        lin = linear_fn or F.linear
        return self.all_reduce(lin(x, w))

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        """[n, v_local] -> [n, v_local * N]: the shard tiled N times (the bytes
        an all-gather delivers; every rank then samples the full row)."""
        return t.repeat(1, self.tp_size)


_SCRATCH: dict = {}


def _scratch(device, n: int, dtype) -> torch.Tensor:
    key = (str(device), dtype)
    b = _SCRATCH.get(key)
    if b is None or b.numel() < n:
        b = torch.empty(max(n, 1 << 20), dtype=dtype, device=device)
        _SCRATCH[key] = b
    return b


def sim_context(tp: int, max_bytes: int = 64 << 20, ep: int = 1) -> SimParallelContext:
    """``ep`` = tp for a MoE model: experts sharded over the same ranks (EP=8:
    one Mixtral expert per rank), attention tensor-parallel."""
    pc = SimParallelContext(tp_size=tp, tp_rank=0, ep_size=ep, ep_rank=0)
    pc.custom_ar = LoopbackAR(tp, max_bytes)
    return pc


def a2a_model_us(nbytes: int, world: int, hop_us: float = XGMI_HOP_US) -> float:
    """Modelled equal-split all-to-all of ``nbytes`` per rank over a full
    xGMI mesh: (N-1)/N of them leave over N-1 links at once, one hop."""
    return hop_us + nbytes / (world * XGMI_LINK_GBPS * 1e3)


def _time_us(fn, reps: int = 20) -> float:
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    ev1.synchronize()
    return ev0.elapsed_time(ev1) * 1e3 / reps


def _fused_epilogue(car, T: int, H: int, mode: int) -> bool:
    """The layer executor's fused all-reduce + add + RMSNorm applies (ops/layer_exec.py fits / ar_fuse)."""
    return (car is not None and mode in (1, 2) and hasattr(car, "addnorm")
            and T * H * 2 + 4 * T <= car.max_bytes and (mode == 1 or (H // 8) % car.world == 0))


def _fused_standin_us(car, T: int, H: int, mode: int, device) -> float:
    from ..ops import norm as NORM
    x = torch.zeros(T, H, dtype=torch.bfloat16, device=device)
    res = torch.zeros_like(x)
    y = torch.empty_like(x)
    w = torch.ones(H, dtype=torch.bfloat16, device=device)
    fused = _time_us(lambda: car.addnorm(x, res, w, y, 1e-5, mode))
    plain = _time_us(lambda: NORM.rmsnorm(x, w, 1e-5, residual=res, out=y))
    return max(0.0, fused - plain)


def project(rows_hist: dict, pc: SimParallelContext, hidden: int, n_layers: int, device, moe_k: int = 0) -> dict:
    """Collective time of a simulated run: for every forward size T seen
    (``rows_hist`` = {T: forwards}) the layer's collectives, timed as stood in
    on this GPU and as modelled over xGMI (:func:`xgmi_model_us`,
    :func:`a2a_model_us`).  Dense: two [T, hidden] bf16 all-reduces per layer.
    MoE (``moe_k`` = top-k, EP = TP): one all-reduce (o_proj) and the three
    fixed-capacity all-to-alls of ``parallel/ep.py`` (dispatch, combine, row
    all-gather).  ``projected`` wall = measured wall - stand-in + modelled (the
    collectives are serial in the step's stream).  ``modelled_s_by_hop``: the
    same model at each hop latency of ``HOP_SENSITIVITY_US``.  Dense steps whose
    all-reduces the layer executor fuses with the residual add + RMSNorm time
    that fused kernel less the rmsnorm it replaces (``per_T[T]["standin"]``);
    the others time the plain all-reduce."""
    standin_us = model_us = 0.0
    by_hop = {h: 0.0 for h in HOP_SENSITIVITY_US}
    per_t = {}
    N = pc.tp_size
    for T, n in sorted(rows_hist.items()):
        t = torch.zeros(T * hidden, dtype=torch.bfloat16, device=device)
        car = pc.custom_ar
        mode = car.mode_for(t) if car is not None else 0
        if not moe_k and _fused_epilogue(car, T, hidden, mode):
            # the dense executor's collective: the fused all-reduce + add + RMSNorm, less
            # the rmsnorm launch it replaces (ops/layer_exec.py ar_fuse)
            s_us = _fused_standin_us(car, T, hidden, mode, device)
            kind = "fused"
        else:
            s_us = _time_us(lambda: pc.all_reduce(t))
            kind = "allreduce"

        m_us = xgmi_model_us(T * hidden * 2, N, mode)
        n_ar = 1 if moe_k else 2
        s_tot, m_tot = n_ar * s_us, n_ar * m_us
        h_tot = {h: n_ar * xgmi_model_us(T * hidden * 2, N, mode, h) for h in by_hop}
        if moe_k:
            per = (T + N - 1) // N
            for row_elems in ((per * moe_k) * (hidden + 8), (per * moe_k) * hidden, per * hidden):
                nb = N * row_elems * 2
                if car is not None and car.a2a_fits(nb):
                    send = torch.zeros(N, row_elems, dtype=torch.bfloat16, device=device)
                    recv = torch.empty_like(send)
                    s_tot += _time_us(lambda: car.all_to_all(send, recv))
                m_tot += a2a_model_us(nb, N)
                for h in by_hop:
                    h_tot[h] += a2a_model_us(nb, N, h)
        k = n_layers * n
        for h in by_hop:
            by_hop[h] += k * h_tot[h]
        standin_us += k * s_tot
        model_us += k * m_tot
        per_t[int(T)] = {"forwards": int(n), "mode": mode, "standin": kind, "standin_us": round(s_tot, 2),
                         "model_us": round(m_tot, 2)}
    return {"standin_s": standin_us / 1e6, "modelled_s": model_us / 1e6, "per_T": per_t,
            "modelled_s_by_hop": {h: v / 1e6 for h, v in by_hop.items()}}
