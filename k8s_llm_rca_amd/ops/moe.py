"""MoE routing ops (B11/B12): top-k router, expert permutation, weighted combine."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._lib import check, lib, ptr, scratch, stream_ptr, use_hip


def route_topk(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """softmax -> top-k -> renormalise.  Returns (weights fp32 [T,k], ids int32 [T,k])."""
    T, E = logits.shape
    if use_hip(logits):
        assert logits.dtype == torch.bfloat16 and logits.is_contiguous()
        w = torch.empty(T, k, dtype=torch.float32, device=logits.device)
        ids = torch.empty(T, k, dtype=torch.int32, device=logits.device)
        check(lib().k8s_moe_route(ptr(logits), T, E, k, ptr(w), ptr(ids), stream_ptr(logits)), "moe_route")
        return w, ids
    p = torch.softmax(logits.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    return w / w.sum(-1, keepdim=True), ids.int()


def align(ids: torch.Tensor, E: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Sort the T*k (token, slot) pairs by expert.  Returns (order, inv, offsets[E+1]) int32."""
    flat = ids.reshape(-1).contiguous()
    n = flat.numel()
    if use_hip(flat):
        order = torch.empty(n, dtype=torch.int32, device=flat.device)
        inv = torch.empty(n, dtype=torch.int32, device=flat.device)
        offsets = torch.empty(E + 1, dtype=torch.int32, device=flat.device)
        check(lib().k8s_moe_align(ptr(flat), n, E, 0, ptr(order), ptr(inv), ptr(offsets), stream_ptr(flat)),
              "moe_align")
        return order, inv, offsets
    order = torch.argsort(flat.long(), stable=True).int()
    inv = torch.empty_like(order)
    inv[order.long()] = torch.arange(n, dtype=torch.int32)
    counts = torch.bincount(flat.long(), minlength=E)
    offsets = torch.zeros(E + 1, dtype=torch.int32)
    offsets[1:] = torch.cumsum(counts, 0).int()
    return order, inv, offsets


def combine(y_perm: torch.Tensor, inv: torch.Tensor, w: torch.Tensor, T: int, k: int) -> torch.Tensor:
    """out[t] = sum_j w[t,j] * y_perm[inv[t*k+j]]."""
    H = y_perm.shape[1]
    out = torch.empty(T, H, dtype=y_perm.dtype, device=y_perm.device)
    if use_hip(y_perm):
        assert y_perm.is_contiguous() and w.dtype == torch.float32
        check(lib().k8s_moe_combine(ptr(y_perm), ptr(inv), ptr(w), T, k, H, ptr(out), stream_ptr(y_perm)),
              "moe_combine")
        return out
    g = y_perm.float()[inv.long()].view(T, k, H)
    out.copy_((g * w.view(T, k, 1)).sum(1).to(out.dtype))
    return out


def grouped_gemm(a: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, fuse_silu: bool = False,
                 out: Optional[torch.Tensor] = None, splits: int = 1, glds: int = 0) -> torch.Tensor:
    """B13: rows offsets[e]..offsets[e+1] of ``a`` times ``w[e]^T`` for every
    expert in one launch (``w`` [E, N, K]).  ``fuse_silu``: ``a`` is the
    gate_up output [rows, 2K] and the activation silu(gate) * up is formed on
    the fly.  ``splits`` > 1 splits K over workgroups (fp32 partials + a
    reduce; see grouped_gemm.hip).  ``glds`` = 10 + NB runs the LDS-DMA strip
    kernel with NB stages instead (64-row tiles: decode batches).  Offsets stay
    on the device (no host sync)."""
    E, N, K = w.shape
    rows = a.shape[0]
    if out is None:
        out = torch.empty(rows, N, dtype=a.dtype, device=a.device)
    if rows == 0:
        return out
    if glds and use_hip(a) and not fuse_silu and N % 64 == 0 and K % (64 * splits) == 0:
        # the LDS-DMA strip kernel (csrc/kernels/gemm_stream.hip grouped_glds_kernel)
        assert a.dtype == torch.bfloat16 and w.is_contiguous() and a.stride(1) == 1 and out.is_contiguous()
        max_tiles = (rows + 63) // 64 + E
        part = _split_scratch(a.device, splits * rows * N) if splits > 1 else None
        check(lib().k8s_grouped_glds(ptr(a), a.stride(0), ptr(w), ptr(out), out.stride(0), ptr(offsets), E, N, K,
                                     max_tiles, glds, splits, ptr(part), rows, stream_ptr(a)), "grouped_glds")
        return out
    if use_hip(a) and N % 128 == 0 and K % (64 * splits) == 0:
        assert a.dtype == torch.bfloat16 and w.is_contiguous() and a.stride(1) == 1 and out.is_contiguous()
        assert a.shape[1] == (2 * K if fuse_silu else K)
        max_tiles = (rows + 63) // 64 + E
        part = _split_scratch(a.device, splits * rows * N) if splits > 1 else None
        check(lib().k8s_grouped_gemm(ptr(a), a.stride(0), ptr(w), ptr(out), out.stride(0), ptr(offsets), E, N, K,
                                     max_tiles, int(fuse_silu), splits, ptr(part), rows, stream_ptr(a)),
              "grouped_gemm")
        return out
    offs = offsets.tolist()
    for e in range(E):
        lo, hi = offs[e], offs[e + 1]
        if hi <= lo:
            continue
        x = a[lo:hi].float()
        if fuse_silu:
            x = torch.nn.functional.silu(x[:, :K]) * x[:, K:]
        out[lo:hi] = (x @ w[e].float().t()).to(out.dtype)
    return out


def grouped_big_ok(rows: int, N: int, K: int, silu: bool) -> bool:
    """What the grouped form of csrc/kernels/gemm_big.hip accepts."""
    return rows > 0 and K % 128 == 0 and N % (128 if silu else 256) == 0


def grouped_big(x: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, silu: bool = False,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """B13 at prefill sizes on the 8-phase MFMA GEMM (csrc/kernels/gemm_big.hip,
    grouped form): rows offsets[e]..offsets[e+1] of ``x`` times ``w[e]^T`` in one
    launch with the offsets read on the device (no host sync, capturable).
    ``silu``: ``w`` [E, 2I, K] is the gate_up weight (gate rows first) and the
    result is the SwiGLU activation [rows, I] -- gate_up is never written."""
    from .linear import BIG_PIPE
    E, Nw, K = w.shape
    N = Nw // 2 if silu else Nw
    rows = x.shape[0]
    if out is None:
        out = torch.empty(rows, N, dtype=x.dtype, device=x.device)
    if rows == 0:
        return out
    assert x.dtype == torch.bfloat16 and w.is_contiguous() and x.stride(1) == 1 and x.shape[1] == K
    assert offsets.dtype == torch.int32 and offsets.is_cuda and grouped_big_ok(rows, N, K, silu)
    check(lib().k8s_gemm_big_grouped(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), ptr(offsets), E, rows, N,
                                     K, int(silu), BIG_PIPE, stream_ptr(x)), "gemm_big_grouped")
    return out


_scratch = {}


def _split_scratch(dev: torch.device, n: int) -> torch.Tensor:
    t = _scratch.get(dev)
    if t is None or t.numel() < n:
        if t is not None:  # never freed: graphs captured earlier replay at its address (ops/linear.py _scratch)
            from . import linear as LIN
            LIN._retired_scratch.append(t)
        t = scratch(max(n, 1 << 20), torch.float32, dev)
        _scratch[dev] = t
    return t


def reserve_split_scratch(dev: torch.device, max_rows: int, N: int, splits: int) -> None:
    """Allocate the split-K partial buffer before any HIP-graph capture."""
    _split_scratch(dev, max_rows * N * splits)
