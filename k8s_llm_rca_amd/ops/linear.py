"""Projection GEMMs: hand-written skinny MFMA GEMM for decode shapes, hipBLASLt otherwise."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ._lib import check, lib, ptr, stream_ptr

SKINNY_MAX_M = int(os.environ.get("K8SRCA_SKINNY_MAX_M", "16"))
# measured on MI355X (tools/bench_kernels.py): the skinny kernel beats hipBLASLt
# ~2x on the small-N decode projections (o_proj / QKV) for M <= 16 and ties or
# loses on the wide ones; beyond M = 16 its L2-read X operand is the bottleneck.
SKINNY_MAX_NK = 8192 * 4096
_enabled = os.environ.get("K8SRCA_SKINNY", "1") == "1"


def set_skinny(enabled: bool) -> None:
    global _enabled
    _enabled = enabled


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """``x @ w.T`` for ``x`` [M, K] and ``w`` [N, K] (bf16)."""
    M, K = x.shape
    N = w.shape[0]
    if (_enabled and x.is_cuda and (M == 1 or (M <= SKINNY_MAX_M and N * K <= SKINNY_MAX_NK))
            and x.dtype == torch.bfloat16 and K % 256 == 0
            and N % 16 == 0 and x.stride(1) == 1 and w.is_contiguous()):
        if out is None:
            out = torch.empty((M, N), dtype=x.dtype, device=x.device)
        check(lib().k8s_gemm_skinny(ptr(x), x.stride(0), ptr(w), ptr(out), out.stride(0), M, N, K,
                                    stream_ptr(x)), "gemm_skinny")
        return out
    if out is None:
        return F.linear(x, w)
    return torch.matmul(x, w.t(), out=out)
