"""Fused residual-add + RMSNorm (B2) and SwiGLU (B8)."""
from __future__ import annotations

from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr, use_hip


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``y = rmsnorm(x + residual) * w``; when ``residual`` is given it is updated in place to ``x + residual``."""
    T, H = x.shape
    if out is None:
        out = torch.empty((T, H), dtype=x.dtype, device=x.device)
    if use_hip(x):
        assert x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and H % 8 == 0
        assert x.stride(1) == 1 and out.is_contiguous() and weight.is_contiguous() and H <= 16384
        if residual is not None:
            assert residual.is_contiguous() and residual.shape == (T, H)
        check(lib().k8s_rmsnorm(ptr(x), ptr(residual), ptr(weight), ptr(out), T, H, x.stride(0), out.stride(0),
                                float(eps), stream_ptr(x)), "rmsnorm")
        return out
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
        residual.copy_(xf.to(residual.dtype))
        xf = residual.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    out.copy_((xf * torch.rsqrt(var + eps) * weight.float()).to(out.dtype))
    return out


def splitk_addnorm(part: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor, eps: float,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``rmsnorm(bf16(part.sum(0)) + residual) * w`` with ``residual`` updated in
    place: the reduction of a split-K GEMM's fp32 partials ``part``
    ``[splits, T, H]`` fused into the residual add + RMSNorm that consumes it
    (the native layer executor's epilogue for split-K o / down projections)."""
    S, T, H = part.shape
    if out is None:
        out = torch.empty((T, H), dtype=residual.dtype, device=residual.device)
    if use_hip(residual):
        assert part.dtype == torch.float32 and part.is_contiguous() and residual.is_contiguous()
        assert residual.shape == (T, H) and out.is_contiguous() and weight.dtype == torch.bfloat16
        check(lib().k8s_splitk_addnorm(ptr(part), S, ptr(residual), ptr(weight), ptr(out), T, H, out.stride(0),
                                       float(eps), stream_ptr(residual)), "splitk_addnorm")
        return out
    acc = part[0].clone()
    for s in range(1, S):
        acc += part[s]
    return rmsnorm(acc.to(residual.dtype), weight, eps, residual=residual, out=out)


def silu_mul(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    T, I2 = gu.shape
    inter = I2 // 2
    if out is None:
        out = torch.empty((T, inter), dtype=gu.dtype, device=gu.device)
    if use_hip(gu):
        assert gu.is_contiguous() and out.is_contiguous() and inter % 8 == 0 and gu.dtype == torch.bfloat16
        check(lib().k8s_silu_mul(ptr(gu), ptr(out), T, inter, stream_ptr(gu)), "silu_mul")
        return out
    g, u = gu.float().split(inter, dim=-1)
    out.copy_((torch.nn.functional.silu(g) * u).to(out.dtype))
    return out


def nonfinite_flag(x: torch.Tensor, flag: torch.Tensor) -> None:
    """Debug: ``flag[0] = 1`` (int32, device) when ``x`` holds a NaN / inf;
    never clears it.  CPU tensors: the same test in PyTorch."""
    if use_hip(x):
        xc = x.contiguous()
        check(lib().k8s_nonfinite_flag(ptr(xc), xc.numel(), ptr(flag), stream_ptr(x)), "nonfinite_flag")
        return
    if not torch.isfinite(x).all():
        flag[0] = 1
