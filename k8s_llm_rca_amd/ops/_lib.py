"""Loader for ``libk8srca_hip.so`` (all hand-written gfx950 kernels, C ABI).

The library is loaded with ctypes *after* ``import torch`` so it binds to the
HIP runtime torch already mapped (same SONAME ``libamdhip64.so.7``) and shares
torch's device context and streams.  On a GPU box a missing or broken library
is a hard error (ops never silently fall back to eager PyTorch on device
tensors); CPU tensors use the fp32 PyTorch references in the op modules.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import _build
from ..knobs import KNOBS, push_native

_lib = None
_lock = threading.Lock()
_err = None

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float

_SIGS = {
    "k8s_rmsnorm": [P, P, P, P, I, I, I, I, F, P],
    "k8s_silu_mul": [P, P, I, I, P],
    "k8s_unpack_step": [P, I, I, I, P, P, P, P, P, P, P, P, P, I, P],
    "k8s_rope_kv": [P, I, P, P, P, P, P, I, I, I, I, P],
    "k8s_splitk_rope_kv": [P, I, P, I, P, P, P, P, P, I, I, I, I, P],
    "k8s_attn_decode": [P, I, P, P, P, I, P, P, I, I, I, I, F, P, I, P, P, I, I, P, I, P, I, P],
    "k8s_attn_prefill": [P, I, P, P, P, I, P, P, P, P, P, P, P, P, I, P, P, P, P, I, P, P, I, I, I, F, P, I, P],
    "k8s_sample": [P, I, I, I, I, P, P, P, P, P, I, P, P, P, P, P, P, I, P, P, P, I],
    "k8s_gemm_skinny": [P, I, P, P, I, I, I, I, P],
    "k8s_gemm_skinny_rope": [P, I, P, P, I, I, I, I, P, P, P, P, P, I, I, I, P],
    "k8s_gemm_mid": [P, I, P, P, I, I, I, I, I, I, P, P],
    "k8s_gemm_mid_part": [P, I, P, P, I, I, I, I, I, I, P, P],
    "k8s_gemm_stream": [P, I, P, P, I, I, I, I, I, I, P, P],
    "k8s_gemm_big": [P, I, P, P, I, I, I, I, I, I, P],
    "k8s_gemm_big_split": [P, I, P, P, I, I, I, I, I, I, P, P],
    "k8s_gemm_big_part": [P, I, P, P, I, I, I, I, I, I, P, P],
    "k8s_gemm_big_grouped": [P, I, P, P, I, P, I, I, I, I, I, I, P],
    "k8s_gemm_big_rope": [P, I, P, P, I, I, I, I, P, P, P, P, P, I, I, I, I, P],
    "k8s_gemm_big_ws_bytes": [],
    "k8s_gemm_big_set_ws": [P],
    "k8s_gemm_big_claim_ws": [P],
    "k8s_gemm_big_tail_foreign": [],
    "k8s_gemm_stream_silu": [P, I, P, P, I, I, I, I, I, P],
    "k8s_gemm_stream_silu_norm": [P, I, P, I, P, P, P, F, P, P, I, I, I, I, I, P],
    "k8s_gemm_skinny_rope_norm": [P, I, P, I, P, P, P, F, P, P, I, I, I, I, P, P, P, P, P, I, I, I, P],
    "k8s_gemm_stream_part": [P, I, P, P, I, I, I, I, I, I, P, P],
    "k8s_grouped_glds": [P, I, P, P, I, P, I, I, I, I, I, I, P, I, P],
    "k8s_splitk_addnorm": [P, I, P, P, P, I, I, I, F, P],
    "k8s_gemm_mid_num_cfgs": [],
    "k8s_blaslt_gemm": [P, I, P, P, I, I, I, I, P, ctypes.c_size_t, P],
    "k8s_blaslt_gemm2": [P, I, P, P, I, I, I, I, P, ctypes.c_size_t, P, I],
    "k8s_blaslt_num_plans": [],
    "k8s_blaslt_tune": [P, I, P, P, I, I, I, I, P, ctypes.c_size_t, I, I, P, P],
    "k8s_blaslt_clear_tuning": [],
    "k8s_blaslt_sweep": [P, I, P, I, ctypes.c_size_t, P, I, I, I, I, P, ctypes.c_size_t, I, P, I, P, P, P],
    "k8s_blaslt_set_algo": [I, I, I, I],
    "k8s_blaslt_set_algo_range": [I, I, I, I, I],
    "k8s_blaslt_heuristic_index": [I, I, I, ctypes.c_size_t],
    "k8s_gemm_mid_cfg": [I, P],
    "k8s_moe_route": [P, I, I, I, P, P, P],
    "k8s_moe_align": [P, I, I, I, P, P, P, P],
    "k8s_moe_combine": [P, P, P, I, I, I, P, P],
    "k8s_grouped_gemm": [P, I, P, P, I, P, I, I, I, I, I, I, P, I, P],
    "k8s_grouped_gemm_part": [P, I, P, P, I, P, I, I, I, I, I, I, P, I, P],
    "k8s_substr_search": [P, P, P, I, P, I, P, P, P],
    "k8s_graph_expand2": [P, P, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P],
    "k8s_state_lookup": [P, P, P, P, P, P, P, I, I, I, I, P, P, P, I, P, P, P],
    "k8s_window_mark": [I, P],
    "k8s_host_flag": [P, I, P],
    "k8s_kv_stage": [P, P, P, ctypes.c_long, I, I, P, I, I, P],
    "k8s_host_register": [P, ctypes.c_long],
    "k8s_host_unregister": [P],
    "k8s_memcpy_async": [P, P, ctypes.c_long, P],
    "k8s_set_knob": [I, I],
    "k8s_nonfinite_flag": [P, ctypes.c_long, P, P],
    "k8s_get_knob": [I],
    "k8s_walks": [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P, P, P, P],
}
# entry points whose C return type is not int
_RESTYPES = {"k8s_gemm_big_ws_bytes": ctypes.c_long, "k8s_gemm_big_tail_foreign": ctypes.c_long}


def lib():
    """The loaded library; raises if unavailable."""
    global _lib, _err
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            # K8SRCA_HIP_LIB: an alternate build of the same sources (compile-time
            # A/Bs, e.g. tools/_nt_ab.sh); the in-tree library otherwise
            path = KNOBS.hip_lib or _build.hip_lib_path()
            if not os.path.exists(path):
                if KNOBS.autobuild:
                    _build.build_hip()
                else:
                    raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
            L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            for name, args in _SIGS.items():
                fn = getattr(L, name, None)
                if fn is None:
                    continue
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, ctypes.c_int)
            push_native(L)
            _lib = L
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except Exception:  # noqa: BLE001
        return False


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(t: torch.Tensor = None) -> int:
    """Raw hipStream_t of the current stream on ``t``'s device.  The C fast
    path skips the Stream object torch.cuda.current_stream() builds (~4 us a
    call; an eager 8B forward issues ~350 kernels)."""
    if _raw_stream is not None:
        if t is not None and t.device.index is not None:
            return _raw_stream(t.device.index)
        return _raw_stream(torch.cuda.current_device())
    return torch.cuda.current_stream(t.device if t is not None else None).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


_SYNC_DEBUG = KNOBS.sync_debug


def scratch(shape, dtype, device) -> torch.Tensor:
    """An uninitialised device buffer that kernels must write before they read
    (split-K / split-KV partials, activations).  Knob ``poison``: filled with
    NaN instead, so a read of an unwritten element is loud, not stale data."""
    if isinstance(shape, int):
        shape = (shape,)
    if KNOBS.poison and dtype.is_floating_point:
        return torch.full(shape, float("nan"), dtype=dtype, device=device)
    return torch.empty(shape, dtype=dtype, device=device)


def check(rc: int, name: str) -> None:
    """Raise on a launch error.  ``K8SRCA_SYNC_DEBUG=1`` (SURVEY.md §5.2 debug
    mode) also synchronises after every kernel so an asynchronous fault is
    reported at the op that caused it, not at a later sync."""
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    if _SYNC_DEBUG and torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError(f"{name}: device fault surfaced at sync: {e}") from e


def use_hip(*tensors) -> bool:
    """True when the op must run on the HIP kernels (device tensors)."""
    for t in tensors:
        if t is not None and t.is_cuda:
            if _lib is None:
                lib()  # fail loudly when the native library is missing
            return True
    return False
