"""Lightweight span recorder + ROCTX ranges.

``span(name)`` records wall time per stage into a process-wide aggregator
(count / total / max) and, when ``K8SRCA_ROCTX=1`` and
``librocprofiler-sdk-roctx.so`` is loadable, pushes a ROCTX range so
``rocprofv3 --marker-trace`` shows pipeline stages next to the HIP kernels.
"""
from __future__ import annotations

from ..knobs import KNOBS
import contextlib
import ctypes
import os
import threading
import time
from typing import Dict

_lock = threading.Lock()
_stats: Dict[str, list] = {}
_roctx = None
_roctx_tried = False


def _get_roctx():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        if KNOBS.roctx:
            for lib in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                        "libroctx64.so"):
                try:
                    _roctx = ctypes.CDLL(lib)
                    _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    break
                except OSError:
                    continue
    return _roctx


@contextlib.contextmanager
def span(name: str):
    rt = _get_roctx()
    if rt is not None:
        rt.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        if rt is not None:
            rt.roctxRangePop()
        with _lock:
            s = _stats.get(name)
            if s is None:
                _stats[name] = [1, dt, dt]
            else:
                s[0] += 1
                s[1] += dt
                if dt > s[2]:
                    s[2] = dt


def record(name: str, seconds: float) -> None:
    with _lock:
        s = _stats.get(name)
        if s is None:
            _stats[name] = [1, seconds, seconds]
        else:
            s[0] += 1
            s[1] += seconds
            s[2] = max(s[2], seconds)


def snapshot(reset: bool = False) -> Dict[str, Dict[str, float]]:
    with _lock:
        out = {k: {"count": v[0], "total_s": v[1], "mean_ms": 1e3 * v[1] / max(1, v[0]), "max_ms": 1e3 * v[2]}
               for k, v in _stats.items()}
        if reset:
            _stats.clear()
    return out


def reset() -> None:
    with _lock:
        _stats.clear()
