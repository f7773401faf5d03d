"""Does a swept hipBLASLt solution keep its swept time once registered?
For a few (M, N, K): k8s_blaslt_sweep (every solution, cold rotated weights)
-> best index + time; then k8s_blaslt_set_algo(M, N, K, idx) and time the
engine's own call path (ops/linear.py lib_gemm) on the same rotated weights,
next to the heuristic's plan.

    python3 tools/blaslt_check.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402
from k8s_llm_rca_amd.ops._lib import lib, ptr, stream_ptr  # noqa: E402


def time_lib(x, w, y, nw, iters=8):
    for i in range(2):
        L.lib_gemm(x, w[i % nw], out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        L.lib_gemm(x, w[i % nw], out=y)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = torch.device("cuda")
    L.reserve_lib_workspace(dev)
    ws = L._blaslt_ws[dev]
    for M, N, K in [(2048, 28672, 4096), (1536, 28672, 4096), (4096, 4096, 14336), (256, 6144, 4096)]:
        nw = max(2, min(12, int(1.2e9 // (N * K * 2))))
        w = torch.randn(nw, N, K, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        L.clear_lib_tuning()
        t_heur = time_lib(x, w, y, nw)
        idx = (ctypes.c_int * 4)()
        us = (ctypes.c_float * 4)()
        times = (ctypes.c_float * 1)()
        n = lib().k8s_blaslt_sweep(ptr(x), K, ptr(w), nw, N * K, ptr(y), N, M, N, K, ptr(ws), L.BLASLT_WS_BYTES,
                                   8, stream_ptr(x), 4, idx, us, times)
        rc = lib().k8s_blaslt_set_algo(M, N, K, int(idx[0]))
        t_reg = time_lib(x, w, y, nw)
        t_reg2 = time_lib(x, w, y, nw)
        print(f"M {M} N {N} K {K}: lib heuristic {t_heur:.1f} us | sweep heuristic {times[0]:.1f} best {us[0]:.1f} "
              f"(idx {idx[0]}, n {n}) | registered (rc {rc}) {t_reg:.1f} / {t_reg2:.1f} us", flush=True)
        L.clear_lib_tuning()
        del w, x, y


if __name__ == "__main__":
    main()
