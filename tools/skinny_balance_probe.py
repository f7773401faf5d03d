"""M = 1 skinny GEMM time vs N at K = 4096 (cold weights): is the qkv projection
(N = 6144 -> 384 workgroups on 256 CUs) paying a second partial round?"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops._lib import check, lib, stream_ptr  # noqa: E402


def t_us(fn, iters=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


K = 4096
for M in (1, 8):
    for N in (2048, 4096, 6144, 8192, 10240, 12288):
        ws = [torch.randn(N, K, dtype=torch.bfloat16, device="cuda") for _ in range(max(2, (1 << 30) // (N * K * 2)))]
        x = torch.randn(M, K, dtype=torch.bfloat16, device="cuda")
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        c = [0]

        def run():
            c[0] += 1
            w = ws[c[0] % len(ws)]
            check(lib().k8s_gemm_skinny(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, stream_ptr()), "skinny")
        us = t_us(run)
        print(f"M={M} N={N:6d} WGs={N // 16:4d}  {us:6.2f} us  {N * K * 2 / us / 1e6:5.2f} TB/s", flush=True)
        del ws
