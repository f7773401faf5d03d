"""Compare BLAS backends / TunableOp on the decode-shape projections (run on GPU)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from tools.bench_kernels import timeit  # noqa: E402

shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
mode = sys.argv[1] if len(sys.argv) > 1 else "default"
if mode == "rocblas":
    torch.backends.cuda.preferred_blas_library("cublas")
for M in (16, 64, 128, 256):
    row = []
    for n, k in shapes:
        x = torch.randn(M, k, device="cuda").bfloat16()
        w = torch.randn(n, k, device="cuda").bfloat16()
        us = timeit(lambda: torch.nn.functional.linear(x, w), iters=20)
        row.append(f"N{n}K{k}:{us:6.1f}us {n * k * 2 / us / 1e6:4.2f}TB/s")
    print(mode, f"M{M}", " | ".join(row), flush=True)
