"""Decode-regime projection GEMMs at one M, each candidate kernel run in
isolation with cold (rotated) weights, for a kernel trace: run under
``rocprofv3 --kernel-trace`` and split the time per (kernel, grid) with
``tools/trace_by_grid.py --match gemm`` to separate the main kernel from its
split-K reduce.  Prints the candidate order and each one's event-timed cost.

    rocprofv3 --kernel-trace --output-format csv -d /tmp/p -o run -- python3 tools/gemm_probe.py --m 128
"""
import argparse
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=128)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--only", default="grp:x8,grp:x4,grp:x2,stream4:x8,stream4:x4,stream4:x2,stream8:x4,stream8:x2")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    shapes = [(6144, 4096), (4096, 4096), (4096, 14336)]
    keep = set(a.only.split(","))
    for N, K in shapes:
        wl = [torch.randn(N, K, device=dev).bfloat16() for _ in range(8)]  # > MALL: every call cold
        x = torch.randn(a.m, K, device=dev).bfloat16()
        lib_t = None
        for name, fn in [("lib", lambda x, w: torch.matmul(x, w.t()))] + L.candidate_kernels(a.m, N, K):
            if name != "lib" and name not in keep:
                continue
            for i in range(3):
                fn(x, wl[i % 8])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                fn(x, wl[i % 8])
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            lib_t = lib_t or us
            print(f"M{a.m} N{N} K{K} {name:14s} {us:7.1f} us  {N * K * 2 / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
