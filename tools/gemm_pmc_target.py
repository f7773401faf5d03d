"""A short fixed workload for tools/pmc.sh: the 8B decode projections at one M on the
dispatch's kernels (gate_up + SwiGLU cfg 23, o cfg 14 x4, qkv cfg 23 x4, down cfg 23 x8),
cold rotated weights, 40 launches each.  python tools/gemm_pmc_target.py [M]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 96
L.reserve_mid_scratch(torch.device("cuda"), 256, 28672)
x4 = torch.randn(M, 4096, dtype=torch.bfloat16, device="cuda")
x14 = torch.randn(M, 14336, dtype=torch.bfloat16, device="cuda")
runs = [("gate_up", 28672, 4096, lambda w: L.gemm_stream_silu(x4, w, 23)),
        ("o", 4096, 4096, lambda w: L.gemm_stream(x4, w, 14, 4)),
        ("qkv", 6144, 4096, lambda w: L.gemm_stream(x4, w, 23, 4)),
        ("down", 4096, 14336, lambda w: L.gemm_stream(x14, w, 23, 8))]
for name, N, K, fn in runs:
    ws = [torch.randn(N, K, dtype=torch.bfloat16, device="cuda") * 0.02 for _ in range(max(2, (1 << 30) // (N * K * 2)))]
    for i in range(40):
        fn(ws[i % len(ws)])
    torch.cuda.synchronize()
    del ws
print("done", M)
