"""The engine's decode-size projection GEMMs (its dispatch-table choice, the
fused epilogue forms included) at one M, on cold rotated weights, for a kernel
trace or PMC pass (tools/pmc.sh) -- and event-timed per projection.

    python tools/decode_gemm_probe.py --m 96 [--shapes qkv,o,gate_up,down] [--iters 64]

Prints, per projection, the (kind, cfg, splits) the dispatch picks, us per
call and the weight-streaming rate; the per-layer sum is what a decode step
pays 32 times (Llama-3-8B).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.models.config import get_config  # noqa: E402
from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=96)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--copies", type=int, default=8, help="weight copies rotated (> MALL: every call cold)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    mc = get_config(a.model)
    LIN.reserve_lib_workspace(dev)
    assert LIN.load_dispatch(LIN.dispatch_path(a.model)), "dispatch table"
    LIN.reserve_dispatch_scratch(dev)
    H, I, D = mc.hidden, mc.intermediate, mc.head_dim
    shapes = {"qkv": ((mc.n_heads + 2 * mc.n_kv_heads) * D, H), "o": (H, mc.n_heads * D), "gate_up": (2 * I, H),
              "down": (H, I)}
    M = a.m
    torch.manual_seed(0)
    tot = 0.0
    for name in a.shapes.split(","):
        N, K = shapes[name]
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(a.copies)]
        x = torch.randn(M, K, device=dev).bfloat16()
        if name == "gate_up":
            pick = LIN.swiglu_choice(M, N, K)
            fn = (lambda w: LIN.swiglu_gemm(x, w)) if pick else (lambda w: LIN.linear(x, w))
        else:
            pick = LIN.select_gemm(M, N, K)
            fn = lambda w: LIN.linear(x, w)  # noqa: E731
        for w in ws:
            fn(w)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            fn(ws[i % len(ws)])
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        tot += us
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "pick": list(pick) if pick else None,
                          "us": round(us, 2), "tbps": round(N * K * 2 / us / 1e6, 2)}), flush=True)
    print(json.dumps({"M": M, "us_per_layer": round(tot, 1)}))


if __name__ == "__main__":
    main()
