"""Replay the prefill-attention launches of a recorded run (K8S_RCA_SHAPE_TRACE)
for rocprofv3 PMC passes: the real mix of chunk sizes / contexts, not one shape.

    python tools/prof_prefill_replay.py --trace profiles/r2_shape_trace.jsonl --samples 40
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402
from tools.bench_kernels import make_meta  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default="profiles/r2_shape_trace.jsonl")
    ap.add_argument("--samples", type=int, default=40)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--max-q", type=int, default=0, help="only chunks with at most this many tokens (0: all)")
    ap.add_argument("--min-q", type=int, default=0)
    a = ap.parse_args()
    nq, nkv, BS, dev = 32, 8, 64, "cuda"
    steps = [json.loads(l)["p"] for l in open(a.trace)]
    steps = [[(c, q) for c, q in s if q >= a.min_q and (a.max_q == 0 or q <= a.max_q)] for s in steps]
    steps = [s for s in steps if s]
    g = torch.Generator().manual_seed(0)
    idx = torch.randperm(len(steps), generator=g)[: a.samples].tolist()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot_ms = 0.0
    for i in idx:
        ctx = [c for c, q in steps[i]]
        ql = [q for c, q in steps[i]]
        meta, nb = make_meta(ctx, ql, nq, nkv, BS, dev, False)
        kc = torch.empty(nb, nkv, BS, 128, device=dev, dtype=torch.bfloat16).normal_()
        vc = torch.empty(nb, nkv, 128, BS, device=dev, dtype=torch.bfloat16).normal_()
        T = sum(ql)
        q = torch.randn(T, (nq + 2 * nkv) * 128, device=dev).bfloat16()
        out = torch.empty(T, nq * 128, device=dev).bfloat16()
        A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out)
        e0.record()
        for _ in range(a.iters):
            A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out)
        e1.record()
        torch.cuda.synchronize()
        tot_ms += e0.elapsed_time(e1) / a.iters
    print(f"ok {len(idx)} steps, q in [{a.min_q}, {a.max_q or 'inf'}]: {tot_ms * 1e3 / len(idx):.1f} us per step")


if __name__ == "__main__":
    main()
