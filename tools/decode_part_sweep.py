"""Keys per decode work item at low concurrency: time the paged decode
attention (work-list kernel + split-KV reduce) for a few rows over cold K/V
(every call reads a different copy of the caches, as a layer does at
concurrency 1), per candidate partition size.

    python tools/decode_part_sweep.py [--rows 1,2,4,8] [--ctx 2048,5000,8000] [--parts 64,128,192,256,384,512]

Prints one JSON line per (rows, ctx): us per call for every part size and the
planner's own choice (ops/attention.py:plan_decode_split).
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.ops import attention as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,2,4,8")
    ap.add_argument("--ctx", default="2048,5000,8000")
    ap.add_argument("--parts", default="64,128,192,256,384,512")
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--iters", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    nq, nkv, BS, D = 32, 8, 64, 128
    torch.manual_seed(0)
    for S in [int(v) for v in a.rows.split(",")]:
        for c in [int(v) for v in a.ctx.split(",")]:
            ctx = [c] * S
            nb = S * ((c + BS - 1) // BS)
            kc = torch.empty(nb * a.copies, nkv, BS, D, device=dev, dtype=torch.bfloat16).normal_()
            vc = torch.empty(nb * a.copies, nkv, D, BS, device=dev, dtype=torch.bfloat16).normal_()
            q = torch.randn(S, (nq + 2 * nkv) * D, device=dev).bfloat16()
            out = torch.empty(S, nq * D, device=dev).bfloat16()
            row = {"rows": S, "ctx": c, "planner": A.plan_decode_split(ctx, nkv)[1]}
            ref = None
            for P in [int(v) for v in a.parts.split(",")]:
                metas = []
                for i in range(a.copies):
                    bt = (torch.arange(nb, dtype=torch.int32).view(S, -1) + i * nb).to(dev)
                    m = A.AttnMeta(block_tables=bt, ctx_lens=torch.tensor(ctx, dtype=torch.int32, device=dev),
                                   q_start=torch.arange(S + 1, dtype=torch.int32, device=dev), num_seqs=S, decode=True)
                    metas.append(A.attach_decode_plan(m, ctx, nq, nkv, BS, dev, part=P))
                o = A.paged_attention(q, kc, vc, metas[0], nq, nkv, 1 / math.sqrt(D)).float()
                if ref is None:
                    ref = o
                err = (o - ref).abs().max().item()
                # one HIP graph of `iters` calls: eager launches would time the host, not the kernels
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(a.iters):
                        A.paged_attention(q, kc, vc, metas[i % a.copies], nq, nkv, 1 / math.sqrt(D), out=out)
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                row[f"P{P}"] = round(e0.elapsed_time(e1) * 1e3 / a.iters, 2)
                row[f"err{P}"] = round(err, 4)
            print(json.dumps(row), flush=True)
            del kc, vc


if __name__ == "__main__":
    main()
