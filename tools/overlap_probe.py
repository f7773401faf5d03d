"""Decode attention and prefill attention of the same (mixed) engine step run
concurrently on two HIP streams vs one after the other, on the recorded step
shapes (profiles/r2_shape_trace.jsonl): is there headroom for overlapping the
MFMA-heavy prefill attention with the HBM-bound decode attention?

Variants per sampled mixed step (one layer's attention, Llama-3-8B heads):
  seq        decode (2048 waves) then prefill, one stream
  conc2048   decode on stream A, prefill on stream B (decode grid 2048 waves)
  conc1024   same, decode grid 1024 waves (one wave per SIMD: leaves VGPRs for prefill waves)
  dec1024    decode alone at 1024 waves

    python3 tools/overlap_probe.py [--samples 40]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402

nq, nkv, BS, D = 32, 8, 64, 128


def build(ctx, qlen, first_block, dev, decode):
    S = len(ctx)
    nbs = [(c + BS - 1) // BS for c in ctx]
    maxb = max(nbs)
    bt = torch.zeros(S, maxb, dtype=torch.int32)
    u = first_block
    for s, n in enumerate(nbs):
        bt[s, :n] = torch.arange(u, u + n, dtype=torch.int32)
        u += n
    qs = [0]
    for l in qlen:
        qs.append(qs[-1] + l)
    meta = A.AttnMeta(block_tables=bt.to(dev), ctx_lens=torch.tensor(ctx, dtype=torch.int32, device=dev),
                      q_start=torch.tensor(qs, dtype=torch.int32, device=dev), num_seqs=S, decode=decode,
                      ctx_lens_host=list(ctx), q_start_host=qs)
    if decode:
        A.attach_decode_plan(meta, ctx, nq, nkv, BS, dev)
    else:
        A.attach_plan(meta, A.plan_prefill(qs, nq // nkv, BS, list(ctx), nkv=nkv), dev)
    return meta, u


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default="profiles/r2_shape_trace.jsonl")
    ap.add_argument("--samples", type=int, default=40)
    ap.add_argument("--min-q", type=int, default=64, help="only steps with >= this many prefill tokens")
    a = ap.parse_args()
    dev = torch.device("cuda")
    steps = [json.loads(l) for l in open(a.trace)]
    mixed = [s for s in steps if s["d"] and s["p"] and sum(q for _, q in s["p"]) >= a.min_q]
    g = torch.Generator().manual_seed(0)
    idx = torch.randperm(len(mixed), generator=g)[: a.samples].tolist()
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    tot = {"seq": 0.0, "conc2048": 0.0, "conc1024": 0.0, "dec2048": 0.0, "dec1024": 0.0, "pre": 0.0}
    scale = 1 / math.sqrt(D)
    for i in idx:
        st = mixed[i]
        md, nb = build(st["d"], [1] * len(st["d"]), 0, dev, True)
        mp, nb = build([c for c, _ in st["p"]], [q for _, q in st["p"]], nb, dev, False)
        kc = torch.empty(nb, nkv, BS, D, device=dev, dtype=torch.bfloat16).normal_()
        vc = torch.empty(nb, nkv, D, BS, device=dev, dtype=torch.bfloat16).normal_()
        qd = torch.randn(len(st["d"]), (nq + 2 * nkv) * D, device=dev).bfloat16()
        T = sum(q for _, q in st["p"])
        qp = torch.randn(T, (nq + 2 * nkv) * D, device=dev).bfloat16()
        od = torch.empty(len(st["d"]), nq * D, device=dev).bfloat16()
        op = torch.empty(T, nq * D, device=dev).bfloat16()

        def dec(grid):
            md.grid_waves = grid
            A.paged_attention(qd, kc, vc, md, nq, nkv, scale, out=od)

        def pre():
            A.paged_attention(qp, kc, vc, mp, nq, nkv, scale, out=op)

        def timed(fn, reps=6):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps * 1e3

        def conc(grid):
            cur = torch.cuda.current_stream()
            sA.wait_stream(cur)
            sB.wait_stream(cur)
            with torch.cuda.stream(sA):
                dec(grid)
            with torch.cuda.stream(sB):
                pre()
            cur.wait_stream(sA)
            cur.wait_stream(sB)

        tot["seq"] += timed(lambda: (dec(2048), pre()))
        tot["conc2048"] += timed(lambda: conc(2048))
        tot["conc1024"] += timed(lambda: conc(1024))
        tot["dec2048"] += timed(lambda: dec(2048))
        tot["dec1024"] += timed(lambda: dec(1024))
        tot["pre"] += timed(pre)
        del kc, vc
    n = len(idx)
    for k, v in tot.items():
        print(f"{k:9s} {v / n:8.1f} us per layer-step (mean of {n} mixed steps)", flush=True)


if __name__ == "__main__":
    main()
