"""Decode attention at the headline shape (125 rows x ~4.7k keys, Llama-3-8B
heads) in isolation: scattered vs contiguous pages, per-kernel time under a
kernel trace (run under rocprofv3 --kernel-trace --stats; tools/_decode_probe.sh).

    python3 tools/decode_probe.py
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402

nq, nkv, BS, D = 32, 8, 64, 128


def meta_for(ctx, contiguous, dev, part=None):
    S = len(ctx)
    nbs = [(c + BS - 1) // BS for c in ctx]
    total = sum(nbs)
    perm = torch.arange(total) if contiguous else torch.randperm(total, generator=torch.Generator().manual_seed(1))
    maxb = max(nbs)
    bt = torch.zeros(S, maxb, dtype=torch.int32)
    used = 0
    for s, n in enumerate(nbs):
        bt[s, :n] = perm[used:used + n].int()
        used += n
    qs = list(range(S + 1))
    meta = A.AttnMeta(block_tables=bt.to(dev), ctx_lens=torch.tensor(ctx, dtype=torch.int32, device=dev),
                      q_start=torch.tensor(qs, dtype=torch.int32, device=dev), num_seqs=S, decode=True,
                      ctx_lens_host=list(ctx), q_start_host=qs)
    A.attach_decode_plan(meta, ctx, nq, nkv, BS, dev, part=part)
    return meta, total


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    rows = int(os.environ.get("PROBE_ROWS", "125"))
    lo, hi = int(os.environ.get("PROBE_CTX_LO", "3000")), int(os.environ.get("PROBE_CTX_HI", "6400"))
    ctx = (torch.randint(lo, hi, (rows,), generator=g)).tolist()
    parts = [None] + [int(v) for v in os.environ.get("PROBE_PARTS", "").split(",") if v]
    for contiguous, part in [(False, None), (True, None)] + [(False, p) for p in parts[1:]]:
        meta, nb = meta_for(ctx, contiguous, dev, part)
        kc = torch.empty(nb, nkv, BS, D, device=dev, dtype=torch.bfloat16).normal_()
        vc = torch.empty(nb, nkv, D, BS, device=dev, dtype=torch.bfloat16).normal_()
        q = torch.randn(len(ctx), (nq + 2 * nkv) * D, device=dev).bfloat16()
        out = torch.empty(len(ctx), nq * D, device=dev).bfloat16()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(D), out=out)
        torch.cuda.synchronize()
        e0.record()
        n = 20
        for _ in range(n):
            A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(D), out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        by = sum(ctx) * nkv * 512
        print(f"{'contiguous' if contiguous else 'scattered'} part={part}: {us:.1f} us per call (decode + reduce), "
              f"{by / us / 1e6:.2f} TB/s, part {meta.part_size}, items {meta.n_items}", flush=True)
        del kc, vc


if __name__ == "__main__":
    main()
