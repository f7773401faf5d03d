"""Interleaved A/B of the decode attention's K/V cache policy (knob
decode_kv_nt: non-temporal loads vs the default policy) on the decode steps of
a recorded run (shape trace), in one process: bit-identity and us per step.

    python tools/decode_nt_ab.py TRACE.jsonl[.gz] [--samples 40] [--rounds 3] [--shared 0]

``--shared L``: the first L keys of every row sit on pages shared by groups
of 42 rows (the assistants' common prompt pages), which the default policy
can keep in L2 / MALL and the nt policy may not.
"""
import argparse
import gzip
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.knobs import set_knob  # noqa: E402
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402
from tools.bench_kernels import make_meta, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--samples", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shared", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    op = gzip.open if a.trace.endswith(".gz") else open
    steps = [json.loads(line) for line in op(a.trace, "rt")]
    dec = [s["d"] for s in steps if len(s["d"]) >= 32]
    g = torch.Generator().manual_seed(0)
    idx = torch.randperm(len(dec), generator=g)[: a.samples].tolist()
    nq, nkv, BS = 32, 8, 64
    tot = {False: [], True: []}
    byts = 0
    for i in idx:
        ctx = dec[i]
        B = len(ctx)
        meta, nb = make_meta(ctx, [1] * B, nq, nkv, BS, dev, True)
        if a.shared:
            ls = a.shared // BS
            bt = meta.block_tables.cpu()
            for s0 in range(0, B, 42):
                bt[s0:s0 + 42, :ls] = bt[s0, :ls].clone()
            meta.block_tables = bt.to(dev)
        kc = torch.empty(nb, nkv, BS, 128, device=dev, dtype=torch.bfloat16).normal_()
        vc = torch.empty(nb, nkv, 128, BS, device=dev, dtype=torch.bfloat16).normal_()
        q = torch.randn(B, (nq + 2 * nkv) * 128, device=dev).bfloat16()
        outs = {}
        for nt in (False, True):
            set_knob("decode_kv_nt", nt)
            outs[nt] = A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128)).clone()
        assert torch.equal(outs[False], outs[True])
        out = torch.empty(B, nq * 128, device=dev).bfloat16()
        t = {False: [], True: []}
        for _ in range(a.rounds):
            for nt in (False, True):
                set_knob("decode_kv_nt", nt)
                t[nt].append(timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out),
                                    iters=10, warm=2))
        for nt in (False, True):
            tot[nt].append(statistics.median(t[nt]))
        byts += sum(ctx) * nkv * 512
        del kc, vc
    set_knob("decode_kv_nt", False)
    res = {}
    for nt in (False, True):
        us = sum(tot[nt])
        res["nt" if nt else "default"] = {"us_per_step": round(us / len(idx), 1), "tbps": round(byts / us / 1e6, 3)}
    res["gain_pct"] = round(100 * (sum(tot[False]) - sum(tot[True])) / sum(tot[False]), 2)
    res["shared_keys"] = a.shared
    print(json.dumps(res))


if __name__ == "__main__":
    main()
