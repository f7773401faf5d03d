"""hipBLASLt heuristic vs the swept solution table (data/blaslt_algos_<model>.json)
on the prefill-sized projection GEMMs of a recorded headline run.

Replays every step of ``--trace`` with M > 256 (M = decode rows + prefill
tokens) through the native hipBLASLt front end (ops/linear.py lib_gemm) with
cold, rotated weights, and prints the summed time per M range.  Run once with
K8S_BLASLT_ALGOS=0 and once with =1 (the front end caches each shape's plan at
first use, so the two variants need separate processes).  ``--pad`` also times
each M padded up to the next ladder point the table was swept at.

    K8S_BLASLT_ALGOS=1 python3 tools/blaslt_ab.py --trace profiles/r2_shape_trace.jsonl
"""
import argparse
import json
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def bucket(M):
    b = 1 << (M.bit_length() - 1)
    step = max(1, b // 32)
    return (M + step - 1) // step * step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default="profiles/r2_shape_trace.jsonl")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--pad", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    L.reserve_lib_workspace(dev)
    n_alg = L.load_lib_algos(L.lib_algos_path(a.model))
    table = json.load(open(L.lib_algos_path(a.model))).get("algos", {})
    steps = [json.loads(l) for l in open(a.trace)]
    Ms = [len(s["d"]) + sum(q for _, q in s["p"]) for s in steps]
    freq = Counter(bucket(M) for M in Ms if M > 256)
    print(f"algos registered {n_alg}; {sum(freq.values())} steps with M > 256, {len(freq)} buckets", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = Counter()
    for name, (N, K) in SHAPES.items():
        nw = max(2, min(12, int(1.2e9 // (N * K * 2))))
        w = torch.randn(nw, N, K, device=dev).bfloat16()
        ladder = sorted(int(m) for m in table.get(f"{N},{K}", {}))
        for M, cnt in sorted(freq.items()):
            Mr = M
            if a.pad:
                up = [m for m in ladder if m >= M]
                Mr = up[0] if up and up[0] - M <= max(64, M // 8) else M
            x = torch.randn(Mr, K, device=dev).bfloat16()
            y = torch.empty(Mr, N, device=dev, dtype=torch.bfloat16)
            for i in range(2):
                L.lib_gemm(x, w[i % nw], out=y)
            torch.cuda.synchronize()
            e0.record()
            for i in range(a.iters):
                L.lib_gemm(x, w[i % nw], out=y)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            rng = "M<=1024" if M <= 1024 else "M<=2048" if M <= 2048 else "M>2048"
            tot[rng] += us * cnt * 32
            tot[name] += us * cnt * 32
            del x, y
        del w
        print(f"{name:8s} {tot[name] / 1e6:.3f} s", flush=True)
    for k in ("M<=1024", "M<=2048", "M>2048"):
        print(f"range {k:8s} {tot[k] / 1e6:.3f} s", flush=True)
    print(f"total {sum(tot[n] for n in SHAPES) / 1e6:.3f} s (algos={os.environ.get('K8S_BLASLT_ALGOS', '0')}, "
          f"pad={a.pad})", flush=True)


if __name__ == "__main__":
    main()
