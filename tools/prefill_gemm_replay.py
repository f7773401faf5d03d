"""Replay the prefill-size projection GEMMs of a recorded run (knob shape_trace:
``K8SRCA_SHAPE_TRACE=path python bench.py ...``) with the engine's own
choices -- the dispatch / gemm_big table, the SwiGLU-fused gate_up -- and
report time and TFLOP/s per step-size bucket: which M ranges the mixed
steps' weight passes waste.

    python tools/prefill_gemm_replay.py trace.jsonl [--model llama3-8b]

A step's M is its decode rows + prefill tokens (every projection runs over
all of them); steps with M <= 256 are the decode GEMMs' (not replayed here).
"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.models.config import get_config  # noqa: E402
from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402


def timeit(fn, iters=6, warm=2):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def bucket(M):
    b = 1 << (M.bit_length() - 1)
    step = max(1, b // 16)
    return (M + step - 1) // step * step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--out", default=None, help="write the per-M table as JSON lines")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    mc = get_config(a.model)
    LIN.reserve_lib_workspace(dev)
    LIN.load_lib_algos(LIN.lib_algos_path(a.model))
    LIN.load_dispatch(LIN.dispatch_path(a.model))
    LIN.load_big(LIN.big_path(a.model))
    LIN.reserve_dispatch_scratch(dev)
    H, I, D = mc.hidden, mc.intermediate, mc.head_dim
    shapes = {"qkv": ((mc.n_heads + 2 * mc.n_kv_heads) * D, H), "o": (H, mc.n_heads * D), "gate_up": (2 * I, H),
              "down": (H, I)}
    W = {k: (torch.randn(n, kk, device=dev) * 0.02).bfloat16() for k, (n, kk) in shapes.items()}
    flops_row = 2.0 * sum(n * k for n, k in shapes.values())
    steps = [json.loads(line) for line in open(a.trace)]
    Ms = [len(s["d"]) + sum(q for _, q in s["p"]) for s in steps]
    Ms = [M for M in Ms if M > 256]
    cache = {}

    def layer_us(M):
        if M not in cache:
            x = {k: torch.randn(M, w.shape[1], device=dev).bfloat16() for k, w in W.items()}
            t = {}
            for k, w in W.items():
                if k == "gate_up" and LIN.swiglu_choice(M, w.shape[0], w.shape[1]):
                    t[k] = timeit(lambda: LIN.swiglu_gemm(x[k], w))
                else:
                    t[k] = timeit(lambda: LIN.linear(x[k], w))
            picks = {k: list(LIN.select_gemm(M, w.shape[0], w.shape[1])) for k, w in W.items()}
            cache[M] = (t, picks)
        return cache[M]

    ranges = [(256, 512), (512, 1024), (1024, 2048), (2048, 4096), (4096, 1 << 20)]
    agg = collections.defaultdict(lambda: [0, 0, 0.0, 0.0])  # steps, rows, us, flops
    rows_out = []
    for M in Ms:
        Mb = bucket(M)
        t, picks = layer_us(Mb)
        us = sum(t.values()) * mc.n_layers * M / Mb
        r = next(rg for rg in ranges if rg[0] < M <= rg[1])
        g = agg[r]
        g[0] += 1
        g[1] += M
        g[2] += us
        g[3] += flops_row * M * mc.n_layers
    tot = sum(g[2] for g in agg.values())
    for r in ranges:
        g = agg.get(r)
        if not g:
            continue
        print(json.dumps({"M_range": f"{r[0] + 1}-{r[1]}", "steps": g[0], "rows": g[1], "s": round(g[2] / 1e6, 3),
                          "share": round(g[2] / tot, 3), "tflops": round(g[3] / g[2] / 1e6, 0)}), flush=True)
    for Mb in sorted(cache):
        t, picks = cache[Mb]
        us = sum(t.values())
        rows_out.append({"M": Mb, "us_layer": round(us, 1), "tflops": round(flops_row * Mb / us / 1e6, 0),
                         **{f"us_{k}": round(v, 1) for k, v in t.items()}, "picks": picks})
    print(json.dumps({"total_s": round(tot / 1e6, 3), "steps": len(Ms)}))
    if a.out:
        with open(a.out, "w") as f:
            for r in rows_out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
