"""A/B of the LDS-DMA decode GEMM's hand-issued LDS reads (K8SRCA_GLDS_HAND).

For every Llama-3-8B projection at decode batch sizes, the dispatch table's
LDS-DMA configuration (data/gemm_dispatch_llama3-8b.json, cfg 13-16 / 23-24)
runs with hipcc's own fragment reads (HAND=0: lgkmcnt(0) before every MFMA
group) and with the hand-issued reads and counted waits (HAND=1), interleaved
in one process on cold rotated weights (one copy per layer); checks that both
give bit-identical outputs.

usage (GPU box): python tools/glds_hand_ab.py [--ms 64,96,128,160,192] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from k8s_llm_rca_amd.knobs import KNOBS, set_knob  # noqa: E402

from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,96,128,160,192")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    table = json.load(open(os.path.join(LIN.DATA_DIR, "gemm_dispatch_llama3-8b.json")))["shapes"]
    names = {"6144,4096": "qkv", "4096,4096": "o", "4096,14336": "down", "28672,4096": "gate_up"}
    rows = []
    for key, name in names.items():
        N, K = (int(v) for v in key.split(","))
        ws = [torch.randn(N, K, device=dev).bfloat16() for _ in range(a.layers)]
        for M in (int(m) for m in a.ms.split(",")):
            ent = min(table[key], key=lambda e: abs(e["m"] - M))
            cfg, splits = ent.get("cfg"), ent.get("splits") or 1
            if ent["kind"] != "stream" or not cfg or cfg < 13:
                continue
            x = torch.randn(M, K, device=dev).bfloat16()
            outs = {}
            for h in ("0", "1"):
                set_knob("glds_hand", h)
                outs[h] = LIN.gemm_stream(x, ws[0], cfg, splits).clone()
            torch.cuda.synchronize()
            same = bool(torch.equal(outs["0"], outs["1"]))
            res = {"0": [], "1": []}
            it = [0]

            def run():
                LIN.gemm_stream(x, ws[it[0] % a.layers], cfg, splits)
                it[0] += 1
            for _ in range(a.rounds):
                for h in ("0", "1"):
                    set_knob("glds_hand", h)
                    res[h].append(timed(run, a.iters))
            line = {"shape": name, "M": M, "cfg": cfg, "splits": splits, "bit_identical": same,
                    "us_hipcc_reads": round(statistics.median(res["0"]), 2),
                    "us_hand_reads": round(statistics.median(res["1"]), 2)}
            line["tbps_hand"] = round(N * K * 2 / line["us_hand_reads"] / 1e6, 2)
            rows.append(line)
            print(json.dumps(line), flush=True)
    set_knob("glds_hand", True)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "glds_hand_ab.jsonl")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
