"""Summarise idle gaps between consecutive kernels of a rocprofv3 kernel trace.

    python tools/trace_gaps.py run_kernel_trace.csv [FROM_FRAC] > gaps.json

FROM_FRAC (0..1) drops the kernels that start in the first part of the trace
(setup + warmup) so the busy/idle figures describe the timed region.

Gaps are attributed to the (previous kernel -> next kernel) name pair, so host
work between steps (after the sampling kernel) separates from launch gaps
inside a forward.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*>", "", n)
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "hipblaslt_gemm"
    return n.split("::")[-1][:60]


def main(path, from_frac=0.0):
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ks.sort()
    if from_frac > 0:  # e.g. the timed step of a warmup + timed run
        t_cut = ks[0][0] + from_frac * (ks[-1][1] - ks[0][0])
        ks = [k for k in ks if k[0] >= t_cut]
    busy_end = ks[0][1]
    total_gap = 0
    hist = defaultdict(lambda: [0, 0])
    pairs = defaultdict(lambda: [0, 0])
    big = defaultdict(lambda: [0, 0])  # >= 1 ms gaps only
    prev = ks[0][2]
    for s, e, n in ks[1:]:
        if s > busy_end:
            g = s - busy_end
            total_gap += g
            b = "<10us" if g < 1e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
            hist[b][0] += 1
            hist[b][1] += g
            pairs[(prev, n)][0] += 1
            pairs[(prev, n)][1] += g
            if g >= 1e6:
                big[(prev, n)][0] += 1
                big[(prev, n)][1] += g
        if e > busy_end:
            busy_end = e
            prev = n
    span = ks[-1][1] - ks[0][0]
    top = sorted(pairs.items(), key=lambda kv: -kv[1][1])[:25]
    out = {"kernels": len(ks), "span_s": span / 1e9, "gap_s": total_gap / 1e9,
           "hist": {k: {"n": v[0], "s": v[1] / 1e9} for k, v in hist.items()},
           "top_pairs": [{"prev": p[0], "next": p[1], "n": v[0], "s": round(v[1] / 1e9, 4)} for p, v in top],
           "big_gap_pairs": [{"prev": p[0], "next": p[1], "n": v[0], "s": round(v[1] / 1e9, 4)}
                             for p, v in sorted(big.items(), key=lambda kv: -kv[1][1])[:10]]}
    mid = int(len(ks) * 0.7)
    win = []
    for s_, e_, n in ks[mid:mid + 400]:
        win.append([round((s_ - ks[mid][0]) / 1e3, 1), round((e_ - s_) / 1e3, 1), n])
    out["window_us"] = win  # [start offset, duration, name] of 400 consecutive kernels
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
