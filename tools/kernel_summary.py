"""Group a rocprofv3 ``*_kernel_stats.csv`` into op categories.

    python tools/kernel_summary.py run_kernel_stats.csv [--top 12]

Prints one line per category (total ms, share, calls) and the top kernels,
so profiles/ summaries can be compared between runs without the full CSV.
"""
import argparse
import csv
import re
from collections import defaultdict

CATS = [
    ("attn_decode", r"attn_decode|attn_reduce"),
    ("attn_prefill", r"attn_prefill"),
    ("gemm_hipblaslt", r"^(Custom_)?Cijk"),
    ("gemm_big", r"gemm_big|big_reduce"),  # hand-written 256x256 prefill GEMM (+ fused epilogues)
    ("gemm_decode", r"gemm_skinny|gemm_mid|gemm_glds|gemm_stream"),  # M <= 256 weight-streaming kernels
    ("gemm_grouped", r"grouped_gemm|grouped_glds|grouped_reduce"),  # MoE experts, and split-K dense GEMMs (dispatch 'grp')
    ("moe", r"moe"),
    ("norm_rope_act", r"rmsnorm|rope|silu|layernorm|relu"),
    ("sampling", r"sample|gumbel|argmax"),
    ("allreduce", r"allreduce|\bar_kernel|ar_addnorm|a2a_kernel|ncclDevKernel|rccl"),
    ("graph", r"graph|csr|contains|walk|expand"),
]


def category(name: str) -> str:
    short = re.sub(r"^void ", "", name)
    short = re.sub(r"^k8s::", "", short)
    for cat, pat in CATS:
        if re.search(pat, short):
            return cat
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    cats = defaultdict(lambda: [0.0, 0])
    for r in rows:
        c = cats[category(r["Name"])]
        c[0] += float(r["TotalDurationNs"])
        c[1] += int(r["Calls"])
    print(f"total kernel time {tot / 1e6:.1f} ms")
    for k, (ns, n) in sorted(cats.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:16s} {ns / 1e6:10.1f} ms {100 * ns / tot:6.2f} %  {n:8d} calls")
    print("top kernels:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        nm = re.sub(r"\(.*", "", r["Name"])[:90]
        print(f"  {float(r['TotalDurationNs']) / 1e6:10.1f} ms {float(r['Percentage']):6.2f} %  "
              f"{int(r['Calls']):8d} x {float(r['AverageNs']) / 1e3:8.1f} us  {nm}")


if __name__ == "__main__":
    main()
