"""Per-kernel time split by launch grid size, from a rocprofv3 kernel trace.

    python tools/trace_by_grid.py run_kernel_trace.csv [--match rmsnorm|rope|silu] [--top 40]

Shows where a small kernel's time goes by problem size (a decode step's
~100-row launch vs a prefill chunk's thousands of rows): calls, total ms and
median us per (kernel, grid) row, sorted by total time.
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="rmsnorm|rope|silu")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    pat = re.compile(a.match)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        n = r["Kernel_Name"]
        if not pat.search(n):
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]))
        agg[(re.sub(r"\(.*", "", n)[:48], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for v in agg.values())
    print(f"total {tot / 1e3:.1f} ms over {sum(len(v) for v in agg.values())} launches matching /{a.match}/")
    for (n, g), v in rows[: a.top]:
        v.sort()
        print(f"{sum(v) / 1e3:9.1f} ms {len(v):8d} x med {v[len(v) // 2]:7.2f} us  wgs {g:7d}  {n}")


if __name__ == "__main__":
    main()
