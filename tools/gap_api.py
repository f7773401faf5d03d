"""Which host API calls overlap the GPU's idle gaps (rocprofv3 kernel + HIP API trace).

    python tools/gap_api.py run_kernel_trace.csv run_hip_api_trace.csv [--min-us 200]

For every idle gap >= min-us between consecutive kernels, sums the time of
the HIP API calls that overlap it, by API name and thread -- e.g. a
synchronising call or a slow graph launch shows up as the dominant row.
"""
import argparse
import bisect
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("api")
    ap.add_argument("--min-us", type=float, default=200)
    a = ap.parse_args()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40])
                for r in csv.DictReader(open(a.kernels)))
    gaps = []
    end = ks[0][1]
    prev = ks[0][2]
    for s, e, n in ks[1:]:
        if s - end >= a.min_us * 1e3:
            gaps.append((end, s, prev, n))
        if e > end:
            end, prev = e, n
    # one pass over the API calls: each call is matched to the gaps it overlaps by a
    # bisect on the (sorted, disjoint) gap starts -- O(calls log gaps); progress lines keep
    # a long trace from looking hung
    g_starts = [g[0] for g in gaps]
    by = collections.defaultdict(float)
    cnt = collections.Counter()
    tot = sum(g1 - g0 for g0, g1, _, _ in gaps)
    with open(a.api) as f:
        for n_row, r in enumerate(csv.DictReader(f)):
            if n_row % 500_000 == 0:
                print(f"# api rows {n_row}", flush=True)
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            j = bisect.bisect_right(g_starts, e0) - 1
            while j >= 0 and gaps[j][1] > s0:
                g0, g1 = gaps[j][0], gaps[j][1]
                ov = min(e0, g1) - max(s0, g0)
                if ov > 0:
                    key = (r["Function"], r.get("Thread_Id", ""))
                    by[key] += ov
                    cnt[key] += 1
                j -= 1
    print(f"{len(gaps)} gaps >= {a.min_us} us, {tot / 1e6:.1f} ms idle")
    for (f, t), v in sorted(by.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v / 1e6:9.1f} ms overlap  {cnt[(f, t)]:7d} calls  thread {t}  {f}")


if __name__ == "__main__":
    main()
