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
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", ""))
                 for r in csv.DictReader(open(a.api)))
    starts = [x[0] for x in api]
    by = collections.defaultdict(float)
    cnt = collections.Counter()
    tot = 0.0
    for g0, g1, p, n in gaps:
        tot += g1 - g0
        i = bisect.bisect_left(starts, g0 - 50_000_000)  # calls that began up to 50 ms before the gap
        for s, e, f, t in api[i:]:
            if s > g1:
                break
            ov = min(e, g1) - max(s, g0)
            if ov > 0:
                by[(f, t)] += ov
                cnt[(f, t)] += 1
    print(f"{len(gaps)} gaps >= {a.min_us} us, {tot / 1e6:.1f} ms idle")
    for (f, t), v in sorted(by.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v / 1e6:9.1f} ms overlap  {cnt[(f, t)]:7d} calls  thread {t}  {f}")


if __name__ == "__main__":
    main()
