"""GPU idle gaps grouped by the kind of step that preceded them.

    python tools/gap_steps.py run_kernel_trace.csv [--min-us 100] [--from-frac 0.5]

Splits the kernel timeline at idle gaps >= min-us (step boundaries where the
host was behind), and reports how much idle follows decode-only segments vs
segments with prefill attention, bucketed by the segment's GPU time -- i.e.
whether short steps (host work > GPU work) or something else leaves the GPU idle.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("--min-us", type=float, default=100)
    ap.add_argument("--from-frac", type=float, default=0.0)
    a = ap.parse_args()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(a.kernels)))
    t0 = ks[0][0] + a.from_frac * (ks[-1][1] - ks[0][0])
    ks = [k for k in ks if k[0] >= t0]
    segs = []  # (busy_ns, has_prefill, gap_after_ns, n_kernels)
    cur = [0, False, 0]
    end = ks[0][1]
    seg_start = ks[0][0]
    for s, e, n in ks:
        if s - end >= a.min_us * 1e3:
            segs.append((end - seg_start, cur[1], s - end, cur[2]))
            cur = [0, False, 0]
            seg_start = s
        cur[1] |= "attn_prefill" in n
        cur[2] += 1
        end = max(end, e)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for busy, pf, gap, n in segs:
        b = next(x for x in (2, 5, 10, 20, 50, 1e9) if busy / 1e6 <= x)
        k = ("prefill" if pf else "decode", b)
        agg[k][0] += 1
        agg[k][1] += gap / 1e6
        agg[k][2] += busy / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"{len(segs)} segments; idle {tot:.1f} ms after them")
    for k, (n, g, b) in sorted(agg.items()):
        print(f"  {k[0]:8s} busy<={k[1]:>5} ms: {n:5d} segs, idle after {g:8.1f} ms (avg {g / n:6.2f}), busy {b:8.1f} ms")


if __name__ == "__main__":
    main()
