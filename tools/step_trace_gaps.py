"""Step-boundary idle from the engine's step trace (knob ``step_trace``).

    python tools/step_trace_gaps.py trace.jsonl [--from-frac 0.3]

Per forward k the trace holds its GPU start / end (timing events around the
forward's whole enqueued work, on one GPU clock) and three host times: the end
of the last token wait before it (``t_wait``: the sample of step k-2 landed,
i.e. about when the GPU began forward k-1), the start of step k's scheduling
(``t_step``) and the forward's enqueue (``t_enq0``).  The GPU idles between
forwards k-1 and k when the host's path wait -> enqueue is longer than forward
k-1 itself; this splits that path into post-processing (wait -> step start)
and scheduling + packing (step start -> enqueue), by the kinds of the steps
around the gap.
"""
import argparse
import collections
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-frac", type=float, default=0.3)
    ap.add_argument("--min-ms", type=float, default=0.05)
    a = ap.parse_args()
    rs = [json.loads(l) for l in open(a.trace) if l.strip()]
    rs = [r for r in rs if "g0" in r]
    rs.sort(key=lambda r: r["g0"])
    rs = rs[int(a.from_frac * len(rs)):]
    span = rs[-1]["g1"] - rs[0]["g0"]
    busy = sum(r["g1"] - r["g0"] for r in rs)
    gaps = []
    for p, r in zip(rs, rs[1:]):
        g = r["g0"] - p["g1"]
        if g < a.min_ms:
            continue
        post = (r["t_step"] - r["t_wait"]) if r.get("t_step") is not None and r.get("t_wait") is not None else None
        sched = (r["t_enq0"] - r["t_step"]) if r.get("t_step") is not None else None
        gaps.append((g, p, r, post, sched))
    tot = sum(g for g, *_ in gaps)
    print(f"forwards {len(rs)}, GPU span {span / 1e3:.2f} s, inside forwards {busy / 1e3:.2f} s "
          f"({100 * busy / span:.1f} %), gaps >= {a.min_ms} ms between forwards: {len(gaps)} = {tot / 1e3:.3f} s "
          f"({100 * tot / span:.1f} %)")
    by = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
    for g, p, r, post, sched in gaps:
        k = (p["kind"], r["kind"])
        b = by[k]
        b[0] += 1
        b[1] += g
        b[2] += post or 0.0
        b[3] += sched or 0.0
        b[4] += p["g1"] - p["g0"]
    # inside a forward: GPU waiting for the host's packing + upload at its start (gk - g0)
    ks = [r for r in rs if r.get("gk") is not None]
    if ks:
        waits = [r["gk"] - r["g0"] for r in ks]
        tot_w = sum(waits)
        by_k = collections.defaultdict(lambda: [0, 0.0])
        for r, w in zip(ks, waits):
            by_k[r["kind"]][0] += 1
            by_k[r["kind"]][1] += w
        print(f"step start -> upload landed (GPU waits for packing + upload): {tot_w / 1e3:.3f} s "
              f"({100 * tot_w / span:.1f} % of the span); " +
              ", ".join(f"{k}: {n} steps, mean {w / n:.3f} ms" for k, (n, w) in by_k.items()))
    print("prev -> next kind      n     gap ms   mean gap   mean post   mean sched   mean prev GPU ms")
    for k, (n, g, po, sc, f) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[0]:>6} -> {k[1]:<6} {n:6d} {g:10.1f} {g / n:10.3f} {po / n:11.3f} {sc / n:12.3f} {f / n:14.3f}")
    hist = collections.Counter()
    for g, *_ in gaps:
        hist[next(x for x in (0.1, 0.5, 1, 2, 5, 1e9) if g <= x)] += 1
    print("gap histogram (<= ms):", dict(sorted(hist.items())))
    big = sorted(gaps, key=lambda x: -x[0])[:12]
    print("largest gaps: gap, prev kind/nd/np/GPU ms, next kind/nd/np, post ms, sched ms")
    for g, p, r, post, sched in big:
        print(f"  {g:7.3f}  {p['kind']}/{p['nd']}/{p['np']}/{p['g1'] - p['g0']:.2f}  {r['kind']}/{r['nd']}/{r['np']}"
              f"  {post if post is None else round(post, 3)}  {sched if sched is None else round(sched, 3)}")


if __name__ == "__main__":
    main()
