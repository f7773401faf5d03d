"""Bucketed hipBLASLt solution choice for the prefill-sized projections.

The per-ladder-point sweep (tools/blaslt_sweep.py) picks, at ONE M, the
fastest of several hundred noisy timings (a winner's curse at compute-bound
sizes) and its table was applied to every M up to the next ladder point; the
replay of recorded steps ran slower with it (profiles/r2_blaslt_ab/).  Here
each M bucket [lo, hi] gets: the top candidates of a sweep at its middle,
each then REGISTERED and re-timed through the engine's own call path
(ops/linear.py lib_gemm, cold rotated weights, median of repeats) at lo, mid
and hi next to the heuristic; a candidate is kept only if it beats the
heuristic at all three points and by --min-gain on their sum.

    python3 tools/blaslt_tune_buckets.py --emit   # writes data/blaslt_algos_<model>.json ("buckets")
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402
from k8s_llm_rca_amd.ops._lib import lib, ptr, stream_ptr  # noqa: E402

SHAPES = {"llama3-8b": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]}


def timed(x, w, y, nw, reps=3, iters=6):
    for i in range(2):
        L.lib_gemm(x, w[i % nw], out=y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0.record()
        for i in range(iters):
            L.lib_gemm(x, w[i % nw], out=y)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / iters * 1e3)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--edges", default="257,321,385,449,513,641,769,897,1025,1281,1537,1793,2049,2561,3073,3585,"
                    "4097,5121,6145,8449")
    ap.add_argument("--cands", type=int, default=4)
    ap.add_argument("--min-gain", type=float, default=1.03)
    ap.add_argument("--tol", type=float, default=1.02, help="a candidate may not be slower than this at any point")
    ap.add_argument("--emit", action="store_true")
    ap.add_argument("--out", default=None, help="also write the table here (e.g. under gpurun_out/)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    L.reserve_lib_workspace(dev)
    ws = L._blaslt_ws[dev]
    edges = [int(v) for v in a.edges.split(",")]
    buckets = [(edges[i], edges[i + 1] - 1) for i in range(len(edges) - 1)]
    table = {}
    tot_h = tot_b = 0.0
    for N, K in SHAPES[a.model]:
        nw = max(2, min(12, int(1.2e9 // (N * K * 2))))
        w = torch.randn(nw, N, K, device=dev).bfloat16()
        for lo, hi in buckets:
            mid = (lo + hi) // 2 // 8 * 8
            pts = [lo, mid, hi]
            xs = {m: torch.randn(m, K, device=dev).bfloat16() for m in pts}
            ys = {m: torch.empty(m, N, device=dev, dtype=torch.bfloat16) for m in pts}
            L.clear_lib_tuning()
            th = [timed(xs[m], w, ys[m], nw) for m in pts]
            idx = (ctypes.c_int * a.cands)()
            us = (ctypes.c_float * a.cands)()
            n = lib().k8s_blaslt_sweep(ptr(xs[mid]), K, ptr(w), nw, N * K, ptr(ys[mid]), N, mid, N, K, ptr(ws),
                                       L.BLASLT_WS_BYTES, 6, stream_ptr(w), a.cands, idx, us, None)
            # candidates: the sweep's top solutions at mid, and the heuristic's own
            # picks at M inside / just above the bucket (its choice is not monotone in M)
            cands = [int(idx[c]) for c in range(max(n, 0))]
            for m in sorted({lo, mid, hi, hi + 64, hi + 128, hi + (hi - lo + 1) // 2}):
                hi_idx = lib().k8s_blaslt_heuristic_index(m, N, K, L.BLASLT_WS_BYTES)
                if hi_idx >= 0 and hi_idx not in cands:
                    cands.append(hi_idx)
            best = None
            for cid in cands:
                L.clear_lib_tuning()
                if lib().k8s_blaslt_set_algo_range(lo, hi, N, K, cid) != 0:
                    continue
                tc = [timed(xs[m], w, ys[m], nw) for m in pts]
                if all(t <= h * a.tol for t, h in zip(tc, th)) and (best is None or sum(tc) < sum(best[1])):
                    best = (cid, tc)
            L.clear_lib_tuning()
            keep = best is not None and sum(th) / sum(best[1]) > a.min_gain
            tot_h += sum(th)
            tot_b += sum(best[1]) if keep else sum(th)
            print(f"N {N:6d} K {K:6d} M [{lo:5d},{hi:5d}] heuristic {' / '.join(f'{t:.1f}' for t in th)} us"
                  + (f"  cand {best[0]} of {len(cands)} {' / '.join(f'{t:.1f}' for t in best[1])} us ({sum(th) / sum(best[1]):.2f}x)"
                     if best else "  no candidate beats it everywhere") + ("  KEEP" if keep else ""), flush=True)
            if keep:
                table.setdefault(f"{N},{K}", []).append([lo, hi, best[0]])
            del xs, ys
        del w
    print(f"sum over buckets: heuristic {tot_h:.1f} us, chosen {tot_b:.1f} us ({tot_h / max(tot_b, 1e-9):.3f}x)",
          flush=True)
    doc = {"model": a.model, "note": "tools/blaslt_tune_buckets.py: per (N,K) [lo, hi, hipBLASLt solution index], "
           "each verified at lo/mid/hi on the engine's call path", "buckets": table}
    for path in ([L.lib_algos_path(a.model)] if a.emit else []) + ([a.out] if a.out else []):
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("wrote", path, flush=True)


if __name__ == "__main__":
    main()
