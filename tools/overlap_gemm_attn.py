"""Can an HBM-bound decode attention overlap a compute-bound prefill GEMM?

The r2 probe (tools/overlap_probe.py) paired decode attention with PREFILL
ATTENTION -- both stream K/V through HBM / L2 and did not overlap.  A mixed
engine step also holds the opposite pairing: the decode rows' attention
(435 us per layer at the headline shape, at the HBM roof, few MFMAs) and the
prefill rows' projections (hipBLASLt at ~1.2-1.5 PFLOP/s, MFMA-bound).  This
times, at the headline decode shape (125 rows x 3-6.4k keys, scattered pages)
and a prefill GEMM of M rows (gate_up 28672 x 4096 by default):
attention alone, GEMM alone, and both issued on two streams at once (the
attention's persistent grid capped at several sizes so GEMM workgroups can
land beside it).  Interleaved rounds, one process.

    python tools/overlap_gemm_attn.py [--m 4096] [--rounds 5]
"""
import argparse
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402
from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402
from tools.decode_probe import meta_for  # noqa: E402

nq, nkv, BS, D = 32, 8, 64, 128


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=28672)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--grids", default="0,1024,512,256")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    ctx = (torch.randint(3000, 6400, (125,), generator=g)).tolist()
    meta, nb = meta_for(ctx, False, dev, None)
    kc = torch.empty(nb, nkv, BS, D, device=dev, dtype=torch.bfloat16).normal_()
    vc = torch.empty(nb, nkv, D, BS, device=dev, dtype=torch.bfloat16).normal_()
    q = torch.randn(len(ctx), (nq + 2 * nkv) * D, device=dev).bfloat16()
    out = torch.empty(len(ctx), nq * D, device=dev).bfloat16()
    x = (torch.rand(a.m, a.k, device=dev) * 2 - 1).bfloat16()
    ws = [((torch.rand(a.n, a.k, device=dev) * 2 - 1) * 0.02).bfloat16() for _ in range(2)]
    y = torch.empty(a.m, a.n, device=dev).bfloat16()
    s_att, s_gemm = torch.cuda.Stream(), torch.cuda.Stream()
    full = meta.grid_waves or min(A.DECODE_WAVE_SLOTS, meta.n_items * nkv)

    def attn(grid):
        meta.grid_waves = grid or full
        for _ in range(a.reps):
            A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(D), out=out)

    def gemm():
        for i in range(a.reps):
            LIN.lib_gemm(x, ws[i % 2], y)

    def timed(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    def both(grid):
        def run():
            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(cur)
            s_att.wait_event(ev)
            s_gemm.wait_event(ev)
            with torch.cuda.stream(s_att):
                attn(grid)
            with torch.cuda.stream(s_gemm):
                gemm()
            cur.wait_stream(s_att)
            cur.wait_stream(s_gemm)
        return run

    grids = [int(v) for v in a.grids.split(",")]
    arms = {"gemm": gemm}
    for gr in grids:
        arms[f"attn_g{gr or full}"] = lambda gr=gr: attn(gr)
        arms[f"both_g{gr or full}"] = both(gr)
    for fn in arms.values():
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for _ in range(a.rounds):
        for k, fn in arms.items():
            res[k].append(timed(fn))
    med = {k: statistics.median(v) for k, v in res.items()}
    print(f"M={a.m} N={a.n} K={a.k}: gemm alone {med['gemm']:.1f} us per call", flush=True)
    for gr in grids:
        gname = gr or full
        at, bo = med[f"attn_g{gname}"], med[f"both_g{gname}"]
        print(f"  attention grid {gname:5d}: alone {at:7.1f} us   both {bo:7.1f} us   serial sum {at + med['gemm']:7.1f} us"
              f"   overlap saves {100 * (1 - bo / (at + med['gemm'])):5.1f} %", flush=True)


if __name__ == "__main__":
    main()
