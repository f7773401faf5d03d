"""A/B of the TP push epilogue on the tp-sim loopback (one GPU, world 8).

For Llama-3-70B TP=8 rank shapes (o: N = 8192, K = 1024; down: K = 3584) at
decode batch sizes, times the row-parallel output + all-reduce + residual add +
RMSNorm both ways, interleaved, with the dispatch table's GEMM choice:
  staged (pull): stream GEMM -> y, then the fused addnorm (stage y into the own
                 slot, flag, read every rank's slot);
  push:          the stream GEMM stores into every rank's slot (one-shot) or the
                 owner's (two-shot) + per-strip flags, then the consumer sums its
                 local slots.
Loopback = the real kernels moving the real bytes over local HBM, waits skipped:
a stand-in, not xGMI.  Also times the GEMM alone, so the collective's
share of each pair can be read off.

usage (GPU box): python tools/push_ab.py [--ms 16,32,64,128,192,256] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402
from k8s_llm_rca_amd.ops._lib import stream_ptr  # noqa: E402
from k8s_llm_rca_amd.parallel.tpsim import LoopbackAR  # noqa: E402
from k8s_llm_rca_amd.parallel.xgmi import ONE_SHOT_MAX  # noqa: E402


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
    ap.add_argument("--ms", default="16,32,64,128,192,256")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    car = LoopbackAR(a.world, 64 << 20)
    H = 8192
    assert LIN.load_dispatch(LIN.dispatch_path("llama3-70b", 8)), "70B TP=8 dispatch table"
    rows = []
    for name, K in (("o", 1024), ("down", 3584)):
        w = torch.randn(H, K, device=dev).bfloat16()
        nw = torch.ones(H, device=dev).bfloat16()
        for M in (int(m) for m in a.ms.split(",")):
            kind, cfg, splits = LIN.select_gemm(M, H, K)
            mode = 1 if M * H * 2 <= ONE_SHOT_MAX else 2
            if kind != LIN.KIND_STREAM or not car.push_ok(H, M, mode) or (splits == 1 and cfg < 13):
                print(json.dumps({"shape": name, "M": M, "skip": f"kind {kind} cfg {cfg}"}), flush=True)
                continue
            x = torch.randn(M, K, device=dev).bfloat16()
            res = torch.randn(M, H, device=dev).bfloat16()
            y = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
            out = torch.empty(M, H, device=dev, dtype=torch.bfloat16)

            def pull():
                LIN.gemm_stream(x, w, cfg, splits, out)
                car.addnorm(out, res, nw, y, 1e-5, mode)

            def push():
                car.linear_push_addnorm(x, w, res, nw, y, 1e-5, cfg, splits, mode)

            def gemm():
                LIN.gemm_stream(x, w, cfg, splits, out)

            part = LIN._scratch(dev, splits * M * H).data_ptr() if splits > 1 else None
            S = H // (128 if (splits == 1 and cfg > 20) else 64)

            def producer():  # loopback: no waits, the epoch only moves with a consumer
                car.L.k8s_gemm_stream_push(x.data_ptr(), K, w.data_ptr(), M, H, K, cfg, splits, part, car.id, mode,
                                           stream_ptr(x))

            def consumer():
                car.L.k8s_ar_push_addnorm_bf16(car.id, res.data_ptr(), nw.data_ptr(), y.data_ptr(), M, H, 1e-5,
                                               mode, S, stream_ptr(x))

            def staged_an():
                car.addnorm(out, res, nw, y, 1e-5, mode)
            fns = (("pull", pull), ("push", push), ("gemm", gemm), ("producer", producer), ("consumer", consumer),
                   ("addnorm", staged_an))
            t = {k: [] for k, _ in fns}
            for _ in range(a.rounds):
                for k, fn in fns:
                    t[k].append(timed(fn, a.iters))
            med = {k: round(statistics.median(v), 2) for k, v in t.items()}
            line = {"shape": name, "M": M, "cfg": cfg, "splits": splits, "mode": mode,
                    "us_pull_pair": med["pull"], "us_push_pair": med["push"], "us_gemm_alone": med["gemm"],
                    "us_push_gemm_alone": med["producer"], "us_push_consumer_alone": med["consumer"],
                    "us_staged_addnorm_alone": med["addnorm"], "us_saved": round(med["pull"] - med["push"], 2)}
            rows.append(line)
            print(json.dumps(line), flush=True)
    car.close()
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "push_ab.jsonl")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
