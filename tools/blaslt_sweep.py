"""Every hipBLASLt solution for the model's projections at a ladder of M
(csrc/kernels/blaslt.hip k8s_blaslt_sweep): heuristic first choice vs the
fastest solution, cold rotated weights.  --emit writes the winners (solution
indices, where they beat the heuristic by > --min-gain) to
data/blaslt_algos_<model>.json, which the engine registers at init
(ops/linear.py load_lib_algos).

    python3 tools/blaslt_sweep.py --model llama3-8b --emit
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402
from k8s_llm_rca_amd.ops._lib import lib, ptr, stream_ptr  # noqa: E402

SHAPES = {"llama3-8b": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ms", default="256,320,384,448,512,640,768,1024,1536,2048,3072,4096")
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--min-gain", type=float, default=1.03)
    ap.add_argument("--emit", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    L.reserve_lib_workspace(dev)
    ws = L._blaslt_ws[dev]
    table = {}
    tot_h = tot_b = 0.0
    for N, K in SHAPES[a.model]:
        nw = max(2, min(16, int(1.2e9 // (N * K * 2))))
        w = torch.randn(nw, N, K, device=dev).bfloat16()
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            idx = (ctypes.c_int * 4)()
            us = (ctypes.c_float * 4)()
            times = (ctypes.c_float * 1)()
            n = lib().k8s_blaslt_sweep(ptr(x), K, ptr(w), nw, N * K, ptr(y), N, M, N, K, ptr(ws), L.BLASLT_WS_BYTES,
                                       a.iters, stream_ptr(x), 4, idx, us, times)
            if n <= 0:
                print(f"M {M} N {N} K {K}: sweep failed {n}", flush=True)
                continue
            h = times[0]
            gain = h / us[0] if us[0] > 0 else 0
            tot_h += h
            tot_b += min(h, us[0])
            tf = 2 * M * N * K / us[0] / 1e6
            print(f"M {M:5d} N {N:6d} K {K:6d}  heuristic {h:7.1f}us  best {us[0]:7.1f}us ({gain:4.2f}x, {tf:5.0f} TF)"
                  f"  idx {idx[0]}  next {[round(us[i], 1) for i in range(1, n)]}", flush=True)
            if gain > a.min_gain:
                table.setdefault(f"{N},{K}", {})[str(M)] = int(idx[0])
            del x, y
        del w
    print(f"total heuristic {tot_h:.1f} us  best {tot_b:.1f} us", flush=True)
    if a.emit:
        path = os.path.join(L.DATA_DIR, f"blaslt_algos_{a.model}.json")
        with open(path, "w") as f:
            json.dump({"model": a.model, "note": "tools/blaslt_sweep.py: hipBLASLt solution index per (N,K) per "
                       "ladder M (used from that M up to the next ladder point)", "algos": table}, f, indent=1)
        print("wrote", path)


if __name__ == "__main__":
    main()
