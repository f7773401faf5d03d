"""xGMI all-reduce kernel cost on ONE GPU (loopback communicator, parallel/tpsim.py).

Times the one-shot / two-shot kernels at the TP decode message sizes with the
waits skipped: what is left is the kernel's own cost -- staging, the publish
(fences + flag stores), the peer-slot reads -- over local uncached memory.
``K8SRCA_AR_FENCE_ALL`` A/B (a system fence in every wave vs one per block),
interleaved rounds in one process.

    python tools/ar_probe.py [--world 8] [--reps 50]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from k8s_llm_rca_amd.knobs import KNOBS, set_knob  # noqa: E402

from k8s_llm_rca_amd.parallel.tpsim import LoopbackAR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    car = LoopbackAR(a.world, 8 << 20)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # a GEMM-sized dirty footprint in L2 before each call, as in a decode layer
    dirty = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    print(f"world {a.world}; us per call (median of {a.rounds} rounds x {a.reps} reps)")
    print(f"{'bytes':>9} {'mode':>4} {'fence1':>8} {'fence_all':>9} {'fence1+dirty':>12}")
    for nb in (16 << 10, 64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20):
        t = torch.zeros(nb // 2, dtype=torch.bfloat16, device="cuda")
        mode = car.mode_for(t)
        res = {"0": [], "1": [], "d": []}
        for _ in range(a.rounds):
            for fa in ("0", "1", "d"):
                set_knob("ar_fence_all", fa == "1")
                for _ in range(3):
                    car(t, mode)
                torch.cuda.synchronize()
                if fa == "d":
                    tot = 0.0
                    for _ in range(a.reps):
                        dirty.fill_(1)
                        e0.record()
                        car(t, mode)
                        e1.record()
                        e1.synchronize()
                        tot += e0.elapsed_time(e1)
                    res[fa].append(tot * 1e3 / a.reps)
                    continue
                e0.record()
                for _ in range(a.reps):
                    car(t, mode)
                e1.record()
                e1.synchronize()
                res[fa].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        med = {k: statistics.median(v) for k, v in res.items()}
        print(f"{nb:>9} {mode:>4} {med['0']:>8.1f} {med['1']:>9.1f} {med['d']:>12.1f}", flush=True)
    set_knob("ar_fence_all", False)
    car.close()


if __name__ == "__main__":
    main()
