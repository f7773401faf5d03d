"""Per-thread CPU time of a bench run (where the host's GIL time goes).

    python tools/thread_cpu.py [bench args...]

Runs the bench in-process and, at exit, prints user+system CPU seconds per
thread name group (engine loop vs pipeline workers vs torch/HIP runtime
threads) next to the wall time, from psutil's per-thread counters.
"""
import collections
import os
import sys
import threading
import time

import psutil

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from k8s_llm_rca_amd.bench import rca_bench
    proc = psutil.Process()
    names = {}
    cpu = {}
    stop = threading.Event()

    def sample():
        for th in proc.threads():
            cpu[th.id] = th.user_time + th.system_time

    def watch():  # names and CPU by native id (pipeline threads come and go)
        while not stop.is_set():
            for t in threading.enumerate():
                if t.native_id:
                    names[t.native_id] = t.name
            sample()
            time.sleep(0.2)

    threading.Thread(target=watch, daemon=True, name="watch").start()
    t0 = time.perf_counter()
    rc = rca_bench.main(sys.argv[1:])
    wall = time.perf_counter() - t0
    stop.set()
    sample()
    groups = collections.defaultdict(lambda: [0.0, 0])
    for tid, c in cpu.items():
        n = names.get(tid, "native")
        key = n.split("-")[0].split(" ")[0].rstrip("0123456789_") or n
        groups[key][0] += c
        groups[key][1] += 1
    print(f"wall {wall:.1f} s; process cpu {sum(v[0] for v in groups.values()):.1f} s", file=sys.stderr)
    for k, (cpu, n) in sorted(groups.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:24s} {n:5d} threads {cpu:8.2f} s cpu", file=sys.stderr)
    return rc


if __name__ == "__main__":
    sys.exit(main())
