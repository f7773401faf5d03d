"""Which HIP / torch operation keeps a native runtime thread busy?

The serving process carries one native thread (created by the HIP runtime,
blocked in KFD's wait-events ioctl between bursts) that burns ~0.7 of a core
in the headline bench (``native_threads.busiest``).  This probe runs one kind
of operation at a time -- eager kernel launches, HIP-graph replays, small
pinned H2D / D2H copies, event record + query / synchronize -- and reports the
CPU seconds every native thread of the process spent in each phase, so the
operation that wakes the thread shows up as the phase where it accumulates.

usage (GPU box): python tools/hip_thread_probe.py [--n 20000]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def native_cpu():
    py = {t.native_id for t in threading.enumerate()}
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for t in os.listdir("/proc/self/task"):
        tid = int(t)
        if tid in py:
            continue
        try:
            with open(f"/proc/self/task/{t}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
            out[tid] = (int(parts[11]) + int(parts[12])) / tick
        except (OSError, ValueError, IndexError):
            pass
    return out


def phase(name, fn, res):
    torch.cuda.synchronize()
    c0, t0 = native_cpu(), time.perf_counter()
    fn()
    torch.cuda.synchronize()
    c1, dt = native_cpu(), time.perf_counter() - t0
    d = sorted(((c1[t] - c0.get(t, 0.0), t) for t in c1), reverse=True)[:2]
    res[name] = {"wall_s": round(dt, 3), "top_native_cpu_s": [round(x, 3) for x, _ in d]}
    print(name, json.dumps(res[name]), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--phases", default="", help="comma list of phase names (default: all)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    x = torch.zeros(1024, device=dev)
    pin = torch.zeros(64, dtype=torch.int32).pin_memory()
    dsmall = torch.zeros(64, dtype=torch.int32, device=dev)
    res = {}
    n = a.n

    def kernels():
        for _ in range(n):
            x.add_(1.0)

    def graph():
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                x.add_(1.0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                x.add_(1.0)
        for _ in range(n // 20):
            g.replay()

    def h2d():
        for _ in range(n // 4):
            dsmall.copy_(pin, non_blocking=True)

    def d2h():
        for _ in range(n // 4):
            pin.copy_(dsmall, non_blocking=True)

    def ev_query():
        for _ in range(n // 4):
            x.add_(1.0)
            e = torch.cuda.Event()
            e.record()
            while not e.query():
                pass

    def ev_sync():
        for _ in range(n // 4):
            x.add_(1.0)
            e = torch.cuda.Event()
            e.record()
            e.synchronize()

    def idle():
        time.sleep(2.0)

    def pin_churn():  # the engine's per-step metadata upload: fresh host tensor -> pin_memory() -> H2D
        for _ in range(n // 10):
            h = torch.arange(256, dtype=torch.int32).pin_memory()
            h.to(dev, non_blocking=True)

    def pageable_h2d():
        for _ in range(n // 10):
            torch.arange(256, dtype=torch.int32).to(dev, non_blocking=True)

    def d2h_event_sync():  # the sampler's token read-back
        for _ in range(n // 10):
            x.add_(1.0)
            pin.copy_(dsmall, non_blocking=True)
            e = torch.cuda.Event()
            e.record()
            e.synchronize()

    side = torch.cuda.Stream(dev)

    def two_streams():  # the graph mirror's own stream, fetches synchronised by events
        for _ in range(n // 10):
            with torch.cuda.stream(side):
                dsmall.add_(1)
                pin.copy_(dsmall, non_blocking=True)
                e = torch.cuda.Event()
                e.record(side)
            x.add_(1.0)
            e.synchronize()

    def item_sync():
        for _ in range(n // 10):
            x.add_(1.0)
            float(x[0].item())

    from k8s_llm_rca_amd.ops import linear as LIN
    from k8s_llm_rca_amd.ops import norm as NRM
    xa = torch.randn(2048, 4096, device=dev).bfloat16()
    wa = torch.randn(4096, 4096, device=dev).bfloat16()

    def lib_gemm():  # the engine's prefill GEMMs (measured dispatch: hipBLASLt / gemm_big)
        for _ in range(n // 40):
            LIN.linear(xa, wa)

    def torch_matmul():
        for _ in range(n // 40):
            torch.matmul(xa, wa.t())

    def lib_norm():
        wn = torch.ones(4096, device=dev).bfloat16()
        xs = xa[:128]
        for _ in range(n // 4):
            NRM.rmsnorm(xs, wn, 1e-5)

    def big_graph():  # a decode-step-sized graph: ~400 kernels
        s2 = torch.cuda.Stream()
        with torch.cuda.stream(s2):
            x.add_(1.0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(400):
                x.add_(1.0)
        for _ in range(n // 400):
            g.replay()

    idx = torch.randint(0, 1024, (4096,), device=dev)

    def index_ops():  # torch kernels that carry a device-side assert (index bounds)
        for _ in range(n // 4):
            x.index_select(0, idx)

    xb = torch.randn(4096, 4096, device=dev).bfloat16()
    wb = torch.randn(28672, 4096, device=dev).bfloat16()

    def big_gemm():  # long hand-written GEMM kernels, few launches (gemm_big: no library call)
        for _ in range(max(1, n // 200)):
            LIN.gemm_big(xb, wb)

    def _queue_gemms(k):
        for _ in range(k):
            LIN.gemm_big(xb, wb)
        e = torch.cuda.Event()
        e.record()
        return e

    def wait_sync():  # a host thread blocked in a HIP wait while the GPU works
        for _ in range(5):
            _queue_gemms(max(1, n // 1000)).synchronize()

    def wait_poll():  # the same work, the host polling the event with short sleeps
        for _ in range(5):
            e = _queue_gemms(max(1, n // 1000))
            while not e.query():
                time.sleep(0.0002)

    def one_matmul():  # a single library GEMM: does it switch the thread on for later work?
        torch.matmul(xa, wa.t())

    def memsets():
        for _ in range(n // 4):
            dsmall.zero_()

    phases = {"idle_2s": idle, "eager_kernels": kernels, "graph_replays": graph, "h2d_pinned": h2d,
              "d2h_pinned": d2h, "event_query": ev_query, "event_sync": ev_sync, "pin_churn": pin_churn,
              "pageable_h2d": pageable_h2d, "d2h_event_sync": d2h_event_sync, "two_streams": two_streams,
              "item_sync": item_sync, "lib_gemm": lib_gemm, "torch_matmul": torch_matmul, "lib_norm": lib_norm,
              "big_graph": big_graph, "memsets": memsets, "index_ops": index_ops, "big_gemm": big_gemm,
              "wait_sync": wait_sync, "wait_poll": wait_poll, "one_matmul": one_matmul}
    # --phases runs the named phases in the given order; "name#k" repeats a phase
    for label in (a.phases.split(",") if a.phases else list(phases)):
        phase(label, phases[label.split("#")[0]], res)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.environ.get("PROBE_OUT", "gpurun_out/hip_thread_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
