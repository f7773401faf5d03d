"""Decode attention beside a prefill GEMM on CU-partitioned HIP streams.

Round 3 (tools/overlap_gemm_attn.py, profiles/r3/overlap/) found that the
HBM-bound decode attention and the MFMA-bound prefill GEMM never co-execute
when both are issued on plain streams: gemm_big's 512-thread workgroups need a
whole CU's register file (8 waves x ~246 VGPRs) and every CU already holds an
attention wave, so the second kernel only starts as the first drains.

This probe partitions the chip instead: the attention stream is created with a
CU mask (hipExtStreamCreateWithCUMask) of 8*m CUs per XCD, the GEMM stream
with the complement (or all CUs), and the two run at once.  The mask bits are
chosen so that the split is per XCD under either bit -> (XCD, CU) mapping
(round-robin or blocked): bit i is in the attention set iff (i // 8) % 4 < m.

Reports, per M and split: attention alone on its share, GEMM alone on its
share, both at once, and the serial full-chip sum -- the saving a two-stream
nano-batched mixed step could reach at that split.

    python tools/coexec_cumask.py [--m 2048,4096] [--rounds 5]
"""
import argparse
import ctypes
import json
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


def hip():
    L = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    L.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                              ctypes.POINTER(ctypes.c_uint32)]
    L.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    return L


def mask_words(n_cu: int, pick) -> list:
    words = [0] * ((n_cu + 31) // 32)
    for i in range(n_cu):
        if pick(i):
            words[i // 32] |= 1 << (i % 32)
    return words


def masked_stream(L, words, dev):
    s = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = L.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    return torch.cuda.ExternalStream(s.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="2048,4096")
    ap.add_argument("--rows", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--splits", default="1,2,3")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    L = hip()
    LIN.reserve_big_ws(dev, enable=False)  # the split tail's workspace belongs to one stream: off for every arm
    g = torch.Generator().manual_seed(0)
    ctx = (torch.randint(4000, 8000, (a.rows,), generator=g)).tolist()
    meta, nb = meta_for(ctx, False, dev, None)
    kc = torch.empty(nb, nkv, BS, D, device=dev, dtype=torch.bfloat16).normal_()
    vc = torch.empty(nb, nkv, D, BS, device=dev, dtype=torch.bfloat16).normal_()
    q = torch.randn(len(ctx), (nq + 2 * nkv) * D, device=dev).bfloat16()
    out = torch.empty(len(ctx), nq * D, device=dev).bfloat16()
    full_grid = meta.grid_waves or min(A.DECODE_WAVE_SLOTS, meta.n_items * nkv)
    N2, K = 2 * 14336, 4096
    ws = [((torch.rand(N2, K, device=dev) * 2 - 1) * 0.02).bfloat16() for _ in range(2)]
    kv_bytes = sum(ctx) * nkv * 2 * D * 2

    def attn(grid):
        meta.grid_waves = grid
        for _ in range(a.reps):
            A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(D), out=out)

    def timed(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    def on(stream, fn):
        def run():
            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(cur)
            stream.wait_event(ev)
            with torch.cuda.stream(stream):
                fn()
            cur.wait_stream(stream)
        return run

    def both(s1, f1, s2, f2):
        def run():
            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(cur)
            s1.wait_event(ev)
            s2.wait_event(ev)
            with torch.cuda.stream(s1):
                f1()
            with torch.cuda.stream(s2):
                f2()
            cur.wait_stream(s1)
            cur.wait_stream(s2)
        return run

    results = []
    full = masked_stream(L, mask_words(n_cu, lambda i: True), dev)
    for M in [int(v) for v in a.m.split(",")]:
        x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        y = torch.empty(M, N2 // 2, device=dev).bfloat16()

        def gemm(x=x, y=y):
            for i in range(a.reps):
                LIN.gemm_big(x, ws[i % 2], y, silu=True)

        # the GEMM split into a part sized to run on the 8 CUs/XCD the attention leaves idle
        # (m = 3) while it streams, and the rest on the whole chip after it
        n1 = 34 * 128  # act columns of part 1 (~30 % of 14336)
        w1 = [((torch.rand(2 * n1, K, device=dev) * 2 - 1) * 0.02).bfloat16() for _ in range(2)]
        w2 = [((torch.rand(N2 - 2 * n1, K, device=dev) * 2 - 1) * 0.02).bfloat16() for _ in range(2)]
        y1 = torch.empty(M, n1, device=dev).bfloat16()
        y2 = torch.empty(M, N2 // 2 - n1, device=dev).bfloat16()

        def gemm1(x=x, y1=y1):
            for i in range(a.reps):
                LIN.gemm_big(x, w1[i % 2], y1, silu=True)

        def gemm2(x=x, y2=y2):
            for i in range(a.reps):
                LIN.gemm_big(x, w2[i % 2], y2, silu=True)

        hi = torch.cuda.Stream(priority=-1)
        arms = {"attn_full": on(full, lambda: attn(full_grid)), "gemm_full": on(full, gemm),
                "both_unmasked": both(full, lambda: attn(full_grid), torch.cuda.Stream(), gemm),
                # the attention on a high-priority stream: its waves are dispatched first as GEMM tiles retire
                "both_attn_high_prio": both(hi, lambda: attn(full_grid), torch.cuda.Stream(), gemm)}
        for m in [int(v) for v in a.splits.split(",")]:
            sa = masked_stream(L, mask_words(n_cu, lambda i, m=m: (i // 8) % 4 < m), dev)
            sg = masked_stream(L, mask_words(n_cu, lambda i, m=m: (i // 8) % 4 >= m), dev)
            share = n_cu * m // 4
            # the attention's persistent grid: 2 waves per SIMD of its share (its VGPR occupancy)
            grid = min(full_grid, share * 8)
            arms[f"attn_m{m}"] = on(sa, lambda grid=grid: attn(grid))
            arms[f"gemm_m{m}"] = on(sg, gemm)
            arms[f"both_m{m}"] = both(sa, lambda grid=grid: attn(grid), sg, gemm)
            arms[f"both_m{m}_gall"] = both(sa, lambda grid=grid: attn(grid), full, gemm)
            if m == 3:
                def split_run(sa=sa, sg=sg, grid=grid):
                    cur = torch.cuda.current_stream()
                    ev = torch.cuda.Event()
                    ev.record(cur)
                    sa.wait_event(ev)
                    sg.wait_event(ev)
                    with torch.cuda.stream(sa):
                        attn(grid)
                    with torch.cuda.stream(sg):
                        gemm1()
                    cur.wait_stream(sa)
                    cur.wait_stream(sg)
                    gemm2()
                arms["split_m3_then_full"] = split_run
        for fn in arms.values():
            fn()
        torch.cuda.synchronize()
        res = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                res[k].append(timed(fn))
        med = {k: statistics.median(v) for k, v in res.items()}
        serial = med["attn_full"] + med["gemm_full"]
        flop = 2.0 * M * N2 * K
        row = {"M": M, "rows": a.rows, "ctx_mean": sum(ctx) / len(ctx), "us": med, "serial_us": serial,
               "attn_full_TBps": kv_bytes / med["attn_full"] / 1e6, "gemm_full_TFs": flop / med["gemm_full"] / 1e6}
        print(f"M={M}: attention alone {med['attn_full']:.1f} us ({row['attn_full_TBps']:.2f} TB/s), "
              f"gate_up gemm_big alone {med['gemm_full']:.1f} us ({row['gemm_full_TFs']:.0f} TFLOP/s), "
              f"serial {serial:.1f} us, both unmasked {med['both_unmasked']:.1f} us, attention on a high-priority "
              f"stream {med['both_attn_high_prio']:.1f} us ({100 * (1 - med['both_attn_high_prio'] / serial):+.1f} %)",
              flush=True)
        for m in [int(v) for v in a.splits.split(",")]:
            bo, bg = med[f"both_m{m}"], med[f"both_m{m}_gall"]
            if m == 3:
                sp = med["split_m3_then_full"]
                print(f"  attention on 24 CUs/XCD + 30 % of the GEMM on the other 8, then the rest on all: {sp:.1f} us "
                      f"({100 * (1 - sp / serial):+.1f} % vs serial)", flush=True)
            print(f"  attention on {8 * m} CUs/XCD: attn {med[f'attn_m{m}']:.1f} us "
                  f"({kv_bytes / med[f'attn_m{m}'] / 1e6:.2f} TB/s), gemm on the rest {med[f'gemm_m{m}']:.1f} us; "
                  f"both {bo:.1f} us ({100 * (1 - bo / serial):+.1f} % vs serial), "
                  f"gemm on all CUs {bg:.1f} us ({100 * (1 - bg / serial):+.1f} %)", flush=True)
        results.append(row)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
