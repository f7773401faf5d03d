"""A/B of the prefill-size GEMM (csrc/kernels/gemm_big.hip) against hipBLASLt.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), random
operands, cold weights (one copy per layer of the model cycled through, like the
engine's per-layer weights), Llama-3-8B projection shapes.  Prints per (shape, M)
the median us and TFLOP/s of each arm, and for gate_up the SwiGLU-fused arm vs
hipBLASLt + silu_mul.

usage: python tools/big_gemm_ab.py [--ms 512,1024,...] [--rounds 5] [--layers 4] [--splits 2,4]
                                   [--emit data/gemm_big_llama3-8b.json]

``--emit`` writes the dispatch ranges the engine loads (ops/linear.py
load_big): per (N, K) the M ranges where the best gemm_big arm (any K split)
is within ``--margin`` of hipBLASLt (default -0.03: ties within 3 % go to the
in-tree kernel), and for gate_up the SwiGLU arm vs hipBLASLt + silu_mul; a
range reaches halfway to the next measured M (the last one is open).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402
from k8s_llm_rca_amd.ops import norm as NRM  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="512,1024,1536,2048,3072,3584,4096,6144,8192")
    ap.add_argument("--shapes", default="qkv,o,gu,down")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--pipes", default="1,5")
    ap.add_argument("--out", default="")
    ap.add_argument("--splits", default="2,4", help="K splits tried for the plain form ('' = none)")
    ap.add_argument("--emit", default="")
    ap.add_argument("--margin", type=float, default=-0.03)
    ap.add_argument("--model", default="llama3-8b", help="projection shapes of this preset (per TP rank)")
    ap.add_argument("--tp", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda")
    from k8s_llm_rca_amd.models.config import get_config
    mc = get_config(a.model)
    H, I, tp = mc.hidden, mc.intermediate // a.tp, a.tp
    nq, nkv = mc.n_heads // tp, max(1, mc.n_kv_heads // tp)
    shapes = {"qkv": ((nq + 2 * nkv) * mc.head_dim, H), "o": (H, nq * mc.head_dim), "gu": (2 * I, H), "down": (H, I)}
    pipes = [int(p) for p in a.pipes.split(",")]
    rows = []
    for name in a.shapes.split(","):
        N, K = shapes[name]
        ws = [(torch.rand(N, K, device=dev) * 2 - 1).mul_(0.02).bfloat16() for _ in range(a.layers)]
        for M in (int(m) for m in a.ms.split(",")):
            x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            arms = {"blaslt": lambda i: LIN.lib_gemm(x, ws[i % a.layers], y)}
            for p in pipes:
                arms[f"big{p}"] = lambda i, p=p: LIN.gemm_big(x, ws[i % a.layers], y, pipe=p)
            for sp in (int(v) for v in a.splits.split(",") if v):
                tiles = -(-M // 256) * (N // 256)
                if LIN.big_shape_ok(M, N, K, splits=sp) and tiles < 256:
                    arms[f"big{pipes[0]}s{sp}"] = lambda i, sp=sp: LIN.gemm_big(x, ws[i % a.layers], y, pipe=pipes[0],
                                                                                splits=sp)
            if name == "qkv":  # the RoPE + paged KV-write epilogue vs hipBLASLt + k8s_rope_kv
                from k8s_llm_rca_amd.ops import attention as A
                BS = 64
                cs = A.rope_cos_sin(8192, 500000.0, device=dev)
                pos = torch.arange(M, device=dev, dtype=torch.int32) % 8192
                slots = torch.arange(M, device=dev, dtype=torch.int32)
                nb = (M + BS - 1) // BS
                kc = torch.empty(nb, nkv, BS, 128, device=dev, dtype=torch.bfloat16)
                vc = torch.empty(nb, nkv, 128, BS, device=dev, dtype=torch.bfloat16)
                arms["blaslt+rope"] = lambda i: A.rope_kv_write(LIN.lib_gemm(x, ws[i % a.layers], y), pos, cs, slots,
                                                                 kc, vc, nq, nkv)
                for p in pipes:
                    arms[f"big{p}_rope"] = lambda i, p=p: LIN.gemm_big_rope(x, ws[i % a.layers], pos, cs, slots, kc,
                                                                            vc, nq, nkv, out=y, pipe=p)
            if name == "gu":
                act = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
                arms["blaslt+silu"] = lambda i: NRM.silu_mul(LIN.lib_gemm(x, ws[i % a.layers], y), out=act)
                for p in pipes:
                    arms[f"big{p}_silu"] = lambda i, p=p: LIN.gemm_big(x, ws[i % a.layers], act, silu=True, pipe=p)
            for fn in arms.values():  # warm-up (heuristics, code objects)
                fn(0)
            torch.cuda.synchronize()
            res = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    res[k].append(timed(fn, a.iters))
            flop = 2.0 * M * N * K
            line = {"shape": name, "M": M, "N": N, "K": K}
            for k, v in res.items():
                med = statistics.median(v)
                line[k] = round(med, 1)
                line[k + "_tf"] = round(flop / med / 1e6, 0)
            rows.append(line)
            print(json.dumps(line), flush=True)
            del x, y
        del ws
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    if a.emit:
        emit(rows, a.emit, a.margin)


def emit(rows, path, margin):
    """Dispatch ranges from the measured rows (module docstring)."""
    out = {"source": "tools/big_gemm_ab.py", "ranges": {}, "silu": {}, "rope": {}}
    by = {}
    for r in rows:
        by.setdefault(r["shape"], []).append(r)
    for shape, rs in by.items():
        rs.sort(key=lambda r: r["M"])
        key = f'{rs[0]["N"]},{rs[0]["K"]}'
        for tag, base, pref in (("ranges", "blaslt", "big"), ("silu", "blaslt+silu", "big"),
                                ("rope", "blaslt+rope", "big")):
            if (tag == "silu" and shape != "gu") or (tag == "rope" and shape != "qkv"):
                continue
            picks = []
            for r in rs:
                suf = {"silu": "_silu", "rope": "_rope"}.get(tag)
                arms = [k for k in r if k.startswith(pref) and not k.endswith("_tf")
                        and (k.endswith(suf) if suf else not (k.endswith("_silu") or k.endswith("_rope")))]
                if not arms or base not in r:
                    picks.append(None)
                    continue
                best = min(arms, key=lambda k: r[k])
                sp = int(best.split("s")[-1]) if "s" in best[3:] and tag == "ranges" else 1
                picks.append(sp if r[best] <= r[base] * (1 - margin) else None)
            ranges = []
            for i, (r, sp) in enumerate(zip(rs, picks)):
                if sp is None:
                    continue
                lo = 257 if i == 0 else (rs[i - 1]["M"] + r["M"]) // 2 + 1
                hi = (r["M"] + rs[i + 1]["M"]) // 2 if i + 1 < len(rs) else 1 << 20
                if ranges and ranges[-1][2] == sp and ranges[-1][1] + 1 == lo:
                    ranges[-1][1] = hi
                else:
                    ranges.append([lo, hi, sp])
            if ranges:
                out[tag][key] = ranges
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("emitted", path, json.dumps(out))


if __name__ == "__main__":
    main()
