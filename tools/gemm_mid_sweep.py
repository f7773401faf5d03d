"""Decode-regime GEMM sweep: hipBLASLt vs the hand-written kernels at M <= 256.

    python tools/gemm_mid_sweep.py [--model llama3-8b] [--ms 24,32,...] [--emit]

For every projection shape of the model and every M bucket, times hipBLASLt,
the skinny kernel and every applicable gemm_mid variant (cfg x split-K) with
COLD weights (several copies rotated, > 512 MB per shape, as consecutive
layers are), checks each against an fp32 reference, and prints effective
weight-streaming bandwidth.  ``--emit`` writes the engine's dispatch table
(``data/gemm_dispatch_<model>.json``): a hand-written kernel is chosen only
where it beats hipBLASLt by >= 3 %.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402
from tools.tune_gemms import shapes_for  # noqa: E402

BUCKETS = "1,2,4,8,16,24,32,48,64,96,128,160,192,224,256"


def bench(fn, iters=40):
    for _ in range(4):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ms", default=BUCKETS)
    ap.add_argument("--emit", action="store_true")
    ap.add_argument("--margin", type=float, default=0.97)
    ap.add_argument("--out", default=None, help="write the table here instead of data/ (with --emit)")
    a = ap.parse_args()
    L.clear_dispatch()  # time the raw kernels
    ms = [int(m) for m in a.ms.split(",")]
    shapes = shapes_for(a.model, a.tp)
    dev = torch.device("cuda")
    ws = {}
    for s in shapes:
        ncopy = max(2, (512 << 20) // (s[0] * s[1] * 2) + 1)
        ws[s] = [torch.randn(s, dtype=torch.bfloat16, device=dev) * 0.02 for _ in range(ncopy)]
    L.reserve_mid_scratch(dev, 256, max(n for n, _ in shapes))
    ctr = [0]

    def rot(lst):
        ctr[0] += 1
        return lst[ctr[0] % len(lst)]

    table = {f"{n},{k}": [] for n, k in shapes}
    from k8s_llm_rca_amd.models.config import get_config
    mc = get_config(a.model)
    down = (mc.hidden, mc.intermediate // a.tp) if not mc.n_experts else None
    gate_up = (2 * mc.intermediate // a.tp, mc.hidden) if not mc.n_experts else None
    tot, lm, layer_gb = {}, {}, {}
    t0 = time.time()
    for M in ms:
        for (N, K) in shapes:
            wl = ws[(N, K)]
            w = wl[0]
            x = torch.randn(M, K, dtype=torch.bfloat16, device=dev)
            gb = N * K * 2 / 1e9
            ref = x.float() @ w.float().t()
            lib_t = bench(lambda: torch.matmul(x, rot(wl).t()))
            res = {"hipblaslt": lib_t}
            cands = []
            for name, fn in L.candidate_kernels(M, N, K):
                y = fn(x, w)
                err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                if err > 2e-2:
                    print(f"  !! {name} M{M} N{N} K{K} rel err {err:.3e}", flush=True)
                    continue
                cands.append((bench(lambda: fn(x, rot(wl))), name))
            cands.sort()
            for t, n in cands:
                k = ("mid" if n.startswith("mid") else "grp" if n.startswith("grp") else
                     "stream" if n.startswith("stream") else n)
                res.setdefault(k, t)
            best = {"m": M, "kind": "lib", "t_us": round(lib_t, 2), "lib_us": round(lib_t, 2)}
            if cands and cands[0][0] < a.margin * lib_t:
                t, n = cands[0]
                if n == "skinny":
                    best.update(kind="skinny", t_us=round(t, 2))
                elif n.startswith("grp"):
                    best.update(kind="grp", splits=int(n.split("x")[-1]), t_us=round(t, 2))
                elif n.startswith("stream"):
                    best.update(kind="stream", cfg=int(n[6:].split(":")[0]), splits=int(n.split("x")[-1]),
                                t_us=round(t, 2))
                else:
                    cfg, sp = n[3:].split(":")[0], n.split("x")[-1]
                    best.update(kind="mid", cfg=int(cfg), splits=int(sp), t_us=round(t, 2))
            if best["kind"] == "skinny":
                best["kind"] = "lib" if M > 16 else "skinny"  # skinny is the default path for M <= 16
                if best["kind"] == "lib":
                    best["t_us"] = round(lib_t, 2)
            table[f"{N},{K}"].append(best)
            if (N, K) == down:  # SwiGLU-fused down projection vs silu_mul + the best plain GEMM
                from k8s_llm_rca_amd.ops.norm import silu_mul
                gu = torch.randn(M, 2 * K, dtype=torch.bfloat16, device=dev)
                base = bench(lambda: silu_mul(gu)) + best["t_us"]
                ref2 = silu_mul(gu).float() @ w.float().t()
                fc = []
                for name, fn in L.silu_candidates(M, N, K):
                    err = (fn(gu, w).float() - ref2).abs().max().item() / (ref2.abs().max().item() + 1e-6)
                    if err > 2e-2:
                        print(f"  !! silu {name} M{M} rel err {err:.3e}", flush=True)
                        continue
                    fc.append((bench(lambda: fn(gu, rot(wl))), name))
                fc.sort()
                ent = {"m": M, "kind": "unfused", "t_us": round(base, 2)}
                if fc and fc[0][0] < a.margin * base:
                    t, n = fc[0]
                    ent.update(kind="mid", cfg=int(n[3:].split(":")[0]), splits=int(n.split("x")[-1]), t_us=round(t, 2))
                table.setdefault(f"silu:{N},{K}", []).append(ent)
                print(f"      silu+down: unfused {base:7.1f}us  fused best "
                      + (f"{fc[0][1]} {fc[0][0]:.1f}us" if fc else "-") + f" -> {ent['kind']}", flush=True)
                best_t_layer = min(base, fc[0][0] if fc else base)
                tot.setdefault(M, [0.0, 0.0])
                tot[M][1] += best_t_layer - best["t_us"]  # count the down projection as its fused cost
            if (N, K) == gate_up and M <= L.DISPATCH_MAX_M:
                # the SwiGLU epilogue of the stream kernels (one K split) writes act directly:
                # compare it with the plain pick + silu_mul (what the engine runs otherwise)
                from k8s_llm_rca_amd.ops.norm import silu_mul
                gu = torch.randn(M, N, dtype=torch.bfloat16, device=dev)
                base = bench(lambda: silu_mul(gu)) + best["t_us"]
                g_ref, u_ref = ref.split(N // 2, dim=1)
                ref3 = torch.nn.functional.silu(g_ref) * u_ref
                fc = []
                for cfg, sp in L.stream_candidates(M, N, K):
                    if sp != 1:
                        continue
                    fn = lambda xx, ww, cfg=cfg: L.gemm_stream_silu(xx, ww, cfg)
                    err = (fn(x, w).float() - ref3).abs().max().item() / (ref3.abs().max().item() + 1e-6)
                    if err > 3e-2:
                        print(f"  !! stream-silu {cfg} M{M} rel err {err:.3e}", flush=True)
                        continue
                    fc.append((bench(lambda: fn(x, rot(wl))), cfg))
                fc.sort()
                if fc and fc[0][0] < a.margin * base:
                    best.update(kind="stream", cfg=fc[0][1], splits=1, t_us=round(fc[0][0], 2), swiglu_epilogue=True)
                print(f"      gate_up+silu: {best.get('kind')} {base:7.1f}us unfused, stream-silu best "
                      + (f"cfg {fc[0][1]} {fc[0][0]:.1f}us" if fc else "-")
                      + (" -> fused" if best.get("swiglu_epilogue") else " -> unfused"), flush=True)
            line = "  ".join(f"{k} {v:7.1f}us {gb / (v * 1e-6) / 1e3:5.2f}TB/s" for k, v in res.items())
            top = " | ".join(f"{n} {t:.1f}" for t, n in cands[:3])
            print(f"M{M:4d} N{N:6d} K{K:6d}  {line}   [{top}] -> {best['kind']}", flush=True)
            tot.setdefault(M, [0.0, 0.0])
            if N * a.tp >= mc.vocab_size:  # the LM head runs once per step, not per layer
                lm[M] = (lib_t, best["t_us"])
                continue
            tot[M][0] += lib_t
            tot[M][1] += best["t_us"]
            layer_gb[M] = layer_gb.get(M, 0.0) + gb
    for M, (lt, bt) in tot.items():
        print(f"M{M:4d} per-layer sum (qkv+o+gate_up+silu+down): hipblaslt {lt:8.1f}us  dispatch {bt:8.1f}us  "
              f"({lt / bt:.2f}x, weights {layer_gb.get(M, 0) / (bt * 1e-6) / 1e3:4.2f}TB/s)"
              + (f"   lm_head: hipblaslt {lm[M][0]:7.1f}us  dispatch {lm[M][1]:7.1f}us" if M in lm else ""))
    print(f"sweep took {time.time() - t0:.0f}s")
    if a.emit:
        path = a.out or L.dispatch_path(a.model, a.tp)
        with open(path, "w") as f:
            json.dump({"model": a.model, "tp": a.tp, "device": torch.cuda.get_device_name(),
                       "note": "per-M-bucket fastest kernel, cold weights (tools/gemm_mid_sweep.py)",
                       "shapes": table}, f, indent=1)
        print("wrote", path)


if __name__ == "__main__":
    main()
