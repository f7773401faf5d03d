"""Microbenchmarks of the hot kernels at the RCA workload's shapes (Llama-3-8B).

Prints achieved HBM bandwidth / TFLOP/s per kernel so kernel work can be
prioritised from measurements (run on the GPU box).
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from k8s_llm_rca_amd.knobs import KNOBS, set_knob  # noqa: E402
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402
from k8s_llm_rca_amd.ops import norm as N  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def make_meta(ctx, qlen, nq, nkv, BS, dev, decode, part_size=None):
    S = len(ctx)
    nbs = [(c + BS - 1) // BS for c in ctx]
    maxb = max(nbs)
    perm = torch.randperm(sum(nbs))
    bt = torch.zeros(S, maxb, dtype=torch.int32)
    u = 0
    for s, nb in enumerate(nbs):
        bt[s, :nb] = perm[u:u + nb].int()
        u += nb
    qs = [0]
    for l in qlen:
        qs.append(qs[-1] + l)
    meta = A.AttnMeta(block_tables=bt.to(dev), ctx_lens=torch.tensor(ctx, dtype=torch.int32, device=dev),
                      q_start=torch.tensor(qs, dtype=torch.int32, device=dev), num_seqs=S, decode=decode)
    if decode:
        A.attach_decode_plan(meta, ctx, nq, nkv, BS, dev, part=part_size)
    else:
        A.attach_plan(meta, A.plan_prefill(qs, nq // nkv, BS, list(ctx), nkv=nkv), dev)
    return meta, sum(nbs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all")
    ap.add_argument("--trace", default="profiles/r1_shape_trace_128.jsonl")
    ap.add_argument("--samples", type=int, default=80)
    ap.add_argument("--variants", default="", help="replay: comma list of planner variants (default all)")
    ap.add_argument("--pf-ab", type=int, default=1, help="replay: time the prefill with every kernel of --pf-kinds")
    ap.add_argument("--pf-steps-out", default="", help="replay: per-step prefill timings (JSON lines) to this file")
    ap.add_argument("--pf-targets", default="", help="replay: comma list of prefill split targets (workgroups) to A/B")
    ap.add_argument("--pf-kinds", default="1,0", help="K8SRCA_PF_W8 values to A/B (2 w8, 4 w8 explicit schedule, 0 pg64)")
    args = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    nq, nkv, BS, H, I = 32, 8, 64, 4096, 14336
    res = {}
    if args.what in ("all", "attn"):
        for B, ctxv, ps in [(64, 3400, 256), (64, 3400, 512), (16, 3400, 256), (128, 2000, 256), (64, 800, 256)]:
            ctx = [ctxv] * B
            meta, nb = make_meta(ctx, [1] * B, nq, nkv, BS, dev, True, ps)
            kc = torch.randn(nb, nkv, BS, 128, device=dev).bfloat16()
            vc = torch.randn(nb, nkv, 128, BS, device=dev).bfloat16()
            q = torch.randn(B, (nq + 2 * nkv) * 128, device=dev).bfloat16()
            out = torch.empty(B, nq * 128, device=dev).bfloat16()
            us = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out))
            byts = B * ctxv * nkv * 128 * 2 * 2
            res[f"decode B{B} ctx{ctxv} part{ps}"] = f"{us:.1f}us {byts / us / 1e6:.2f} TB/s"
        # TLB reach: same work, pages scattered over a huge pool (as in the engine's 240 GB pool)
        for pool_gb in (4, 64, 160):
            B, ctxv = 128, 2000
            nb_needed = B * ((ctxv + BS - 1) // BS)
            nb_pool = max(nb_needed, int(pool_gb * 2**30 // (nkv * BS * 128 * 2 * 2)))
            kc = torch.empty(nb_pool, nkv, BS, 128, device=dev, dtype=torch.bfloat16)
            vc = torch.empty(nb_pool, nkv, 128, BS, device=dev, dtype=torch.bfloat16)
            sel = torch.randperm(nb_pool)[:nb_needed]
            kc[sel.to(dev)] = torch.randn(nb_needed, nkv, BS, 128, device=dev).bfloat16()
            vc[sel.to(dev)] = torch.randn(nb_needed, nkv, 128, BS, device=dev).bfloat16()
            meta, _ = make_meta([ctxv] * B, [1] * B, nq, nkv, BS, dev, True, 512)
            meta.block_tables = sel.view(B, -1).int().to(dev)
            q = torch.randn(B, (nq + 2 * nkv) * 128, device=dev).bfloat16()
            out = torch.empty(B, nq * 128, device=dev).bfloat16()
            us = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out))
            res[f"decode B{B} ctx{ctxv} pool{pool_gb}GB"] = f"{us:.1f}us {B * ctxv * nkv * 512 / us / 1e6:.2f} TB/s"
            del kc, vc
            torch.cuda.empty_cache()
        cases = [(512, 3000, 8, 512), (2048, 2048, 2, 512), (64, 3000, 64, 512)]
        cases += [(T, c, S, tw) for (T, c, S) in [(4, 3000, 16), (300, 3000, 2), (600, 3500, 1), (48, 3000, 4)]
                  for tw in (512, 1024, 2048)]
        for T, ctxv, S, tw in cases:
            A.PF_TARGET_WGS = tw
            ctx = [ctxv] * S
            meta, nb = make_meta(ctx, [T] * S, nq, nkv, BS, dev, False)
            kc = torch.randn(nb, nkv, BS, 128, device=dev).bfloat16()
            vc = torch.randn(nb, nkv, 128, BS, device=dev).bfloat16()
            q = torch.randn(T * S, (nq + 2 * nkv) * 128, device=dev).bfloat16()
            out = torch.empty(T * S, nq * 128, device=dev).bfloat16()
            us = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out), iters=10)
            # causal-ish flops: each query attends to (ctx - T + i) keys
            pairs = S * sum(ctxv - T + i + 1 for i in range(T))
            fl = pairs * nq * 128 * 4
            kvb = S * ctxv * nkv * 128 * 2 * 2
            res[f"prefill S{S} q{T} ctx{ctxv} tw{tw} merge{meta.n_merge}"] = \
                f"{us:.1f}us {fl / us / 1e6:.1f} TFLOP/s {kvb / us / 1e6:.2f} TB/s-kv"
        A.PF_TARGET_WGS = 512
    if args.what == "replay":
        # replay the attention shapes of a recorded run (K8S_RCA_SHAPE_TRACE)
        steps = [json.loads(l) for l in open(args.trace)]
        rng = torch.Generator().manual_seed(0)
        dec = [s["d"] for s in steps if s["d"]]
        pre = [s["p"] for s in steps if s["p"]]
        idx = torch.randperm(len(dec), generator=rng)[: args.samples].tolist()
        tot_us = tot_bytes = 0.0
        variants = {"plan_v1": "v1", "plan_makespan": "makespan", "makespan_o128": "makespan:128",
                    "makespan_o512": "makespan:512", "makespan_o64": "makespan:64"}
        if args.variants:
            variants = {k: v for k, v in variants.items() if k in args.variants.split(",")}

        buckets = [(1, 16), (17, 48), (49, 96), (97, 256)]
        for name, fn in variants.items():
            agg = {b: [0.0, 0.0, 0] for b in buckets}
            for n_done, i in enumerate(idx):
                if n_done % 20 == 0:
                    print(f"# decode replay {name} {n_done}/{len(idx)}", flush=True)
                ctx = dec[i]
                B = len(ctx)
                ovh0 = A.DECODE_ITEM_OVERHEAD
                if isinstance(fn, str):
                    A.set_decode_planner(fn.split(":")[0])
                    if ":" in fn:
                        A.DECODE_ITEM_OVERHEAD = int(fn.split(":")[1])
                meta, nb = make_meta(ctx, [1] * B, nq, nkv, BS, dev, True,
                                     part_size=None if isinstance(fn, str) else fn)
                A.set_decode_planner("makespan")
                A.DECODE_ITEM_OVERHEAD = ovh0
                kc = torch.empty(nb, nkv, BS, 128, device=dev, dtype=torch.bfloat16).normal_()
                vc = torch.empty(nb, nkv, 128, BS, device=dev, dtype=torch.bfloat16).normal_()
                q = torch.randn(B, (nq + 2 * nkv) * 128, device=dev).bfloat16()
                out = torch.empty(B, nq * 128, device=dev).bfloat16()
                us = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out),
                            iters=10, warm=2)
                b = next(bb for bb in buckets if bb[0] <= B <= bb[1])
                agg[b][0] += us
                agg[b][1] += sum(ctx) * nkv * 512
                agg[b][2] += 1
            tu = sum(v[0] for v in agg.values())
            tb = sum(v[1] for v in agg.values())
            res[f"replay decode {name} all"] = f"{tu / len(idx):.1f}us/step {tb / tu / 1e6:.2f} TB/s"
            for b, (u, by, n) in agg.items():
                if n:
                    res[f"replay decode {name} B{b[0]}-{b[1]}"] = f"n={n} {u / n:.1f}us/step {by / u / 1e6:.2f} TB/s"
        # prefill: the 8-wave LDS-DMA kernel (K8SRCA_PF_W8=1) and the 4-wave pg64
        # kernel interleaved per recorded step (same process, same data)
        kinds0 = tuple(args.pf_kinds.split(",")) if args.pf_ab else (str(KNOBS.pf_w8),)
        pf_ovh0, pf_all0 = A.PF_OVERHEAD_PAGES, A.PF_MAKESPAN_ALL  # the planner defaults (arms without "@")
        targets = [int(t) for t in args.pf_targets.split(",")] if args.pf_targets else [A.PF_TARGET_WGS]
        # arms: (kernel kind, planner split target in workgroups); the label keeps the old form for one target
        kinds = tuple(k if len(targets) == 1 else f"{k}@{t}" for t in targets for k in kinds0)
        tot = {k: 0.0 for k in kinds}
        per_step = {}
        fl = 0.0
        idx = torch.randperm(len(pre), generator=rng)[: args.samples].tolist()
        for n_done, i in enumerate(idx):
            if n_done % 10 == 0:
                print(f"# prefill replay {n_done}/{len(idx)}", flush=True)  # a long replay never looks hung
            ctx = [c for c, q in pre[i]]
            ql = [q for c, q in pre[i]]
            T = sum(ql)
            for k in kinds:
                set_knob("pf_w8", k.split("@")[0].rstrip("m"))
                # "<kind>m": the 2-dims-per-lane merge kernel (K8SRCA_PF_MERGE16=0)
                set_knob("pf_merge16", not k.split("@")[0].endswith("m"))
                arm = k.split("@")[1] if "@" in k else None
                # "@o<pages>": makespan split choice everywhere; "@h<pages>": only where the
                # fixed-target rule would split; "@<n>": fixed target of n workgroups
                A.PF_OVERHEAD_PAGES = float(arm[1:]) if arm and arm[0] in "oh" else (0.0 if arm else pf_ovh0)
                A.PF_MAKESPAN_ALL = bool(arm and arm[0] == "o") or (pf_all0 and not arm)
                A.PF_TARGET_WGS = int(arm) if arm and arm[0] not in "oh" else targets[0]
                torch.manual_seed(i)
                meta, nb = make_meta(ctx, ql, nq, nkv, BS, dev, False)
                if k == kinds[0]:
                    kc = torch.empty(nb, nkv, BS, 128, device=dev, dtype=torch.bfloat16).normal_()
                    vc = torch.empty(nb, nkv, 128, BS, device=dev, dtype=torch.bfloat16).normal_()
                    q = torch.randn(T, (nq + 2 * nkv) * 128, device=dev).bfloat16()
                    out = torch.empty(T, nq * 128, device=dev).bfloat16()
                us_k = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out),
                              iters=10, warm=2)
                tot[k] += us_k
                per_step.setdefault(i, {"T": T, "n": len(ql), "maxq": max(ql), "ctx": sum(ctx)})[k] = round(us_k, 1)
                per_step[i][f"tiles{k}"] = meta.n_tiles
            fl += sum(sum(c - qq + j + 1 for j in range(qq)) for c, qq in zip(ctx, ql)) * nq * 128 * 4
        for k in kinds:
            res[f"replay prefill {len(idx)} steps PF_W8={k}"] = (f"{tot[k] / len(idx):.1f}us/step "
                                                               f"{fl / tot[k] / 1e6:.1f} TFLOP/s")
        set_knob("pf_w8", kinds0[0])
        A.PF_TARGET_WGS = targets[0]
        A.PF_OVERHEAD_PAGES, A.PF_MAKESPAN_ALL = pf_ovh0, pf_all0
        if args.pf_steps_out:
            with open(args.pf_steps_out, "w") as f:
                for v in per_step.values():
                    f.write(json.dumps(v) + "\n")
    if args.what == "moe":
        from k8s_llm_rca_amd.ops import moe as MO
        E, H, I = 8, 4096, 14336
        w13 = (torch.randn(E, 2 * I, H, device=dev) * 0.02).bfloat16()
        w2 = (torch.randn(E, H, I, device=dev) * 0.02).bfloat16()
        for rows in (16, 64, 256, 1024, 8192):
            counts = torch.full((E,), rows // E)
            counts[: rows % E] += 1
            offs = torch.zeros(E + 1, dtype=torch.int32)
            offs[1:] = torch.cumsum(counts, 0)
            offs_d = offs.to(dev)
            x = torch.randn(rows, H, device=dev).bfloat16()
            gu = torch.randn(rows, 2 * I, device=dev).bfloat16()
            o = offs.tolist()

            def loop():
                for e in range(E):
                    if o[e + 1] > o[e]:
                        g = torch.nn.functional.linear(x[o[e]:o[e + 1]], w13[e])
                        torch.nn.functional.linear(g[:, :I], w2[e])

            us_g = timeit(lambda: (MO.grouped_gemm(x, w13, offs_d), MO.grouped_gemm(gu, w2, offs_d, fuse_silu=True)),
                          iters=10)
            us_l = timeit(loop, iters=10)
            wbytes = (w13.numel() + w2.numel()) * 2
            fl = 2 * rows * 3 * I * H
            res[f"moe rows{rows}"] = (f"grouped {us_g:.0f}us ({wbytes / us_g / 1e6:.2f} TB/s-w, "
                                      f"{fl / us_g / 1e6:.0f} TF) | hipBLASLt loop {us_l:.0f}us")
    if args.what == "moe_split":  # each grouped projection alone; down fused vs silu_mul + unfused
        from k8s_llm_rca_amd.ops import moe as MO
        from k8s_llm_rca_amd.ops import norm as NO
        E, H, I = 8, 4096, 14336
        w13 = (torch.randn(E, 2 * I, H, device=dev) * 0.02).bfloat16()
        w2 = (torch.randn(E, H, I, device=dev) * 0.02).bfloat16()
        for rows in (16, 64, 128, 256, 512, 1024, 2048):
            counts = torch.full((E,), rows // E)
            counts[: rows % E] += 1
            offs = torch.zeros(E + 1, dtype=torch.int32)
            offs[1:] = torch.cumsum(counts, 0)
            offs_d = offs.to(dev)
            x = torch.randn(rows, H, device=dev).bfloat16()
            gu = torch.randn(rows, 2 * I, device=dev).bfloat16()
            act = NO.silu_mul(gu)
            t13 = timeit(lambda: MO.grouped_gemm(x, w13, offs_d), iters=10)
            t2f = timeit(lambda: MO.grouped_gemm(gu, w2, offs_d, fuse_silu=True), iters=10)
            t2u = timeit(lambda: MO.grouped_gemm(act, w2, offs_d), iters=10)
            tsl = timeit(lambda: NO.silu_mul(gu), iters=10)
            sp = {z: timeit(lambda: MO.grouped_gemm(act, w2, offs_d, splits=z), iters=10) for z in (2, 4, 8)}
            sp13 = {z: timeit(lambda: MO.grouped_gemm(x, w13, offs_d, splits=z), iters=10) for z in (2, 4)}
            res[f"moe_split rows{rows}"] = (
                f"w13 {t13:.0f}us ({w13.numel() * 2 / t13 / 1e6:.2f} TB/s) "
                + " ".join(f"x{z} {t:.0f}" for z, t in sp13.items())
                + f" | w2 fused {t2f:.0f}us | silu {tsl:.0f}us + w2 {t2u:.0f}us "
                f"({w2.numel() * 2 / t2u / 1e6:.2f} TB/s) " + " ".join(f"x{z} {t:.0f}" for z, t in sp.items()))
    if args.what == "moe_glds":  # Mixtral expert GEMMs: grouped kernel vs the LDS-DMA strip kernel
        from k8s_llm_rca_amd.ops import moe as MO
        E, H, I = 8, 4096, 14336
        w13 = (torch.randn(E, 2 * I, H, device=dev) * 0.02).bfloat16()
        w2 = (torch.randn(E, H, I, device=dev) * 0.02).bfloat16()
        for rows in (64, 128, 250, 512):
            g = torch.Generator().manual_seed(rows)
            counts = torch.bincount(torch.randint(0, E, (rows,), generator=g), minlength=E)
            offs = torch.zeros(E + 1, dtype=torch.int32)
            offs[1:] = torch.cumsum(counts, 0)
            offs_d = offs.to(dev)
            x = torch.randn(rows, H, device=dev).bfloat16()
            act = torch.randn(rows, I, device=dev).bfloat16()
            ref13, ref2 = MO.grouped_gemm(x, w13, offs_d), MO.grouped_gemm(act, w2, offs_d, splits=2)
            line = []
            for name, wt, inp, ref, base in (("w13", w13, x, ref13, dict()), ("w2", w2, act, ref2, dict(splits=2))):
                tb = timeit(lambda: MO.grouped_gemm(inp, wt, offs_d, **base), iters=10)
                best = (tb, "grouped")
                for cfg in (13, 14, 15, 16):
                    for z in (1, 2, 4):
                        if (wt.shape[2] // z) % 64:
                            continue
                        y = MO.grouped_gemm(inp, wt, offs_d, splits=z, glds=cfg)
                        err = (y.float() - ref.float()).abs().max().item() / (ref.float().abs().max().item() + 1e-6)
                        if err > 2e-2:
                            line.append(f"!!{name} glds{cfg}x{z} err {err:.2e}")
                            continue
                        t = timeit(lambda: MO.grouped_gemm(inp, wt, offs_d, splits=z, glds=cfg), iters=10)
                        best = min(best, (t, f"glds{cfg}x{z}"))
                line.append(f"{name} grouped {tb:.0f}us ({wt.numel() * 2 / tb / 1e6:.2f} TB/s) best {best[1]} "
                            f"{best[0]:.0f}us ({wt.numel() * 2 / best[0] / 1e6:.2f} TB/s)")
            res[f"moe_glds rows{rows}"] = " | ".join(line)
    if args.what == "gemm_big":
        for M in (512, 1024, 2048, 4096, 8192):
            for (n, k) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]:
                x = torch.randn(M, k, device=dev).bfloat16()
                w = torch.randn(n, k, device=dev).bfloat16()
                wt = w.t().contiguous()
                fl = 2 * M * n * k
                us = timeit(lambda: torch.nn.functional.linear(x, w), iters=10)
                us2 = timeit(lambda: torch.mm(x, wt), iters=10)
                res[f"big M{M} N{n} K{k}"] = f"NT {fl / us / 1e6:.0f} TF | NN {fl / us2 / 1e6:.0f} TF"
    if args.what == "gemm_replay":
        # per-step projection GEMMs of a recorded run: M = decode rows + prefill tokens
        from k8s_llm_rca_amd.ops.linear import linear
        steps = [json.loads(l) for l in open(args.trace)]
        Ms = [len(s["d"]) + sum(q for _, q in s["p"]) for s in steps]
        Ss = [len(s["d"]) + len(s["p"]) for s in steps]
        shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
        W = {k: torch.randn(n, kk, device=dev).bfloat16() for k, (n, kk) in shapes.items()}
        lm = torch.randn(128256, 4096, device=dev).bfloat16()
        cache = {}

        def t_of(name, M):
            key = (name, M)
            if key not in cache:
                w = lm if name == "lm" else W[name]
                x = torch.randn(M, w.shape[1], device=dev).bfloat16()
                cache[key] = timeit(lambda: linear(x, w), iters=10, warm=2)
            return cache[key]

        def bucket(M):  # quantise M to keep the run short (<= 3% error)
            if M <= 64:
                return M
            b = 1 << (M.bit_length() - 1)
            step = max(1, b // 32)
            return (M + step - 1) // step * step

        tot = {k: 0.0 for k in list(shapes) + ["lm"]}
        by_range = {}
        fl_range = {}
        for M, S in zip(Ms, Ss):
            Mb = bucket(M)
            rng = "M<=16" if M <= 16 else "M<=64" if M <= 64 else "M<=256" if M <= 256 else "M<=1024" if M <= 1024 \
                else "M>1024"
            for k in shapes:
                us = t_of(k, Mb) * 32
                tot[k] += us
                by_range[rng] = by_range.get(rng, 0.0) + us
                fl_range[rng] = fl_range.get(rng, 0.0) + 2.0 * M * shapes[k][0] * shapes[k][1] * 32
            tot["lm"] += t_of("lm", bucket(S))
        for k, v in tot.items():
            res[f"gemm_replay {k}"] = f"{v / 1e6:.3f} s over {len(Ms)} steps"
        for k, v in sorted(by_range.items()):
            res[f"gemm_replay range {k}"] = f"{v / 1e6:.3f} s {fl_range[k] / (v * 1e-6) / 1e12:6.0f} TFLOP/s ({sum(1 for M in Ms if (k == 'M<=16' and M <= 16) or (k == 'M<=64' and 16 < M <= 64) or (k == 'M<=256' and 64 < M <= 256) or (k == 'M<=1024' and 256 < M <= 1024) or (k == 'M>1024' and M > 1024))} steps)"
    if args.what == "share_test":
        # decode rows whose first L keys sit on the SAME pages in groups of G rows
        # (cross-thread prefix sharing): does the current kernel already get those
        # re-reads from L2 / MALL, i.e. does time track unique or total KV bytes?
        B, ctxv = 125, 4700
        nbs = (ctxv + BS - 1) // BS
        for L, G in [(0, 1), (1024, 42), (1536, 42), (2048, 42), (1536, 4)]:
            ls = L // BS
            n_groups = (B + G - 1) // G
            n_pages = n_groups * ls + B * (nbs - ls)
            perm = torch.randperm(n_pages).int()
            bt = torch.zeros(B, nbs, dtype=torch.int32)
            u = n_groups * ls
            for s_ in range(B):
                g = s_ // G
                bt[s_, :ls] = perm[g * ls:(g + 1) * ls]
                bt[s_, ls:] = perm[u:u + nbs - ls]
                u += nbs - ls
            ctx = [ctxv] * B
            meta, _ = make_meta(ctx, [1] * B, nq, nkv, BS, dev, True)
            meta.block_tables = bt.to(dev)
            kc = torch.empty(n_pages, nkv, BS, 128, device=dev, dtype=torch.bfloat16).normal_()
            vc = torch.empty(n_pages, nkv, 128, BS, device=dev, dtype=torch.bfloat16).normal_()
            q = torch.randn(B, (nq + 2 * nkv) * 128, device=dev).bfloat16()
            out = torch.empty(B, nq * 128, device=dev).bfloat16()
            us = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out), iters=20)
            tot_b = B * ctxv * nkv * 512
            uniq_b = n_pages * BS * nkv * 512
            res[f"share L{L} G{G}"] = (f"{us:.1f}us total {tot_b / us / 1e6:.2f} TB/s unique {uniq_b / us / 1e6:.2f} TB/s "
                                       f"(unique/total {uniq_b / tot_b:.2f})")
            del kc, vc
            torch.cuda.empty_cache()
    if args.what == "decode_sweep":
        for B in (32, 48, 56, 64, 72, 96, 128):
            for ctxv in (1000, 3400):
                for part in (512, 1024):
                    ctx = [ctxv] * B
                    meta, nb = make_meta(ctx, [1] * B, nq, nkv, BS, dev, True, part_size=part)
                    kc = torch.randn(nb, nkv, BS, 128, device=dev).bfloat16()
                    vc = torch.randn(nb, nkv, 128, BS, device=dev).bfloat16()
                    q = torch.randn(B, (nq + 2 * nkv) * 128, device=dev).bfloat16()
                    out = torch.empty(B, nq * 128, device=dev).bfloat16()
                    us = timeit(lambda: A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out))
                    waves = B * nkv * meta.n_parts
                    res[f"decode B{B} ctx{ctxv} part{part} waves{waves}"] = \
                        f"{us:.1f}us {B * ctxv * nkv * 512 / us / 1e6:.2f} TB/s"
    if args.what in ("all", "gemm"):
        for M in (1, 16, 64, 128):
            for (n, k) in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]:
                x = torch.randn(M, k, device=dev).bfloat16()
                w = torch.randn(n, k, device=dev).bfloat16()
                us = timeit(lambda: torch.nn.functional.linear(x, w), iters=20)
                res[f"gemm M{M} N{n} K{k}"] = f"{us:.1f}us {n * k * 2 / us / 1e6:.2f} TB/s"
                if M <= 128:
                    from k8s_llm_rca_amd.ops import linear as LIN
                    LIN.SKINNY_MAX_M = 128
                    us2 = timeit(lambda: LIN.linear(x, w), iters=20)
                    res[f"skinny M{M} N{n} K{k}"] = f"{us2:.1f}us {n * k * 2 / us2 / 1e6:.2f} TB/s"
                    us3 = timeit(lambda: torch.matmul(w, x.t()).t(), iters=20)
                    res[f"swapT M{M} N{n} K{k}"] = f"{us3:.1f}us {n * k * 2 / us3 / 1e6:.2f} TB/s"
    if args.what in ("all", "misc"):
        for T in (64, 4096):
            x = torch.randn(T, H, device=dev).bfloat16()
            r = torch.randn(T, H, device=dev).bfloat16()
            w = torch.ones(H, device=dev).bfloat16()
            us = timeit(lambda: N.rmsnorm(x, w, 1e-5, residual=r))
            res[f"rmsnorm T{T}"] = f"{us:.1f}us {T * H * 2 * 4 / us / 1e6:.2f} TB/s"
            gu = torch.randn(T, 2 * I, device=dev).bfloat16()
            us = timeit(lambda: N.silu_mul(gu))
            res[f"silu_mul T{T}"] = f"{us:.1f}us {T * I * 2 * 3 / us / 1e6:.2f} TB/s"
    for k, v in res.items():
        print(f"{k:40s} {v}")
    out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    json.dump(res, open(os.path.join(out_dir, "bench_kernels.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
