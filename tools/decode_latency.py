"""Per-token decode latency of the Llama-3-8B engine at a fixed batch and context
(HIP-graph decode steps, native executor), for A/B of decode-path fusions.

For each variant (an env-style toggle applied in-process before the engine is
built) and each round: B fresh sequences with random CTX-token prompts are
prefilled (max_new = 1), then B more generate N tokens; the per-token step
time is (t_gen - t_prefill) / (N - 1).  Variants are interleaved round by
round in one process (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/decode_latency.py [--batch 1] [--ctx 5000] [--tokens 200] [--rounds 3]
           [--variants base,silu,full]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine  # noqa: E402
from k8s_llm_rca_amd.ops import linear as LIN  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def apply(variant):
    """Module-level switches the engine's kernels read per call (the dispatch table is global).
    base: no decode epilogue fusions; silu: the stream kernels' SwiGLU epilogue;
    full: + the skinny qkv GEMM's RoPE / KV-write epilogue; c1fuse: silu + the
    split-K variant dispatch table."""
    from k8s_llm_rca_amd.ops import attention as A
    LIN._stream_silu = variant != "base"
    A._skinny_rope = variant == "full"
    if variant == "c1fuse":
        LIN.load_dispatch(os.path.join(ROOT, "tools", "dispatch_c1fuse.json"))
    else:
        LIN.load_dispatch(LIN.dispatch_path("llama3-8b"))


def run_batch(eng, prompts, max_new):
    done = {}
    t0 = time.perf_counter()
    for i, p in enumerate(prompts):
        sid = eng.new_sequence()
        eng.submit(sid, p, None, max_new, temperature=0.0, on_done=lambda g, st, i=i: done.__setitem__(i, g))
    eng.run_until_idle()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, done


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--ctx", type=int, default=5000)
    ap.add_argument("--tokens", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="base,silu,full")
    a = ap.parse_args()
    variants = a.variants.split(",")
    g = torch.Generator().manual_seed(0)
    res = {v: [] for v in variants}
    engines = {}
    for r in range(a.rounds):
        for v in variants:
            apply(v)
            eng = engines.get(v)
            if eng is None:
                eng = engines[v] = LLMEngine(EngineConfig(model="llama3-8b", device="cuda", temperature=0.0,
                                                          kv_max_gb=40, graph_batch_sizes=(1, 2, 4, 8, 16, 32)))
                apply(v)  # the engine's init re-loads the dispatch table
            vocab = 120000
            mk = lambda: [torch.randint(1000, vocab, (a.ctx,), generator=g).tolist() for _ in range(a.batch)]
            tp, _ = run_batch(eng, mk(), 1)
            tg, done = run_batch(eng, mk(), a.tokens)
            n = min(len(x) for x in done.values())
            per = (tg - tp) / max(n - 1, 1) * 1e3
            res[v].append(per)
            print(json.dumps({"variant": v, "round": r, "ms_per_token": round(per, 3), "tokens": n,
                              "graph_steps": eng.stats["graph_steps"]}), flush=True)
    for v in variants:
        print(json.dumps({"variant": v, "median_ms_per_token": round(statistics.median(res[v]), 3),
                          "min": round(min(res[v]), 3)}), flush=True)


if __name__ == "__main__":
    main()
