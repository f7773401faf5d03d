"""Host-side (CPU) profile of engine steps on the GPU: where does the time to
*issue* a mixed prefill+decode step go?

    python tools/prof_host.py --seqs 64 --prompt 1500 --steps 30
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=1500)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--model", default="llama3-8b")
    args = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=args.model, device="cuda", dtype=torch.bfloat16, kv_max_gb=40))
    tok = eng.tok
    sids = [eng.new_sequence() for _ in range(args.seqs)]
    for i, sid in enumerate(sids):
        p = tok.system_prefix("sys") + tok.message("user", ("incident %d " % i) * (args.prompt // 3)) + \
            tok.header("assistant")
        eng.submit(sid, p, None, 400)
    while any(s.pending > 1 for s in eng.seqs.values() if s.req is not None):  # finish the big prefill
        eng.step()
    torch.cuda.synchronize()

    def mixed_steps(n):
        for k in range(n):
            if k % 2 == 0:  # a short forced-token-like extension on a few sequences -> mixed step
                for s in list(eng.seqs.values())[:4]:
                    if s.req is not None:
                        s.tokens.extend([100 + k] * 6)
            eng.step()
        torch.cuda.synchronize()

    mixed_steps(4)
    s0 = dict(eng.stats)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    mixed_steps(args.steps)
    pr.disable()
    wall = time.perf_counter() - t0
    d = {k: eng.stats[k] - s0.get(k, 0) for k in eng.stats if isinstance(eng.stats[k], (int, float))}
    print(f"wall {wall * 1e3 / args.steps:.2f} ms/step  forward_s {d['forward_s'] * 1e3 / args.steps:.2f} ms/step "
          f"steps {d['steps']} graph {d['graph_steps']}")
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(35)
    print(out.getvalue())


if __name__ == "__main__":
    main()
