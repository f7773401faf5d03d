"""Run a model's decode steps at every HIP-graph batch bucket through the
engine (graph capture included) with a few layers: finds a bucket whose
dispatch / executor launch fails before a long bench does.

python tools/exec_bucket_probe.py --model llama3-70b --layers 2"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--sizes", default="")
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda", model_overrides={"n_layers": a.layers},
                                 temperature=0.0, kv_max_gb=40))
    sizes = [int(x) for x in a.sizes.split(",")] if a.sizes else list(eng.cfg.graph_batch_sizes)
    bad = []
    for B in sizes:
        t0 = time.perf_counter()
        done = {}
        for i in range(B):
            sid = eng.new_sequence()
            p = eng.tok.system_prefix("s") + eng.tok.message("user", "probe %d " % i * 5) + eng.tok.header("assistant")
            eng.submit(sid, p, None, 6, temperature=0.0, on_done=lambda g, st, i=i: done.__setitem__(i, g))
        try:
            eng.run_until_idle()
            ok = len(done) == B and all(v is not None for v in done.values()) and eng.error is None
        except Exception as e:  # noqa: BLE001
            ok = False
            print(f"B={B}: {e!r}", flush=True)
        print(f"B={B} ok={ok} {time.perf_counter() - t0:.1f}s captures={eng.stats['captures']}", flush=True)
        if not ok:
            bad.append(B)
        for sid in list(eng.seqs):
            eng.release_sequence(sid)
    print("BAD", bad, flush=True)
    return 0  # the list is the result; a crash still exits non-zero


if __name__ == "__main__":
    sys.exit(main())
