"""Tiny end-to-end check: Llama-3-8B (random init) prefill + constrained decode on one GPU."""
from __future__ import annotations

import time

import torch


def run_smoke(device: str = "cuda:0", model: str = "llama3-8b", max_new: int = 24) -> dict:
    from ..engine.engine import EngineConfig, LLMEngine
    from ..engine.grammar import Choice, Free, Grammar, Lit

    t0 = time.perf_counter()
    eng = LLMEngine(EngineConfig(model=model, device=device, kv_max_gb=2.0, max_batch_tokens=2048,
                                 graph_batch_sizes=(1, 2, 4)))
    sid = eng.new_sequence()
    prompt = eng.tok.system_prefix("You are a k8s expert.") + eng.tok.message("user", "Why is the pod pending?") + \
        eng.tok.header("assistant")
    g = Grammar([Lit('{"kind": '), Choice(['"Pod"', '"Node"', '"PersistentVolumeClaim"'], "k"),
                 Lit(', "why": "'), Free(max_new, min_tokens=4), Lit('"}')])
    out = {}

    def done(gen, st):
        out["text"] = eng.tok.decode(gen)
        out["stats"] = st

    eng.submit(sid, prompt, grammar=g, max_new=max_new, temperature=0.7, seed=1, on_done=done)
    eng.run_until_idle()
    torch.cuda.synchronize()
    assert "text" in out, "generation did not finish"
    assert out["text"].startswith('{"kind": "') and out["text"].endswith('"}'), out["text"]
    # a second run on the same thread must reuse the cached prefix
    prompt2 = eng.seqs[sid].tokens + eng.tok.message("user", "and now?") + eng.tok.header("assistant")
    eng.submit(sid, prompt2, grammar=None, max_new=8, on_done=done)
    eng.run_until_idle()
    torch.cuda.synchronize()
    out["seconds"] = time.perf_counter() - t0
    out["engine"] = dict(eng.stats)
    print("smoke ok:", out["text"][:80], {k: out["engine"][k] for k in ("steps", "graph_steps", "prefill_tokens")},
          f"{out['seconds']:.1f}s")
    return out
