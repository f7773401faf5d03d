"""RCA benchmark: analyses/s and p50 end-to-end latency (BASELINE.json headline).

One *step* = ``incidents`` RCA analyses (locate -> generate query -> analyze,
the full reference pipeline) on this rank's engine against this rank's
synthetic k8s graph, by ``incidents`` concurrent pipelines.  The timed K steps'
K x incidents analyses stream through those pipelines as one work queue (a
pipeline takes its next incident as soon as it finishes one, like the CLI's
``run --concurrency``); ``--sync-steps`` drains every step first instead.  Ranks are independent engine
replicas (data parallel, one process per GPU, TP=1): per-GPU work is fixed as
N grows (weak scaling).  Timing brackets exactly ``steps`` batches with a
barrier + device synchronize on both sides and takes the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import statistics
import sys
import time
from typing import Any, Dict, List, Optional

import torch

METRIC = "RCA analyses/sec + p50 end-to-end latency, Llama-3-8B backend, 10k-node graph"
REF_MAX_ANALYSES_PER_S = 0.033  # 1/(20 s + 10 s) best case of the sequential driver


def _dist_init():
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend)
    rank = dist.get_rank() if world > 1 else 0
    return world, rank


def _barrier(world: int, device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _allreduce_max(x: float, world: int, device) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device if device.type == "cuda" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _allgather_list(xs: List[float], world: int, device) -> List[float]:
    if world == 1:
        return xs
    import torch.distributed as dist
    out: List[Any] = [None] * world
    dist.all_gather_object(out, xs)
    return [v for part in out for v in part]


def run(args) -> Optional[Dict[str, Any]]:
    logging.basicConfig(level=logging.WARNING)
    world, rank = _dist_init()
    if args.gpus and world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    cuda = torch.cuda.is_available() and args.device != "cpu"
    device = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}" if cuda else "cpu")
    if cuda:
        torch.cuda.set_device(device)

    from ..api.graph import GraphQueryExecutor
    from ..api.service import AssistantService
    from ..engine.backend import EngineBackend
    from ..engine.engine import EngineConfig, LLMEngine
    from ..graph.synth import generate_cluster
    from ..pipeline.formats import GenerationBudget
    from ..pipeline.rca import RCAConfig, RCAPipeline, run_batch
    from ..utils import tracing

    n_steps, n_warm, per_step = args.steps, args.warmup, args.incidents
    t_setup = time.perf_counter()
    cluster = generate_cluster(args.graph_nodes, per_step * (n_steps + n_warm), seed=args.seed + 7919 * rank)
    if cuda and args.graph_device:
        from ..graph.device import to_device
        to_device(cluster.stategraph, device)
    pc = None
    tp_mode = args.tp > 1
    if tp_mode:
        import torch.distributed as dist
        from ..parallel.groups import ParallelContext, attach_custom_allreduce
        if world != args.tp:
            raise SystemExit(f"--tp {args.tp} needs WORLD_SIZE={args.tp} (one TP engine over all ranks)")
        pc = attach_custom_allreduce(ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD,
                                                     ep_size=world, ep_rank=rank, ep_group=dist.group.WORLD))
    eng = LLMEngine(EngineConfig(model=args.model, device=str(device),
                                 dtype=torch.bfloat16 if cuda else torch.float32,
                                 kv_max_gb=args.kv_gb, max_batch_tokens=args.max_batch_tokens,
                                 use_graphs=cuda and not args.no_graphs, prefix_sharing=not args.no_prefix_sharing,
                                 seed=args.seed + (0 if tp_mode else rank),
                                 num_blocks=None if cuda else 512), pc)
    if tp_mode and rank > 0:
        eng.serve_worker()  # replays every step rank 0 schedules
        return None
    eng.start()
    svc = AssistantService(EngineBackend(eng, temperature=args.temperature))
    budget = GenerationBudget(semantic_tokens=args.semantic_tokens, explanation_tokens=args.explanation_tokens,
                              conclusion_tokens=args.conclusion_tokens, resolution_tokens=args.resolution_tokens)
    cfg = RCAConfig(model=args.model, hints=not args.no_hints, budget=budget)
    meta_qe = GraphQueryExecutor(cluster.metagraph)
    state_qe = GraphQueryExecutor(cluster.stategraph)
    pipelines = [RCAPipeline(svc, meta_qe, state_qe, cfg) for _ in range(per_step)]
    setup_s = time.perf_counter() - t_setup

    incidents = cluster.incidents
    lat: List[float] = []
    errors: List[str] = []
    n_done = 0
    for w in range(n_warm):
        chunk = incidents[w * per_step:(w + 1) * per_step]
        st = run_batch(None, [i.message for i in chunk], truths=chunk, pipelines=pipelines)
        errors += st.errors
    tracing.reset()
    if not args.no_gc_freeze:
        # the graph store, model config, grammar tables and warm-up results are
        # long-lived: move them out of the collector's generations so a gen-2
        # pass in the timed region does not walk millions of objects while
        # holding the GIL (the engine thread issues kernels under it)
        import gc
        gc.collect()
        gc.freeze()
    stats0 = dict(eng.stats)
    eng.kv.reset_peak()
    t_wall0 = time.time()
    sync_world = 1 if tp_mode else world
    _barrier(sync_world, device)
    t0 = time.perf_counter()
    if args.sync_steps:  # batch-synchronous: every step drains before the next starts
        for s in range(n_steps):
            chunk = incidents[(n_warm + s) * per_step:(n_warm + s + 1) * per_step]
            st = run_batch(None, [i.message for i in chunk], truths=chunk, pipelines=pipelines)
            lat += st.latencies
            errors += st.errors
            n_done += len(st.results)
    else:  # streaming: the K steps' incidents feed one work queue of `incidents` concurrent pipelines
        chunk = incidents[n_warm * per_step:(n_warm + n_steps) * per_step]
        st = run_batch(None, [i.message for i in chunk], truths=chunk, pipelines=pipelines)
        lat += st.latencies
        errors += st.errors
        n_done += len(st.results)
    _barrier(sync_world, device)
    elapsed = time.perf_counter() - t0
    eng.stop()
    eng.stop_workers()
    if eng.error is not None:
        raise eng.error
    max_elapsed = _allreduce_max(elapsed, sync_world, device)
    all_lat = _allgather_list(lat, sync_world, device)
    total = n_done * sync_world
    value = total / max_elapsed
    d = {k: eng.stats[k] - stats0.get(k, 0) for k in eng.stats}
    ttft = sorted(rs.metrics["ttft_s"] for rs in list(svc.runs.values())
                  if rs.run.created_at >= t_wall0 and "ttft_s" in rs.metrics)
    p50 = statistics.median(all_lat) if all_lat else 0.0
    p90 = sorted(all_lat)[int(0.9 * (len(all_lat) - 1))] if all_lat else 0.0
    model_name = {"llama3-8b": "Llama-3-8B", "llama3-70b": "Llama-3-70B",
                  "mixtral-8x7b": "Mixtral-8x7B"}.get(args.model, args.model)
    metric = METRIC if (args.model == "llama3-8b" and args.graph_nodes == 10_000) else (
        f"RCA analyses/sec + p50 end-to-end latency, {model_name} backend, {args.graph_nodes}-node graph")
    res = {
        "metric": metric,
        "value": round(value, 4),
        "unit": "analyses/s",
        "n_gpus": world,
        "steps": n_steps,
        "warmup": n_warm,
        "ms_per_step": round(1000.0 * max_elapsed / n_steps, 2),
        "higher_is_better": True,
        "scaling": "strong" if tp_mode else "weak",
        "vs_baseline": round(value / REF_MAX_ANALYSES_PER_S, 2),
        "dtype": "bf16" if cuda else "fp32",
        "data": "synthetic k8s stategraph (seeded generator, fault injection) + random-init weights",
        "config": {"model": model_name,
                   "global_batch": per_step * sync_world, "seq_len": eng.max_context,
                   "parallelism": f"tp{world}" if tp_mode else f"dp{world}",
                   "graph_nodes": cluster.stategraph.num_nodes,
                   "incidents_per_gpu_per_step": per_step, "grammar_hints": not args.no_hints,
                   "step_mode": "sync" if args.sync_steps else "stream"},
        "p50_latency_s": round(p50, 3),
        "p90_latency_s": round(p90, 3),
        "errors": len(errors),
        "engine": {"steps": d["steps"], "graph_steps": d["graph_steps"], "prefill_tokens": d["prefill_tokens"],
                   "decode_tokens": d["decode_tokens"], "sampled_tokens": d["sampled_tokens"],
                   "forced_tokens": d["forced_tokens"], "forward_s": round(d["forward_s"], 3),
                   "sample_s": round(d["sample_s"], 3), "host_s": round(d["host_s"], 3),
                   "evictions": d["evictions"], "requests": d["requests"],
                   "decode_ctx_tokens": d["decode_ctx_tokens"], "prefill_ctx_tokens": d["prefill_ctx_tokens"],
                   "kv_blocks": eng.kv.num_blocks, "wait_s": round(d["wait_s"], 3),
                   "post_s": round(d["post_s"], 3), "admit_s": round(d["admit_s"], 3),
                   "prefix_hit_tokens": d["prefix_hit_tokens"], "shared_kv_blocks": eng.kv.shared_blocks,
                   "captures": d["captures"], "capture_s": round(d["capture_s"], 3),
                   **{k: round(d[k], 3) for k in ("eager_issue_s", "eager_gpu_s", "graph_issue_s", "graph_gpu_s")}},
        "throughput": {  # rank 0's engine over the timed window
            "prefill_tok_per_s": round(d["prefill_tokens"] / elapsed, 1),
            "decode_tok_per_s": round(d["decode_tokens"] / elapsed, 1),
            "forced_tok_per_s": round(d["forced_tokens"] / elapsed, 1),
            "avg_decode_batch": round(d["decode_tokens"] / max(1, d["steps"]), 1),
            "runs": len(ttft),
            "ttft_p50_s": round(ttft[len(ttft) // 2], 4) if ttft else None,
            "kv_peak_util": round(eng.kv.peak_used / max(1, eng.kv.num_blocks), 4)},
        "setup_s": round(setup_s, 1),
        "blaslt_tune": ({"s": round(eng.t_gemm_tune, 2), "points": len(eng.gemm_tuning),
                         "heuristic_us": round(sum(t[3] for t in eng.gemm_tuning), 1),
                         "tuned_us": round(sum(t[4] for t in eng.gemm_tuning), 1)}
                        if getattr(eng, "gemm_tuning", None) else None),
        "stages": {k: round(v["mean_ms"], 2) for k, v in tracing.snapshot().items()},
    }
    if world > 1 and not tp_mode:
        import torch.distributed as dist
        dist.barrier()
    return res if rank == 0 else None


def parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--gpus", type=int, default=None, help="GPUs (= WORLD_SIZE under torchrun; default 1)")
    p.add_argument("--preset", default=None, choices=sorted(PRESETS), help="a BASELINE.json config")
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (one engine over all ranks)")
    p.add_argument("--device", default="cuda")
    p.add_argument("--incidents", type=int, default=128, help="concurrent RCA analyses per GPU per step")
    p.add_argument("--graph-nodes", type=int, default=10_000)
    p.add_argument("--graph-device", action="store_true", help="mirror the stategraph to HBM (HIP graph kernels)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--kv-gb", type=float, default=None, help="KV pool cap (default: 85%% of free HBM)")
    p.add_argument("--max-batch-tokens", type=int, default=8192)
    p.add_argument("--temperature", type=float, default=0.7)
    p.add_argument("--semantic-tokens", type=int, default=192)
    p.add_argument("--explanation-tokens", type=int, default=40)
    p.add_argument("--conclusion-tokens", type=int, default=80)
    p.add_argument("--resolution-tokens", type=int, default=80)
    p.add_argument("--no-hints", action="store_true")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--no-gc-freeze", action="store_true", help="keep warm-up objects in the GC generations")
    p.add_argument("--sync-steps", action="store_true",
                   help="drain each step's batch before starting the next (default: the K steps' incidents stream "
                        "through the same concurrent pipelines, as `run --concurrency` processes a message file)")
    p.add_argument("--no-prefix-sharing", action="store_true", help="do not share prompt KV pages across threads")
    return p


# One preset per BASELINE.json config; explicit flags override.
PRESETS: Dict[str, Dict[str, Any]] = {
    # "OPT-125m CPU backend, 10-node toy k8s dependency graph, single pod-crash RCA (plumbing, no GPU)"
    "opt125m-cpu-toy": dict(model="opt-125m", device="cpu", graph_nodes=10, incidents=1),
    # the headline: "RCA analyses/sec + p50 latency, Llama-3-8B backend, 10k-node graph"
    "llama3-8b-10k": dict(model="llama3-8b", graph_nodes=10_000),
    # "Llama-3-8B TP=1 bf16 on one MI355X, 1k-node synthetic k8s graph"
    "llama3-8b-1k": dict(model="llama3-8b", graph_nodes=1_000),
    # "Llama-3-8B TP=1, 100k-node synthetic graph (HIP CSR metapath BFS stress)"
    "llama3-8b-100k": dict(model="llama3-8b", graph_nodes=100_000, graph_device=True),
    # "Llama-3-70B TP=8 over xGMI, 10k-node graph, batched multi-incident RCA" (torchrun --nproc-per-node 8)
    "llama3-70b-tp8-10k": dict(model="llama3-70b", tp=8, graph_nodes=10_000),
    # "Mixtral 8x7B MoE backend (grouped GEMM + expert all-to-all over xGMI), 10k-node graph"
    "mixtral-10k": dict(model="mixtral-8x7b", graph_nodes=10_000),
}


def main(argv=None) -> int:
    p = parser()
    pre, _ = p.parse_known_args(argv)
    if pre.preset:
        p.set_defaults(**PRESETS[pre.preset])
    args = p.parse_args(argv)
    res = run(args)
    if res is not None:
        print(json.dumps(res), flush=True)
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        # Orderly teardown: no rank exits while a peer's gloo/RCCL background
        # threads still reference it (an abort at exit fails the torchrun job).
        dist.barrier()
        dist.destroy_process_group()
    return 0
