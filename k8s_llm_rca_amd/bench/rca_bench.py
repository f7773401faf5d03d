"""RCA benchmark: analyses/s and p50 end-to-end latency (BASELINE.json headline).

Each rank runs ``--incidents`` (128) concurrent RCA pipelines (locate ->
generate query -> analyze, the full reference pipeline,
``test_with_file.py:64-204``) on its own engine against its own synthetic k8s
graph, as a steady stream: a pipeline takes its next incident the moment it
finishes one.  One *step* is a fixed quantum (``--quantum``, 16) of completed
analyses per rank: ``--warmup`` steps stream untimed, then exactly ``--steps``
quanta are timed with a barrier + device synchronize on both sides and the max
over ranks is taken.  Ranks are independent engine replicas (data parallel,
one process per GPU, TP=1: weak scaling), or one tensor-parallel engine over
all ranks (``--tp``: strong scaling).  ``bench.py --gpus N`` spawns the N
ranks itself when no launcher did.  A wall-clock budget stops the run and
still prints the JSON line (flagged).  After the timed window the same stream
is optionally measured with the oracle hints off (``no_hints`` in the line).
The graph is built at ``--graph-nodes`` including the injected faults; the
stream cycles the distinct incidents.
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

from ..knobs import KNOBS

METRIC = "RCA analyses/sec + p50 end-to-end latency, Llama-3-8B backend, 10k-node graph"
# The thread-truncation contract is part of the workload definition: the
# reference's threads grow for the whole batch (test_with_file.py:28-38) and its
# server cuts them at the model window; here an overflowing thread drops its
# oldest non-seed turns down to TRUNC_LOW of the window, keeps the system prompt
# and the first KEEP_SEED messages (the reference's seeding messages), and the
# cut point is sticky (engine/backend.py).  These two numbers set how much of
# the prefill is re-prefill after a cut (~half in the steady state), so they
# are pinned here, checked against the backend and reported in the JSON config.
TRUNCATION_CONTRACT = {"trunc_low": 0.5, "keep_seed": 2, "policy": "sticky"}
REF_MAX_ANALYSES_PER_S = 0.033  # 1/(20 s + 10 s) best case of the sequential driver


def _tail_foreign(eng) -> int:
    try:
        from ..ops import linear as LIN
        return LIN.big_tail_foreign(eng.device)
    except Exception:  # noqa: BLE001 -- a CPU engine / no library
        return 0


def _native_cpu() -> Dict[int, tuple]:
    """(user, system) CPU seconds per native (non-Python) thread of this
    process, by thread id."""
    import threading
    try:
        import psutil
        py = {t.native_id for t in threading.enumerate()}
        return {t.id: (t.user_time, t.system_time) for t in psutil.Process().threads() if t.id not in py}
    except Exception:
        return {}


def _native_detail(tid: int, samples: int = 0) -> Dict[str, Any]:
    """What a busy native thread is doing, from /proc (no GPU call, no
    ptrace): its name, kernel wait channel and current system call -- a thread
    spinning in user space shows wchan 0 and mostly user time; one blocked in
    the driver shows an ioctl / futex / poll."""
    out: Dict[str, Any] = {"tid": tid}
    for key, fn in (("comm", "comm"), ("wchan", "wchan"), ("syscall", "syscall")):
        try:
            with open(f"/proc/self/task/{tid}/{fn}") as f:
                v = f.read().strip()
            out[key] = v.split()[0] if key == "syscall" and v else v
        except OSError:
            pass
    if samples:
        # where it spends its time: the current system call sampled every 2 ms
        # ("running" = in user space; a number = blocked / inside that syscall;
        # for ioctl the request code follows, e.g. KFD's wait-events ioctl)
        import time
        hist: Dict[str, int] = {}
        for _ in range(samples):
            try:
                with open(f"/proc/self/task/{tid}/syscall") as f:
                    v = f.read().split()
            except OSError:
                break
            k = v[0] if v else "?"
            if k == "16" and len(v) > 2:  # ioctl: add the request code
                k = f"16:{v[2]}"
            hist[k] = hist.get(k, 0) + 1
            time.sleep(0.002)
        out["syscall_samples"] = dict(sorted(hist.items(), key=lambda kv: -kv[1])[:6])
        try:  # creation order among this process's threads (start time, clock ticks)
            starts = {}
            for t in os.listdir("/proc/self/task"):
                with open(f"/proc/self/task/{t}/stat") as f:
                    starts[int(t)] = int(f.read().rsplit(")", 1)[1].split()[19])
            out["start_rank"] = sorted(starts, key=lambda t: (starts[t], t)).index(tid)
        except (OSError, ValueError, IndexError):
            pass
    return out


def _thread_cpu() -> Dict[str, float]:
    """CPU seconds per thread group of this process (engine / graph batcher /
    RCA pipelines / other): which Python threads compete with the engine
    thread for the interpreter lock over the timed window."""
    import threading
    try:
        import psutil
        per = {t.id: t.user_time + t.system_time for t in psutil.Process().threads()}
    except Exception:
        return {}
    names = {t.native_id: t.name for t in threading.enumerate()}
    out: Dict[str, float] = {}
    for tid, cpu in per.items():
        n = names.get(tid)
        if n is None:  # a native thread (HIP runtime, torch / OpenMP pools): its kernel-side name
            try:
                with open(f"/proc/self/task/{tid}/comm") as f:
                    n = "native:" + "".join(c for c in f.read().strip() if not c.isdigit()).rstrip("-_:")
            except OSError:
                n = "native:?"
        g = "engine" if n == "llm-engine" else "graph_batcher" if n == "graph-batcher" else \
            "pipelines" if n == "rca-stream" else "main" if n == "MainThread" else \
            n if n.startswith("native:") else "other"
        out[g] = out.get(g, 0.0) + cpu
    return out


def _dist_init(tp_mode: bool, same_gpu: bool):
    """Data-parallel replicas exchange only host-side metrics (a barrier, the
    max elapsed time, latency lists): a gloo group, so the DP bench never
    initialises RCCL and runs the same code with any device mapping.  A TP
    engine over separate GPUs uses RCCL's group for the xGMI communicator's
    setup (its data collectives run on the xGMI kernels); TP ranks sharing one
    GPU use gloo (RCCL refuses duplicate devices)."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        backend = "nccl" if (torch.cuda.is_available() and tp_mode and not same_gpu) else "gloo"
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
    on_dev = device.type == "cuda" and dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=device if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _allgather_objects(x: Any, world: int) -> List[Any]:
    if world == 1:
        return [x]
    import torch.distributed as dist
    out: List[Any] = [None] * world
    dist.all_gather_object(out, x)
    return out


def _allgather_list(xs: List[float], world: int, device) -> List[float]:
    if world == 1:
        return xs
    import torch.distributed as dist
    out: List[Any] = [None] * world
    dist.all_gather_object(out, xs)
    return [v for part in out for v in part]


def _window_mark(tag: int, cuda: bool) -> None:
    """A named one-wave kernel at the start (1) / end (2) of the timed window:
    ``tools/window_summary.py`` cuts a rocprofv3 kernel trace to exactly the
    kernels between the two marks (the engine issues on the same stream)."""
    if cuda:
        from ..ops._lib import lib, stream_ptr
        lib().k8s_window_mark(tag, stream_ptr())


# A window whose analyses sampled almost nothing did almost no work (e.g. every
# request ending after a few tokens): such a line is not a measurement.  The
# conclusion + resolution budgets alone are 160 sampled tokens per analysis; a
# normal window samples ~960 (BENCH_r04 work_per_analysis).
SANITY_MIN_SAMPLED_PER_ANALYSIS = 80


def sanity(res: Dict[str, Any]) -> Dict[str, Any]:
    """Checks that the timed window did the work it claims (``ok`` false makes
    bench.py exit non-zero after printing the line)."""
    why = []
    if res["engine"].get("nonfinite_rows", 0):
        why.append(f"{res['engine']['nonfinite_rows']} sampled rows had non-finite logits")
    n = max(1, res["analyses_timed"])
    if res["errors"] > 0.05 * n:
        why.append(f"{res['errors']} of {n} timed analyses failed")
    sp = res["work_per_analysis"]["sampled_tokens"]
    if res["config"]["grammar_hints"] and sp < SANITY_MIN_SAMPLED_PER_ANALYSIS:
        why.append(f"{sp} sampled tokens per analysis (< {SANITY_MIN_SAMPLED_PER_ANALYSIS}): the runs ended early")
    if res["truncated_by_time_budget"]:
        why.append("the time budget cut the window short")
    return {"ok": not why, "reasons": why}


def run(args) -> Optional[Dict[str, Any]]:
    logging.basicConfig(level=logging.WARNING)
    # bind this rank to its GPU's NUMA-local CPU slice before anything starts a
    # thread or touches the GPU (utils/placement.py; every later thread inherits it)
    from ..utils.placement import bind_rank
    placement = bind_rank(int(os.environ.get("LOCAL_RANK", "0")),
                          int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
    world, rank = _dist_init(args.tp > 1, args.same_gpu)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (bench.py spawns the ranks itself)")
    cuda = torch.cuda.is_available() and args.device != "cpu"
    # --same-gpu: every rank on cuda:0 (the one-GPU rehearsal of an N-GPU job: N DP
    # replicas or N TP ranks sharing one MI355X; give each replica --kv-gb)
    device = torch.device(("cuda:0" if args.same_gpu else f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}")
                          if cuda else "cpu")
    if args.same_gpu and cuda and world > 1 and args.kv_gb is None:
        raise SystemExit("--same-gpu with several ranks needs --kv-gb (each rank would size its KV pool "
                         "from the whole GPU's free memory)")
    # CPU-side torch ops of the serving process are tiny (metadata packing, pinned
    # staging): an intra-op pool of OMP_NUM_THREADS spinning workers only competes
    # with the engine thread for the rank's CPU share.  K8SRCA_TORCH_THREADS=N
    # sets the pool size (unset: torch's default).
    nthr = KNOBS.torch_threads
    if nthr:
        torch.set_num_threads(int(nthr))
    if cuda:
        torch.cuda.set_device(device)

    from ..api.graph import GraphQueryExecutor
    from ..api.service import AssistantService
    from ..engine.backend import EngineBackend
    from ..engine.engine import EngineConfig, LLMEngine
    from ..graph.synth import NODES_PER_INCIDENT, generate_cluster
    from ..pipeline.formats import GenerationBudget
    from ..pipeline.rca import IncidentStream, RCAConfig, RCAPipeline
    from ..utils import tracing

    t_start = time.perf_counter()
    deadline = t_start + args.time_budget if args.time_budget else None
    n_steps, n_warm, quantum, conc = args.steps, args.warmup, args.quantum, args.incidents
    nh_steps = 0 if args.no_hints else args.no_hints_steps
    pc = None
    tp_mode = args.tp > 1
    if args.tp_sim > 1:
        # one rank of a TP=N deployment at real shapes, collectives stood in (parallel/tpsim.py)
        if not cuda or world > 1 or tp_mode:
            raise SystemExit("--tp-sim runs ONE process on one GPU")
        from ..models.config import get_config
        from ..parallel.tpsim import sim_context
        pc = sim_context(args.tp_sim, ep=args.tp_sim if get_config(args.model).n_experts else 1)
    if tp_mode:
        import torch.distributed as dist
        from ..parallel.groups import ParallelContext, attach_custom_allreduce
        if world != args.tp:
            raise SystemExit(f"--tp {args.tp} needs WORLD_SIZE={args.tp} (one TP engine over all ranks)")
        pc = attach_custom_allreduce(ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD,
                                                     ep_size=world, ep_rank=rank, ep_group=dist.group.WORLD),
                                     same_gpu=args.same_gpu and cuda)
    eng = LLMEngine(EngineConfig(model=args.model, device=str(device),
                                 dtype=torch.bfloat16 if cuda else torch.float32,
                                 kv_max_gb=args.kv_gb, max_batch_tokens=args.max_batch_tokens,
                                 max_context=args.max_context,
                                 **({"kv_host_gb": args.kv_host_gb} if args.kv_host_gb is not None else {}),
                                 use_graphs=cuda and not args.no_graphs, prefix_sharing=not args.no_prefix_sharing,
                                 seed=args.seed + (0 if tp_mode else rank),
                                 num_blocks=None if cuda else 512), pc)
    if tp_mode and rank > 0:
        eng.serve_worker()  # replays every step rank 0 schedules (no graph, no pipelines on this rank)
        return None
    # distinct incidents: enough that no two concurrent pipelines share one, capped
    # so the injected faults stay within the graph-size target (the stream cycles them)
    need = (n_warm + n_steps + nh_steps) * quantum + 2 * conc  # pre-aging cycles them too
    n_inc = max(1, min(need, int(0.3 * args.graph_nodes / NODES_PER_INCIDENT)))
    cluster = generate_cluster(args.graph_nodes, n_inc, seed=args.seed + 7919 * rank)
    batchers = []
    if cuda and not args.no_graph_device:
        # both graphs resident in HBM; every pipeline's CONTAINS / STATE / var-length
        # operator calls coalesced into one HIP launch per op (graph/batcher.py)
        from ..graph.batcher import enable_batching
        from ..graph.device import to_device
        for g in (cluster.stategraph, cluster.metagraph):
            to_device(g, device)
            batchers.append(enable_batching(g))
    eng.start()
    backend = EngineBackend(eng, temperature=args.temperature, keep_seed=TRUNCATION_CONTRACT["keep_seed"],
                            trunc_low=TRUNCATION_CONTRACT["trunc_low"])
    if (backend.trunc_low, backend.keep_seed) != (TRUNCATION_CONTRACT["trunc_low"], TRUNCATION_CONTRACT["keep_seed"]):
        raise SystemExit(f"truncation {backend.trunc_low}/{backend.keep_seed} differs from the bench contract "
                         f"{TRUNCATION_CONTRACT}")
    svc = AssistantService(backend)
    budget = GenerationBudget(semantic_tokens=args.semantic_tokens, explanation_tokens=args.explanation_tokens,
                              conclusion_tokens=args.conclusion_tokens, resolution_tokens=args.resolution_tokens)
    cfg = RCAConfig(model=args.model, hints=not args.no_hints, budget=budget)
    meta_qe = GraphQueryExecutor(cluster.metagraph)
    state_qe = GraphQueryExecutor(cluster.stategraph)
    pipelines = [RCAPipeline(svc, meta_qe, state_qe, cfg) for _ in range(conc)]
    stream = IncidentStream(pipelines, cluster.incidents, hints=not args.no_hints)
    setup_s = time.perf_counter() - t_start
    # ---- thread regime: the reference keeps ONE set of three threads per driver and
    # pushes every incident of its CSV through them (test_with_file.py:28-38,64), so
    # a steady-state analysis runs against a long history cut at the model window.
    # Each pipeline's threads are pre-aged with --thread-age prior incidents of the
    # stream (the pipeline's own prompts and graph queries; replies drawn on the host
    # through the same grammars: EngineBackend.set_replay) -- their KV is built by
    # the engine's real prefill on each thread's first run, inside the warm-up.
    t_age = time.perf_counter()
    if args.thread_age > 0:
        backend.set_replay(True, seed=args.seed + 104729 * rank)
        stream.pre_age(args.thread_age)
        backend.set_replay(False)
    age_s = time.perf_counter() - t_age
    ctx_aged = backend.thread_stats()

    last = [time.perf_counter()]

    def _poll():
        if eng.error is not None:
            raise RuntimeError(f"engine fault: {eng.error!r}")
        now = time.perf_counter()
        if now - last[0] >= 20.0 and rank == 0:  # progress on stderr (a silent run looks hung)
            last[0] = now
            print(f"[bench] t={now - t_start:.0f}s completed={stream.n_ok} errors={stream.n_err} "
                  f"engine_steps={eng.stats['steps']}", file=sys.stderr, flush=True)

    # ---- warm-up: every pipeline completes an engine analysis on its aged threads
    # (their history prefill is done and they run at steady-state context), and at
    # least W quanta complete in all
    stream.start()
    truncated = not (stream.wait_each(1, deadline, _poll) and stream.wait_ok(n_warm * quantum, deadline, _poll))
    warm_s = time.perf_counter() - t_age - age_s
    tracing.reset()
    if not args.no_gc_freeze:
        # the graph store, model config, grammar tables and warm-up results are
        # long-lived: move them out of the collector's generations so a gen-2
        # pass in the timed region does not walk millions of objects while
        # holding the GIL (the engine thread issues kernels under it)
        import gc
        gc.collect()
        gc.freeze()
    sync_world = 1 if tp_mode else world
    # ---- timed: exactly K quanta of completed analyses, barrier + sync on both sides
    _barrier(sync_world, device)
    stats0 = dict(eng.stats)
    sim0 = dict(eng.sim_rows)
    eng.kv.reset_peak()
    age0 = [p.n_analyses for p in pipelines]
    ctx0 = backend.thread_stats()
    t_wall0 = time.time()
    cpu0, ncpu0 = _thread_cpu(), _native_cpu()
    _window_mark(1, cuda)
    t0 = time.perf_counter()
    base = stream.n_ok
    done_all = stream.wait_ok(base + n_steps * quantum, deadline, _poll)
    t_end = time.perf_counter()
    _window_mark(2, cuda)
    cpu1, ncpu1 = _thread_cpu(), _native_cpu()
    ctx1 = backend.thread_stats()
    # the busiest native threads over the window (HIP runtime / torch pools: one
    # polling thread vs many pool workers)
    ndelta = {t: (u - ncpu0.get(t, (0.0, 0.0))[0], sy - ncpu0.get(t, (0.0, 0.0))[1])
              for t, (u, sy) in ncpu1.items()}
    native_top = sorted((round(u + sy, 2) for u, sy in ndelta.values()), reverse=True)
    busiest = sorted(ndelta.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))[:2]
    n_done = min(stream.n_ok - base, n_steps * quantum)
    _barrier(sync_world, device)
    elapsed = time.perf_counter() - t0
    # outside the timed window: the stream still runs, so the sample sees the same threads busy
    native_busiest = [dict(_native_detail(t, 300 if j == 0 else 0), user_s=round(u, 2), sys_s=round(sy, 2))
                      for j, (t, (u, sy)) in enumerate(busiest)]
    truncated = truncated or not done_all
    d = {k: eng.stats[k] - stats0.get(k, 0) for k in eng.stats}
    sim = None
    if args.tp_sim > 1:
        from ..parallel.tpsim import project
        hist = {T: n - sim0.get(T, 0) for T, n in eng.sim_rows.items() if n - sim0.get(T, 0) > 0}
        pr = project(hist, pc, eng.mc.hidden, eng.mc.n_layers, device,
                     moe_k=eng.mc.top_k if eng.mc.n_experts else 0)
        wall_p = elapsed - pr["standin_s"] + pr["modelled_s"]
        sim = {"tp": args.tp_sim, "rank": 0,
               "ep": pc.ep_size,
               "what": "ONE rank of a TP=%d%s engine at real shapes on one GPU; every collective is a local "
                       "stand-in moving the same bytes (parallel/tpsim.py); a projection, not a scaling "
                       "measurement" % (args.tp_sim, f" / EP={pc.ep_size}" if pc.ep_size > 1 else ""),
               "measured_value": round(n_done / elapsed, 4) if elapsed > 0 else 0.0,
               "standin_collectives_s": round(pr["standin_s"], 3),
               "modelled_xgmi_collectives_s": round(pr["modelled_s"], 3),
               "projected_value": round(n_done / wall_p, 4) if wall_p > 0 else 0.0,
               "projected_ms_per_step": round(1000.0 * wall_p / n_steps, 2),
               "collective_share_modelled": round(pr["modelled_s"] / wall_p, 4) if wall_p > 0 else 0.0,
               # hop-latency sensitivity of the model (one fabric hand-off = 2.5 / 5 / 10 us)
               "projected_value_by_hop_us": {
                   str(h): round(n_done / w, 4) if (w := elapsed - pr["standin_s"] + m) > 0 else 0.0
                   for h, m in pr["modelled_s_by_hop"].items()},
               "per_T": pr["per_T"]}
    gq = {k: 1e3 * v["total_s"] for k, v in tracing.snapshot().items()}
    bstats = [dict(b.stats) for b in batchers]
    lat = stream.window(t0, t_end + 1e-9)
    err_timed = sum(1 for t, _, ok, *_ in list(stream.done) if not ok and t0 <= t <= t_end)
    stage3 = stream.stage3(t0, t_end + 1e-9)
    # ---- optional no-hints window (disclosure): the same engine and stream with the
    # oracle hints off, timed after one full turnover of the in-flight analyses
    nh = None
    if nh_steps and not truncated:
        cfg.hints = False
        stream.hints = False
        n_switch = stream.n_ok + conc
        if stream.wait_ok(n_switch, deadline, _poll):
            t_nh0 = time.perf_counter()
            if stream.wait_ok(n_switch + nh_steps * quantum, deadline, _poll):
                dt = time.perf_counter() - t_nh0
                nh_lat = stream.window(t_nh0, time.perf_counter())
                nh = {"value": round(nh_steps * quantum * sync_world / dt, 4), "steps": nh_steps,
                      "p50_latency_s": round(statistics.median(nh_lat), 3) if nh_lat else None}
    stream.stop()
    svc.close()  # in-flight analyses end fast: their remaining LLM runs fail at once
    clean = stream.join(60.0)
    eng.stop()
    eng.stop_workers()
    if eng.error is not None:
        raise eng.error
    max_elapsed = _allreduce_max(elapsed, sync_world, device)
    all_lat = _allgather_list(lat, sync_world, device)
    total = n_done * sync_world
    value = total / max_elapsed if max_elapsed > 0 else 0.0
    ttft = sorted(rs.metrics["ttft_s"] for rs in list(svc.runs.values())
                  if rs.run.created_at >= t_wall0 and "ttft_s" in rs.metrics)
    p50 = statistics.median(all_lat) if all_lat else 0.0
    p90 = sorted(all_lat)[int(0.9 * (len(all_lat) - 1))] if all_lat else 0.0
    model_name = {"llama3-8b": "Llama-3-8B", "llama3-70b": "Llama-3-70B",
                  "mixtral-8x7b": "Mixtral-8x7B"}.get(args.model, args.model)
    metric = METRIC if (args.model == "llama3-8b" and args.graph_nodes == 10_000) else (
        f"RCA analyses/sec + p50 end-to-end latency, {model_name} backend, {args.graph_nodes}-node graph")
    if args.tp_sim > 1:
        metric = f"PROJECTION (rank 0 of TP={args.tp_sim} simulated on one GPU): " + metric
    placements = [placement] if tp_mode else _allgather_objects(placement, world)
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
                   "global_batch": conc * sync_world, "seq_len": eng.max_context,
                   "parallelism": (f"tp{args.tp_sim}-sim-rank0" if args.tp_sim > 1 else
                                   f"tp{world}" if tp_mode else f"dp{world}"),
                   "graph_nodes": cluster.stategraph.num_nodes, "graph_nodes_target": args.graph_nodes,
                   "distinct_incidents": len(cluster.incidents),
                   "concurrent_analyses_per_gpu": conc, "analyses_per_step": quantum * sync_world,
                   "grammar_hints": not args.no_hints, "step_mode": "stream",
                   "truncation": dict(TRUNCATION_CONTRACT, max_context=eng.max_context)},
        "p50_latency_s": round(p50, 3),
        "p90_latency_s": round(p90, 3),
        "analyses_timed": total,
        "errors": err_timed,
        "errors_total": stream.n_err,
        # timed analyses whose pipeline reached stage 3 (a statepath was analyzed); cni_failure
        # incidents never do: the message names the pod, not the Node the metapath ends at, so
        # message_compatible filters every record (the reference's own filter, generate_query.py:104-129)
        "stage3_reached": stage3,
        "abandoned_at_shutdown": stream.n_abandoned,
        "truncated_by_time_budget": truncated,
        "tokens": {"sampled": d["sampled_tokens"], "forced": d["forced_tokens"], "prefill": d["prefill_tokens"],
                   "recomputed_after_truncation": d["recompute_tokens"],
                   "decode_rows": d["decode_tokens"]},
        "no_hints": nh,
        "tp_sim": sim,
        # which regime the window measures: thread age (incidents each pipeline's
        # three threads carry, replayed + engine-run) and the threads' live context
        "thread_regime": {
            "replayed_incidents_per_pipeline": args.thread_age,
            "incidents_at_t0": {"min": min(age0) if age0 else 0,
                                "mean": round(sum(age0) / max(1, len(age0)), 2)},
            "context_tokens_at_t0": ctx0, "context_tokens_at_end": ctx1,
            "truncations_in_window": ctx1.get("truncations", 0) - ctx0.get("truncations", 0),
            "mean_decode_context": round(d["decode_ctx_tokens"] / max(1, d["decode_tokens"]), 1),
            "replay_s": round(age_s, 1), "warmup_s": round(warm_s, 1)},
        "engine": {"steps": d["steps"], "graph_steps": d["graph_steps"],
                   "forward_s": round(d["forward_s"], 3), "sample_s": round(d["sample_s"], 3),
                   "host_s": round(d["host_s"], 3), "evictions": d["evictions"],
                   "preemptions": d.get("preemptions", 0), "requests": d["requests"],
                   "nonfinite_rows": d.get("nonfinite_rows", 0),
                   # knob nonfinite_check: steps whose layer flags fired, and the first layer seen
                   "nonfinite_flag_steps": d.get("nonfinite_flag_steps", 0),
                   "nonfinite_first_layer": eng.stats.get("nonfinite_first_layer", -1),
                   # why the window's requests ended (a collapse to early ends shows here)
                   "ends": {k[4:]: d.get(k, 0) for k in ("end_grammar", "end_eos", "end_no_allowed", "end_cap")},
                   "decode_ctx_tokens": d["decode_ctx_tokens"], "prefill_ctx_tokens": d["prefill_ctx_tokens"],
                   # work counters of tools/window_summary.py's roofline accounting
                   "prefill_attn_pairs": d["prefill_attn_pairs"], "small_steps": d["small_steps"],
                   "small_rows": d["small_rows"], "big_rows": d["big_rows"],
                   "kv_blocks": eng.kv.num_blocks, "wait_s": round(d["wait_s"], 3),
                   "prefix_hit_tokens": d["prefix_hit_tokens"], "shared_kv_blocks": eng.kv.shared_blocks,
                   "captures": d["captures"], "capture_s": round(d["capture_s"], 3),
                   "prefill_min_tokens": eng.cfg.prefill_min_tokens,
                   "prefill_deferred_steps": d.get("prefill_deferred_steps", 0),
                   # decode-attention KV blocks read per distinct block (sampled every 32nd graph step)
                   "kv_block_reuse": round(d["kv_read_blocks_sampled"] / max(1, d["kv_unique_blocks_sampled"]), 2),
                   "admit_s": round(d["admit_s"], 3), "post_s": round(d["post_s"], 3),
                   # measured GEMM tables in use (decode dispatch; hipBLASLt solution buckets registered)
                   "gemm_dispatch": bool(getattr(eng, "gemm_dispatch", False)),
                   "blaslt_buckets": int(getattr(eng, "lib_algos", 0) or 0),
                   # gemm_big launches that ran without the split tail (a stream other than the engine's)
                   "big_tail_foreign": _tail_foreign(eng),
                   # KV host tier (--kv-host-gb): idle threads swapped out / back in the window
                   **({"swap_outs": d.get("swap_outs", 0), "swap_ins": d.get("swap_ins", 0),
                       "kv_host": eng.kv_host.report()} if getattr(eng, "kv_host", None) is not None else {}),
                   # K8SRCA_STEP_TIMING=1: host issue time vs GPU time of the forwards
                   **({k: round(d[k], 3) for k in ("eager_issue_s", "eager_gpu_s", "graph_issue_s", "graph_gpu_s")}
                      if d["eager_gpu_s"] or d["graph_gpu_s"] else {})},
        # the work behind each timed analysis (sampling varies it run to run by a few %:
        # compare A/B runs per unit of it, not by the headline alone)
        "work_per_analysis": {"decode_ctx_ktokens": round(d["decode_ctx_tokens"] / 1e3 / max(1, n_done), 1),
                              "prefill_tokens": round(d["prefill_tokens"] / max(1, n_done), 1),
                              "sampled_tokens": round(d["sampled_tokens"] / max(1, n_done), 1)},
        "throughput": {  # rank 0's engine over the timed window
            "prefill_tok_per_s": round(d["prefill_tokens"] / elapsed, 1),
            "decode_tok_per_s": round(d["decode_tokens"] / elapsed, 1),
            "sampled_tok_per_s": round(d["sampled_tokens"] / elapsed, 1),
            "forced_tok_per_s": round(d["forced_tokens"] / elapsed, 1),
            "avg_decode_batch": round(d["decode_tokens"] / max(1, d["steps"]), 1),
            "runs": len(ttft),
            "ttft_p50_s": round(ttft[len(ttft) // 2], 4) if ttft else None,
            "kv_peak_util": round(eng.kv.peak_used / max(1, eng.kv.num_blocks), 4)},
        # CPU seconds per thread group over the timed window (GIL competition with the engine thread)
        "host_cpu_s": {k: round(v - cpu0.get(k, 0.0), 2) for k, v in cpu1.items()},
        "native_threads": {"n": len(native_top), "top_cpu_s": native_top[:4], "busiest": native_busiest},
        # every rank's CPU binding (disjoint NUMA-local slices; null = unbound)
        "cpu_affinity": placements,
        "setup_s": round(setup_s, 1),
        "wall_s": round(time.perf_counter() - t_start, 1),
        "clean_shutdown": clean,
        "stages": {k: round(v["mean_ms"], 2) for k, v in tracing.snapshot().items()},
        "graph": {"device": bool(batchers),
                  "query_ms_per_analysis": round(gq.get("graph.query", 0.0) / max(1, n_done), 2),
                  "batched_requests": int(sum(b["requests"] for b in bstats)),
                  "kernel_batches": int(sum(b["launches"] for b in bstats)),
                  "max_batch": int(max([b["max_batch"] for b in bstats] or [0]))},
    }
    if getattr(eng, "tp_tune", None):
        res["tp_collectives"] = eng.tp_tune  # the per-bucket epilogue plan measured on this fabric at init
    res["sanity"] = sanity(res)
    if world > 1 and not tp_mode:
        import torch.distributed as dist
        dist.barrier()
    return res if rank == 0 else None


def parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs = ranks; without torchrun's WORLD_SIZE, bench.py spawns this many rank processes")
    p.add_argument("--preset", default=None, choices=sorted(PRESETS), help="a BASELINE.json config")
    p.add_argument("--steps", type=int, default=10, help="timed steps; one step = --quantum completed analyses per GPU")
    p.add_argument("--warmup", type=int, default=3, help="untimed steps streamed before the timer starts")
    p.add_argument("--quantum", type=int, default=16, help="completed analyses per GPU per step")
    p.add_argument("--thread-age", type=int, default=12,
                   help="prior incidents replayed into every pipeline's threads before the stream starts "
                        "(the reference reuses one set of threads for a whole batch); 12 puts every "
                        "locator / generator / analyzer thread past its first cut at the model window")
    p.add_argument("--time-budget", type=float, default=360.0,
                   help="seconds after start at which the stream stops waiting and the JSON is printed anyway "
                        "(flagged truncated_by_time_budget); 0 = none")
    p.add_argument("--no-hints-steps", type=int, default=3,
                   help="after the timed window, steps measured with the oracle hints off (0 = skip)")
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (one engine over all ranks)")
    p.add_argument("--tp-sim", type=int, default=0,
                   help="project a TP=N engine from ONE GPU: rank 0's shard at real shapes, collectives stood "
                        "in by local kernels moving the same bytes (result line: tp_sim)")
    p.add_argument("--device", default="cuda")
    p.add_argument("--same-gpu", action="store_true",
                   help="every rank on cuda:0: N DP replicas (with --kv-gb) or N TP ranks (xGMI kernels over "
                        "IPC, gloo host group) sharing one GPU -- the one-GPU rehearsal of an N-GPU job")
    # The operating point is chosen by the latency half of the metric: the
    # throughput plateau spans 96-128 concurrent analyses within ~2 % (4.67-4.77 /s,
    # profiles/r5/curve/, profiles/r5/ab_defer96/) while p50 grows with concurrency
    # (Little's law: 17.6 s at 96, 18.7 s at 100, 19.2-19.9 s at 104, 20.2 s at 112,
    # 26.9 s at 128), so the default is the point with p50 a clear second under the
    # reference's 20 s latency floor at the plateau's throughput.
    p.add_argument("--incidents", type=int, default=100,
                   help="concurrent RCA analyses (pipelines) per GPU (default: the p50 < 20 s operating point)")
    p.add_argument("--graph-nodes", type=int, default=10_000)
    p.add_argument("--no-graph-device", action="store_true",
                   help="keep the graphs on the host (default on GPU: HBM mirror + batched HIP graph kernels)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--kv-gb", type=float, default=None, help="KV pool cap (default: 85%% of free HBM)")
    p.add_argument("--kv-host-gb", type=float, default=None,
                   help="KV host tier: GB of page-locked host memory idle threads are swapped to instead of "
                        "dropped (engine/kv_offload.py; TP = 1)")
    p.add_argument("--max-context", type=int, default=None,
                   help="serving window (tokens) a thread is cut at (default: the model's own window); "
                        "reported in config.truncation")
    p.add_argument("--max-batch-tokens", type=int,
                   default=KNOBS.max_batch_tokens)
    p.add_argument("--temperature", type=float, default=0.7)
    p.add_argument("--semantic-tokens", type=int, default=192)
    p.add_argument("--explanation-tokens", type=int, default=40)
    p.add_argument("--conclusion-tokens", type=int, default=80)
    p.add_argument("--resolution-tokens", type=int, default=80)
    p.add_argument("--no-hints", action="store_true")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--no-gc-freeze", action="store_true", help="keep warm-up objects in the GC generations")
    p.add_argument("--no-prefix-sharing", action="store_true", help="do not share prompt KV pages across threads")
    return p


# One preset per BASELINE.json config; explicit flags override.
PRESETS: Dict[str, Dict[str, Any]] = {
    # "OPT-125m CPU backend, 10-node toy k8s dependency graph, single pod-crash RCA (plumbing, no GPU)"
    "opt125m-cpu-toy": dict(model="opt-125m", device="cpu", graph_nodes=10, incidents=1, quantum=1, steps=1,
                            warmup=0, no_hints_steps=0, time_budget=0, thread_age=0),
    # the headline: "RCA analyses/sec + p50 latency, Llama-3-8B backend, 10k-node graph"
    "llama3-8b-10k": dict(model="llama3-8b", graph_nodes=10_000),
    # "Llama-3-8B TP=1 bf16 on one MI355X, 1k-node synthetic k8s graph"
    "llama3-8b-1k": dict(model="llama3-8b", graph_nodes=1_000),
    # "Llama-3-8B TP=1, 100k-node synthetic graph (HIP CSR metapath BFS stress)"
    "llama3-8b-100k": dict(model="llama3-8b", graph_nodes=100_000),
    # "Llama-3-70B TP=8 over xGMI, 10k-node graph, batched multi-incident RCA" (torchrun --nproc-per-node 8)
    "llama3-70b-tp8-10k": dict(model="llama3-70b", tp=8, graph_nodes=10_000),
    # "Mixtral 8x7B MoE backend (grouped GEMM + expert all-to-all over xGMI), 10k-node graph"
    # 32k window: reaching its steady state (every thread cut at the window) takes ~30 prior
    # incidents per thread, whose re-prefill alone outlasts the time budget (12 pre-aged
    # incidents: no timed step in 360 s); 4 keeps the warm-up inside it.  And 128
    # pipelines x 3 threads x ~8k tokens exceed the KV pool left beside 94 GB of experts
    # (1.34 M tokens): 754 preemptions, 36k prefill tokens per analysis, 0.77 /s
    # (profiles/r3/presets/mixtral_128.json) -- 48 concurrent analyses fit
    "mixtral-10k": dict(model="mixtral-8x7b", graph_nodes=10_000, thread_age=4, incidents=48, quantum=6),
    # the same model served with an 8k window (config.truncation.max_context): threads are cut
    # where Llama-3's are, the steady state is reachable (12 pre-aged incidents) and 64 pipelines'
    # KV fits beside the experts -- 1.74 /s at p50 30.5 s, 0 preemptions (profiles/r5/mixtral_8k/)
    # Llama-3-70B on ONE GPU (TP = 1): 141 GB of weights leave ~413k tokens of KV, 20 pipelines' threads;
    # with idle threads swapped to a 140 GB host tier (engine/kv_offload.py) 48 pipelines run without
    # re-prefills: 0.668 analyses/s vs 0.486 at 20 and 0.469 at 40 without it (profiles/r6/kvhost/)
    "llama3-70b-tp1-host": dict(model="llama3-70b", incidents=48, quantum=4, kv_host_gb=140.0),
    # the same two Mixtral configs at twice the concurrency, idle threads on the KV host tier
    # (profiles/r6/kvhost/): 32k window 1.33 -> 1.62 /s at 96 (p50 28.9 -> 47.7 s); 8k window
    # 1.74 -> 2.39 /s at 128 (p50 30.5 -> 58.9 s) -- throughput per GPU for latency
    "mixtral-10k-host": dict(model="mixtral-8x7b", graph_nodes=10_000, thread_age=4, incidents=96, quantum=12,
                             kv_host_gb=120.0),
    "mixtral-10k-8k-host": dict(model="mixtral-8x7b", graph_nodes=10_000, max_context=8192, incidents=128,
                                quantum=16, kv_host_gb=100.0),
    "mixtral-10k-8k": dict(model="mixtral-8x7b", graph_nodes=10_000, max_context=8192, incidents=64, quantum=8),
}


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, argv: List[str]) -> int:
    """``bench.py --gpus N`` without a launcher: start N rank processes (one per
    GPU, torchrun's env contract, rendezvous on 127.0.0.1) and wait for them.
    Runs before anything in this process touches the GPU; the ranks are
    children, never an exec of this process.  Rank 0 prints the JSON line."""
    import subprocess
    port = _free_port()
    script = os.path.abspath(sys.argv[0]) if sys.argv and sys.argv[0].endswith(".py") else None
    cmd = [sys.executable, script] if script else [sys.executable, "-m", "k8s_llm_rca_amd.bench.rca_bench"]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd + list(argv), env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for pr in list(pending):
                code = pr.poll()
                if code is None:
                    continue
                pending.remove(pr)
                if code != 0:
                    rc = rc or code
                    for other in pending:  # one rank died: the collective would hang the rest
                        other.terminate()
            time.sleep(0.2)
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    return rc


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    p = parser()
    pre, _ = p.parse_known_args(argv)
    if pre.preset:
        p.set_defaults(**PRESETS[pre.preset])
    args = p.parse_args(argv)
    if args.gpus and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.tp > world:
        logging.warning("--tp %d > %d ranks: running TP=%d", args.tp, world, world)
        args.tp = world
    res = run(args)
    rc = 0
    if res is not None:
        print(json.dumps(res), flush=True)
        if not res["sanity"]["ok"]:
            print(f"[bench] INVALID window: {'; '.join(res['sanity']['reasons'])}", file=sys.stderr, flush=True)
            rc = 3
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        # Orderly teardown: no rank exits while a peer's gloo/RCCL background
        # threads still reference it (an abort at exit fails the torchrun job).
        dist.barrier()
        dist.destroy_process_group()
    return rc


def exit_now(rc: int) -> None:
    """Exit normally when every pipeline thread has ended (profilers such as
    rocprofv3 flush their output at exit); if one is still parked on a run,
    leave without interpreter teardown instead (tearing the runtime down under
    it aborts the process, exit 134, after the JSON line)."""
    import threading
    sys.stdout.flush()
    sys.stderr.flush()
    if any(t.is_alive() and t.name == "rca-stream" for t in threading.enumerate()):
        os._exit(rc)
    sys.exit(rc)


if __name__ == "__main__":
    exit_now(main())
