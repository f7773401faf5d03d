"""Command-line drivers (the reference's ``test_*.py`` scripts as subcommands).

``python -m k8s_llm_rca_amd <command>``:

* ``gen-graph``  synthetic metagraph + stategraph (JSONL) + incidents CSV
* ``run``        batch RCA: CSV of error messages -> concatenated pretty-JSON
                 results (``test_with_file.py``); ``--resume`` skips messages
                 already in the output; ``--concurrency`` runs that many
                 pipelines against one engine
* ``locate``     stage 1 only: srcKind + locator + metapaths (``test_find_metapath.py``)
* ``query``      stage 2 only for one metapath string (``test_generate_query.py``)
* ``state``      stage 3 only for one entity (``test_check_state.py``)
* ``token-probe`` token accounting over two runs (``test_token.py``)
* ``serve``      OpenAI-Assistants-shaped REST API over the engine, plus the
                 Neo4j HTTP ``/db/{metagraph,stategraph}/tx/commit`` endpoint over
                 the graphs (api/http.py);
                 ``run --server URL`` drives a remote server instead of an
                 in-process engine

Backends: ``engine`` (MI355X LLM engine, default), ``opt-cpu`` (OPT-125m
plumbing backend on CPU, BASELINE config 1) and ``oracle`` (scripted replies
from the grammar hints; no model).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from typing import List, Optional

log = logging.getLogger("k8s_llm_rca_amd")


def _load_cluster(args):
    from .graph import io as GIO
    from .graph.schema import build_metagraph
    from .graph.synth import generate_cluster

    if args.graph_dir:
        meta_p = os.path.join(args.graph_dir, "metagraph.jsonl")
        meta = GIO.load_graph(meta_p, "metagraph") if os.path.exists(meta_p) else build_metagraph()
        state = GIO.load_graph(os.path.join(args.graph_dir, "stategraph.jsonl"), "stategraph")
        inc_p = os.path.join(args.graph_dir, "incidents.csv")
        incidents = GIO.load_incidents_csv(inc_p) if os.path.exists(inc_p) else []
        return meta, state, incidents
    c = generate_cluster(args.graph_nodes, args.incidents, seed=args.seed)
    return c.metagraph, c.stategraph, c.incidents


def _service(args):
    from .api.service import AssistantService, ScriptedBackend, set_default_service

    if args.backend == "oracle":
        from .engine.grammar import hinted_render
        svc = AssistantService(ScriptedBackend(
            lambda rs: hinted_render(rs.response_format, "inspected") if rs.response_format is not None else "ok"))
        set_default_service(svc)
        return svc, None
    import torch
    from .engine.backend import EngineBackend
    from .engine.engine import EngineConfig, LLMEngine

    if args.backend == "opt-cpu":
        cfg = EngineConfig(model="opt-125m", device="cpu", dtype=torch.float32, num_blocks=2048, block_size=64,
                           max_batch_tokens=2048, max_context=2048)
    else:
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        cfg = EngineConfig(model=args.model, device=dev, dtype=torch.bfloat16 if dev == "cuda" else torch.float32,
                           kv_max_gb=args.kv_gb, num_blocks=None if dev == "cuda" else 1024,
                           weights=args.weights, tokenizer=args.tokenizer)
    eng = LLMEngine(cfg)
    eng.start()
    svc = AssistantService(EngineBackend(eng))
    set_default_service(svc)
    return svc, eng


def _budget(args):
    from .pipeline.formats import GenerationBudget
    return GenerationBudget(semantic_tokens=args.semantic_tokens)


def cmd_gen_graph(args) -> int:
    from .graph import io as GIO
    from .graph.synth import generate_cluster

    os.makedirs(args.out, exist_ok=True)
    c = generate_cluster(args.graph_nodes, args.incidents, seed=args.seed)
    GIO.save_graph(c.metagraph, os.path.join(args.out, "metagraph.jsonl"))
    GIO.save_graph(c.stategraph, os.path.join(args.out, "stategraph.jsonl"))
    GIO.save_incidents_csv(c.incidents, os.path.join(args.out, "incidents.csv"))
    print(json.dumps({"out": args.out, **c.stategraph.stats(), "incidents": len(c.incidents)}))
    return 0


def cmd_run(args) -> int:
    from .api.graph import GraphQueryExecutor
    from .graph.io import load_incidents_csv
    from .pipeline.rca import RCAConfig, RCAPipeline, read_messages_csv, read_results, run_batch

    meta, state, incidents = _load_cluster(args)
    if args.messages:
        try:
            truths = load_incidents_csv(args.messages)
            messages = [t.message for t in truths]
            if not any(t.src_kind for t in truths):
                truths = None
        except Exception:  # noqa: BLE001 - plain one-column CSV
            messages, truths = read_messages_csv(args.messages), None
    else:
        messages, truths = [i.message for i in incidents], incidents
    if args.limit:
        messages = messages[: args.limit]
        truths = truths[: args.limit] if truths else None
    if args.resume and args.output and os.path.exists(args.output):
        done = {r.get("error_message") for r in read_results(args.output)}
        keep = [i for i, m in enumerate(messages) if m not in done]
        messages = [messages[i] for i in keep]
        truths = [truths[i] for i in keep] if truths else None
        log.info("resume: %d messages left", len(messages))
    if args.device_graph:
        import torch
        if torch.cuda.is_available():
            from .graph.device import to_device
            to_device(state, "cuda")
    if args.server:
        from .api.http import RemoteAssistantService
        svc, eng = RemoteAssistantService(args.server), None
    else:
        svc, eng = _service(args)
    cfg = RCAConfig(model=args.model, hints=args.hints, budget=_budget(args))
    meta_qe, state_qe = GraphQueryExecutor(meta), GraphQueryExecutor(state)
    t0 = time.time()
    st = run_batch(lambda: RCAPipeline(svc, meta_qe, state_qe, cfg), messages, concurrency=args.concurrency,
                   truths=truths, output_path=args.output)
    wall = time.time() - t0
    if eng is not None:
        eng.stop()
    summary = {"analyses": len(st.results), "completed": st.n_ok, "wall_s": round(wall, 2),
               "analyses_per_s": round(st.analyses_per_s, 3),
               "p50_latency_s": round(st.pct(0.5), 3), "p90_latency_s": round(st.pct(0.9), 3),
               "errors": len(st.errors), "output": args.output}
    if args.output:  # per-stage spans (and engine counters) next to the result file
        from .utils import tracing
        spans = {"stages": tracing.snapshot(), "summary": summary}
        if eng is not None:
            spans["engine"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()}
            spans["engine"]["kv_peak_util"] = round(eng.kv.peak_used / max(1, eng.kv.num_blocks), 4)
        with open(args.output + ".spans.json", "w") as f:
            json.dump(spans, f, indent=1)
    if args.state_out and hasattr(svc, "export_state"):
        with open(args.state_out, "w") as f:
            json.dump(svc.export_state(), f)
    print(json.dumps(summary))
    if args.output is None:
        for r in st.results:
            print(json.dumps(r, indent=4))
    return 0


def cmd_locate(args) -> int:
    from .api.graph import GraphQueryExecutor
    from .pipeline import find_metapath as FM
    from .pipeline import formats as F

    meta, state, incidents = _load_cluster(args)
    svc, eng = _service(args)
    mq, sq = GraphQueryExecutor(meta), GraphQueryExecutor(state)
    msg = args.message or incidents[0].message
    truth = next((i for i in incidents if i.message == msg), None)
    native, external = FM.find_native_external_kinds(mq)
    tmpl = FM.build_prompt_template(native, external)
    loc = FM.setup_root_cause_locator(svc, args.model)
    src = FM.find_srcKind(sq, msg)
    t = (truth.src_kind, truth.dest_kind, truth.path_kinds) if (truth and args.hints) else None
    dr = FM.find_destKind_relevantResources(msg, src, tmpl, loc, F.locator_grammar(native + external, src,
                                                                                     _budget(args), t))
    inter = FM.intermediate_kinds(dr.get("RelevantResources", []), src, dr["DestinationKind"], native, external)
    mps = FM.find_metapath(mq, src, dr["DestinationKind"], inter)
    print(json.dumps({"srcKind": src, "locator": dr, "metapaths": [
        [[r.type, r["srcKind"], r["destKind"], r["key"]] for r in p.relationships] for p in mps]}, indent=2))
    if eng is not None:
        eng.stop()
    return 0


def cmd_query(args) -> int:
    from .api.graph import GraphQueryExecutor
    from .pipeline import formats as F
    from .pipeline import generate_query as GQ

    meta, state, incidents = _load_cluster(args)
    svc, eng = _service(args)
    sq = GraphQueryExecutor(state)
    gen = GQ.setup_cypher_generator(svc, args.model)
    msg = args.message or incidents[0].message
    q = GQ.generate_cypher_query(args.metapath, msg, gen, F.cypher_grammar(args.metapath, msg, args.hints))
    recs = GQ.run_and_filter_query(sq, q)
    print(q)
    for r in recs:
        print(r)
    if eng is not None:
        eng.stop()
    return 0


def cmd_state(args) -> int:
    from .api.graph import GraphQueryExecutor
    from .pipeline import check_state as CS
    from .pipeline import formats as F

    meta, state, incidents = _load_cluster(args)
    svc, eng = _service(args)
    sq = GraphQueryExecutor(state)
    an = CS.setup_state_semantic_analyzer(svc, args.model)
    q = CS.find_strict_states(args.kind, args.id, args.timestamp)
    for c in CS.check_states_existence_and_semantic(sq, q, an, args.message or "", F.semantic_grammar(_budget(args))):
        print(c)
    if eng is not None:
        eng.stop()
    return 0


def cmd_token_probe(args) -> int:
    """The reference's token-accounting probe (test_token.py:1-49): a tutor
    assistant, two messages with a run each, then get_token_usage over the
    window.  The reference sleeps 60 s per run and uses int() second bounds;
    here each run is awaited and the window is taken in float seconds, so the
    usage of fast runs is not lost."""
    from .api.assistant import GenericAssistant
    svc, eng = _service(args)
    tutor = GenericAssistant(svc)
    tutor.create_assistant("You are a personal math tutor. When asked a question, write and run Python code to "
                           "answer the question.", "math-tutor-2", args.model)
    tutor.create_thread()
    print(tutor.assistant.id)
    print(tutor.thread.id)
    start = time.time()
    for m in ("what is the area of a circle with diameter 4", "what is the result for x in 'x + 3 = 15'?"):
        tutor.add_message(m)
        tutor.run_assistant(max_tokens=args.max_tokens)
        print("run assistant ...")
        tutor.wait_get_last_k_message(1)
    usage = tutor.get_token_usage(start, time.time() + 1e-3, 5)
    print(json.dumps(usage))
    if eng is not None:
        eng.stop()
    return 0


def cmd_serve(args) -> int:
    import uvicorn
    from .api.http import create_app
    svc, eng = _service(args)
    meta, state, _ = _load_cluster(args)
    try:
        uvicorn.run(create_app(svc, eng, graphs={"metagraph": meta, "stategraph": state}), host=args.host,
                    port=args.port, log_level="warning")
    finally:
        if eng is not None:
            eng.stop()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="k8s_llm_rca_amd", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)

    def common(sp):
        sp.add_argument("--graph-dir", default=None, help="directory with metagraph/stategraph JSONL + incidents.csv")
        sp.add_argument("--graph-nodes", type=int, default=10_000)
        sp.add_argument("--incidents", type=int, default=16)
        sp.add_argument("--seed", type=int, default=0)
        sp.add_argument("--backend", choices=["engine", "opt-cpu", "oracle"], default="engine")
        sp.add_argument("--model", default="llama3-8b")
        sp.add_argument("--kv-gb", type=float, default=None)
        sp.add_argument("--weights", default=None, help="HF checkpoint dir (config.json + *.safetensors)")
        sp.add_argument("--tokenizer", default=None, help="tokenizer.json (default: the checkpoint's)")
        sp.add_argument("--hints", action=argparse.BooleanOptionalAction, default=True)
        sp.add_argument("--semantic-tokens", type=int, default=192)
        sp.add_argument("-v", "--verbose", action="store_true")

    sp = sub.add_parser("gen-graph")
    common(sp)
    sp.add_argument("--out", required=True)
    sp.set_defaults(fn=cmd_gen_graph)
    sp = sub.add_parser("run")
    common(sp)
    sp.add_argument("--messages", default=None, help="CSV, first column = error message (header skipped)")
    sp.add_argument("--output", default=None, help="append results here (concatenated pretty JSON)")
    sp.add_argument("--resume", action="store_true")
    sp.add_argument("--limit", type=int, default=0)
    sp.add_argument("--concurrency", type=int, default=1)
    sp.add_argument("--device-graph", action="store_true", help="mirror the stategraph to HBM")
    sp.add_argument("--state-out", default=None, help="save assistants/threads JSON for resume")
    sp.add_argument("--server", default=None, help="base URL of a `serve` instance (remote engine)")
    sp.set_defaults(fn=cmd_run)
    sp = sub.add_parser("locate")
    common(sp)
    sp.add_argument("--message", default=None)
    sp.set_defaults(fn=cmd_locate)
    sp = sub.add_parser("query")
    common(sp)
    sp.add_argument("--message", default=None)
    sp.add_argument("--metapath", required=True)
    sp.set_defaults(fn=cmd_query)
    sp = sub.add_parser("state")
    common(sp)
    sp.add_argument("--kind", required=True)
    sp.add_argument("--id", required=True)
    sp.add_argument("--timestamp", required=True)
    sp.add_argument("--message", default=None)
    sp.set_defaults(fn=cmd_state)
    sp = sub.add_parser("token-probe")
    common(sp)
    sp.add_argument("--max-tokens", type=int, default=32)
    sp.set_defaults(fn=cmd_token_probe)
    sp = sub.add_parser("serve")
    common(sp)
    sp.add_argument("--host", default="127.0.0.1")
    sp.add_argument("--port", type=int, default=8000)
    sp.set_defaults(fn=cmd_serve)
    args = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO if args.verbose else logging.WARNING)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
