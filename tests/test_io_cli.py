"""Graph persistence, CLI drivers and assistant-service state round trips."""
import json
import os

import pytest

from k8s_llm_rca_amd.api.service import AssistantService, ScriptedBackend
from k8s_llm_rca_amd.graph import io as GIO
from k8s_llm_rca_amd.graph.cypher import Executor
from k8s_llm_rca_amd.graph.synth import generate_cluster


def test_graph_roundtrip(tmp_path):
    c = generate_cluster(1500, 5, seed=3)
    p = str(tmp_path / "g.jsonl.gz")
    GIO.save_graph(c.stategraph, p)
    g2 = GIO.load_graph(p)
    assert g2.num_nodes == c.stategraph.num_nodes and g2.num_edges == c.stategraph.num_edges
    q = "MATCH (e:EVENT) WHERE e.message CONTAINS $m RETURN e.timestamp AS t"
    for inc in c.incidents:
        a = Executor(c.stategraph).run(q, {"m": inc.message})
        b = Executor(g2).run(q, {"m": inc.message})
        assert [r["t"] for r in a] == [r["t"] for r in b]
    GIO.save_incidents_csv(c.incidents, str(tmp_path / "i.csv"))
    back = GIO.load_incidents_csv(str(tmp_path / "i.csv"))
    assert [i.message for i in back] == c.messages and back[0].path_kinds == c.incidents[0].path_kinds


def test_cli_run_and_resume(tmp_path, capsys):
    from k8s_llm_rca_amd.cli import main
    d = str(tmp_path / "c")
    assert main(["gen-graph", "--graph-nodes", "1500", "--incidents", "4", "--out", d]) == 0
    out = str(tmp_path / "res.json")
    assert main(["run", "--graph-dir", d, "--backend", "oracle", "--output", out, "--limit", "2"]) == 0
    assert main(["run", "--graph-dir", d, "--backend", "oracle", "--output", out, "--resume"]) == 0
    from k8s_llm_rca_amd.pipeline.rca import read_results
    res = read_results(out)
    assert len(res) == 4 and len({r["error_message"] for r in res}) == 4
    spans = json.load(open(out + ".spans.json"))
    assert "rca.analyze" in spans["stages"] and spans["summary"]["analyses"] == 2


def test_service_state_roundtrip():
    svc = AssistantService(ScriptedBackend(lambda rs: "reply"))
    a = svc.create_assistant("ins", "n", "m")
    t = svc.create_thread()
    svc.add_message(t.id, "hi")
    r = svc.create_run(t.id, a.id)
    svc.wait_run(r.id, 5)
    st = json.loads(json.dumps(svc.export_state()))
    svc2 = AssistantService(ScriptedBackend(lambda rs: "x"))
    svc2.import_state(st)
    assert svc2.retrieve_assistant(a.id).instructions == "ins"
    msgs = svc2.list_messages(t.id, order="asc").data
    assert [m.role for m in msgs] == ["user", "assistant"] and msgs[1].text == "reply"


def test_cli_token_probe(capsys):
    import json as _json
    from k8s_llm_rca_amd.cli import main
    assert main(["token-probe", "--backend", "oracle", "--graph-nodes", "100"]) == 0
    usage = _json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert usage["total_tokens"] == usage["prompt_tokens"] + usage["completion_tokens"] > 0


@pytest.mark.slow
def test_bench_dp2_torchrun_cpu_contract(tmp_path):
    """The driver's multi-GPU contract on CPU: torchrun, 2 ranks (gloo), one
    JSON line from rank 0 with the whole-job aggregate."""
    import json as _json
    import os
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--device", "cpu", "--model", "tiny-llama", "--incidents", "2", "--graph-nodes", "300",
           "--quantum", "1", "--no-hints-steps", "0", "--time-budget", "0"]
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = _json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 1 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 4 and d["value"] > 0 and d["errors"] == 0


@pytest.mark.slow
def test_bench_self_spawns_ranks_cpu(tmp_path):
    """``bench.py --gpus 2`` without torchrun starts its 2 ranks itself and
    reports the world RCCL/gloo saw; timing covers exactly K quanta."""
    import json as _json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--quantum", "1", "--device", "cpu", "--model", "tiny-llama", "--incidents", "2", "--graph-nodes", "300",
           "--no-hints-steps", "0", "--time-budget", "0"]  # no budget: a loaded CI box must not truncate
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=root, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = _json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["steps"] == 2
    assert d["analyses_timed"] == 4 and d["errors"] == 0 and not d["truncated_by_time_budget"]
    # the line says which timed analyses reached stage 3
    s3 = d["stage3_reached"]
    assert 0.0 <= s3["fraction"] <= 1.0 and sum(v[1] for v in s3["by_fault"].values()) == d["analyses_timed"] // 2
    assert abs(d["config"]["graph_nodes"] - 300) <= 0.2 * 300
    # the reference's thread regime: every pipeline's threads carry the replayed
    # incidents plus at least one engine-run incident when the timer starts
    reg = d["thread_regime"]
    assert reg["replayed_incidents_per_pipeline"] == 12 and reg["incidents_at_t0"]["min"] >= 13
    assert reg["context_tokens_at_t0"]["threads"] == 6 and reg["mean_decode_context"] > 0


def test_synth_graph_size_tracks_target():
    """The bench's graph is the size it claims, faults included."""
    for target, n_inc in ((1000, 100), (10_000, 600), (10_000, 1000)):
        c = generate_cluster(target, n_inc, seed=5)
        assert abs(c.stategraph.num_nodes - target) <= 0.05 * target, (target, n_inc, c.stategraph.num_nodes)
        assert len(c.incidents) == n_inc


def test_cli_stage_drivers(tmp_path, capsys):
    """The reference's per-stage drivers (test_find_metapath.py,
    test_generate_query.py, test_check_state.py) as CLI subcommands."""
    from k8s_llm_rca_amd.cli import main
    from k8s_llm_rca_amd.graph.io import load_incidents_csv
    d = str(tmp_path / "c")
    assert main(["gen-graph", "--graph-nodes", "600", "--incidents", "12", "--out", d]) == 0
    capsys.readouterr()
    inc = next(i for i in load_incidents_csv(d + "/incidents.csv") if i.fault == "secret_missing")
    base = ["--backend", "oracle", "--graph-dir", d, "--message", inc.message]
    assert main(["locate", *base]) == 0
    out = capsys.readouterr().out
    j = json.loads(out[out.index("{"):])
    assert j["srcKind"] == "Pod" and j["metapaths"]
    mp = ("\n    HasEvent, Event, EVENT, metadata_uid;\n    ReferInternal, Event, Pod, involvedObject_uid;\n"
          "    ReferInternal, Pod, Secret, spec_volumes_secret_secretName;\n")
    assert main(["query", *base, "--metapath", mp]) == 0
    assert "MATCH (evt:EVENT)" in capsys.readouterr().out
    assert main(["state", *base, "--kind", "Pod", "--id", inc.involved_id, "--timestamp", inc.timestamp]) == 0
    assert capsys.readouterr().out.strip()


@pytest.mark.slow
def test_bench_tp2_cpu(tmp_path):
    """``bench.py --gpus 2 --tp 2``: one TP=2 engine (rank 0 schedules, rank 1
    serves the step channel) runs the whole RCA stream; parallelism reads tp2
    and the aggregate counts ONE engine's analyses."""
    import json as _json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--tp", "2", "--steps", "2", "--warmup", "1",
           "--quantum", "1", "--device", "cpu", "--model", "tiny-llama-g8", "--incidents", "2", "--graph-nodes", "300",
           "--no-hints-steps", "0", "--time-budget", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=root, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = _json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "tp2" and d["steps"] == 2
    assert d["analyses_timed"] == 2 and d["errors"] == 0
