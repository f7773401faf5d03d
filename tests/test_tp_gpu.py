"""TP fast path on the GPU (B14 + engine): processes sharing cuda:0.

The box has one GPU, so two TP ranks are two processes on cuda:0 with a gloo
group for the host step channel and the sampling all-gather, and the custom
xGMI all-reduce (IPC buffers, device-side epochs) for every row-parallel
output -- the capturable path that lets TP decode steps replay HIP graphs.
The graph-replayed TP=2 engine must generate exactly what the eager TP=2
engine generates (same kernels, same order), and the native layer executor
must run (TP all-reduce inside k8s_llama_layers)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD)
    pc.custom_ar = XgmiAllReduce(dist.group.WORLD, max_bytes=8 << 20, timeout_s=20.0)
    res = {}
    for graphs in (False, True):
        cfg = EngineConfig(model="tiny-llama", device="cuda:0", num_blocks=64, block_size=64, max_batch_tokens=256,
                           temperature=0.0, use_graphs=graphs)
        model = LlamaModel(get_config("tiny-llama"), "cuda:0", torch.bfloat16, pc, seed=5, init_mode="full_slice")
        eng = LLMEngine(cfg, pc, model=model)
        if rank > 0:
            eng.serve_worker()
        else:
            outs = {}
            for i in range(5):
                sid = eng.new_sequence()
                toks = eng.tok.system_prefix("sys") + eng.tok.message("user", "message %d " % i * (3 + 4 * i)) + \
                    eng.tok.header("assistant")
                eng.submit(sid, toks, None, 24, temperature=0.0 if i % 2 == 0 else 0.8, seed=3,
                           on_done=lambda g, st, i=i: outs.__setitem__(i, g))
            eng.run_until_idle()
            eng.stop_workers()
            res[graphs] = {"outs": outs, "graph_steps": eng.stats["graph_steps"], "exec": model._exec is not None}
        torch.cuda.synchronize()
        dist.barrier()
        del eng, model
    status = pc.custom_ar.status()
    pc.custom_ar.close()
    if rank == 0:
        res["status"] = status
        torch.save(res, os.path.join(out_dir, "r.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_tp2_graph_replay_matches_eager_processes_sharing_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "r.pt"), weights_only=True)
    assert res["status"] == 0
    eager, graph = res[False], res[True]
    assert eager["graph_steps"] == 0 and graph["graph_steps"] > 0
    assert graph["exec"] and eager["exec"]
    assert eager["outs"] == graph["outs"] and all(v is not None and len(v) == 24 for v in graph["outs"].values())
