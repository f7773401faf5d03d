"""TP push epilogue (csrc/kernels/allreduce.hip "push epilogue", gemm_stream.hip
k8s_gemm_stream_push): the row-parallel GEMM stores its output straight into
the all-reduce's slots and raises per-strip flags; the fused all-reduce +
residual add + RMSNorm waits on those flags and sums its local slots.

Checked bit-for-bit against the staged (pull) path -- the same GEMM, then
``XgmiAllReduce.addnorm`` -- at the kernel level with two processes sharing
cuda:0 (real IPC mappings, real flag waits), on the tp-sim loopback at world 8,
and end to end: a TP=2 engine (graph-replayed decode) generates the same tokens
with and without the push epilogue, one-shot and two-shot."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SHARED_GPU_AR_BLOCKS = 32  # tests/test_tp_gpu.py: ranks share one GPU
H, K = 8192, 1024
# (T, cfg, splits, mode): LDS-DMA 64- and 128-column strips, split-K reduce pass, one- and two-shot
CASES = [(16, 15, 1, 1), (64, 14, 1, 2), (128, 14, 2, 2), (200, 13, 1, 2), (96, 23, 1, 1), (32, 14, 2, 1),
         (128, 13, 1, 1), (256, 13, 2, 2)]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _operands(world):
    g = torch.Generator().manual_seed(0)
    res0 = torch.randn(256, H, generator=g).bfloat16()
    nw = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
    xs = [torch.randn(256, K, generator=torch.Generator().manual_seed(10 + p)).bfloat16() for p in range(world)]
    ws = [(0.03 * torch.randn(H, K, generator=torch.Generator().manual_seed(20 + p))).bfloat16() for p in range(world)]
    return res0, nw, xs, ws


def _run_cases(car, rank, world, sim=False):
    from k8s_llm_rca_amd.ops import linear as LIN
    res0, nw, xs, ws = _operands(world)
    nw = nw.cuda()
    out = []
    for T, cfg, splits, mode in CASES:
        assert car.push_ok(H, T, mode), (T, mode)
        x, w = xs[rank][:T].cuda(), ws[rank].cuda()
        r1, r2, r3 = (res0[:T].cuda().clone() for _ in range(3))
        y1, y2, y3 = (torch.empty(T, H, dtype=torch.bfloat16, device="cuda") for _ in range(3))
        part = LIN.gemm_stream(x, w, cfg, splits)
        car.addnorm(part, r1, nw, y1, 1e-5, mode)                        # staged (pull)
        car.linear_push_addnorm(x, w, r2, nw, y2, 1e-5, cfg, splits, mode)  # push, epoch E + 1
        car.linear_push_addnorm(x, w, r3, nw, y3, 1e-5, cfg, splits, mode)  # push, the other parity
        torch.cuda.synchronize()
        row = {"case": (T, cfg, splits, mode), "same": bool(torch.equal(r1, r2) and torch.equal(y1, y2)),
               "same_parity": bool(torch.equal(r2, r3) and torch.equal(y2, y3))}
        if not sim:  # fp32 reference of the whole TP sum (every rank's operands are reproducible here)
            tot = sum(xs[p][:T].float() @ ws[p].float().T for p in range(world))
            r = tot + res0[:T].float()
            y = r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float().cpu()
            row["err_res"] = float((r2.float().cpu() - r).abs().max() / r.abs().max())
            row["err_y"] = float((y2.float().cpu() - y).abs().max() / y.abs().max())
        out.append(row)
    return out


def _push_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = XgmiAllReduce(dist.group.WORLD, max_bytes=8 << 20, timeout_s=60.0, max_blocks=SHARED_GPU_AR_BLOCKS)
    rows = _run_cases(car, rank, world)
    status = car.status()
    car.close()
    torch.save({"rows": rows, "status": status}, os.path.join(out_dir, f"push{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_push_epilogue_bit_identical_two_processes_sharing_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_push_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"push{r}.pt"), weights_only=True) for r in range(2)]
    for r in res:
        assert r["status"] == 0
        for row in r["rows"]:
            assert row["same"] and row["same_parity"], row
            assert row["err_res"] < 1e-2 and row["err_y"] < 2e-2, row


def test_push_epilogue_bit_identical_loopback_world8():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from k8s_llm_rca_amd.parallel.tpsim import LoopbackAR
    car = LoopbackAR(8, 16 << 20)
    try:
        rows = _run_cases(car, 0, 8, sim=True)
    finally:
        car.close()
    assert all(r["same"] and r["same_parity"] for r in rows), rows


def _engine_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.ops import layer_exec as LE
    from k8s_llm_rca_amd.parallel import xgmi
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    from k8s_llm_rca_amd.knobs import set_knob
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    # this test forces each (mode, push) form itself: no init-time fabric tuning
    set_knob("tp_autotune", False)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD)
    pc.custom_ar = xgmi.XgmiAllReduce(dist.group.WORLD, max_bytes=8 << 20, timeout_s=60.0,
                                      max_blocks=SHARED_GPU_AR_BLOCKS)
    one_shot_max = xgmi.ONE_SHOT_MAX
    LE._tp_push_force = True  # tiny-llama's o / down onto the stream GEMM (LDS-DMA / split-K)
    res = {}
    for two_shot in (False, True):
        xgmi.ONE_SHOT_MAX = 0 if two_shot else one_shot_max
        for push in (False, True):
            LE._tp_push = push
            cfg = EngineConfig(model="tiny-llama", device="cuda:0", num_blocks=64, block_size=64,
                               max_batch_tokens=256, temperature=0.0, use_graphs=True)
            model = LlamaModel(get_config("tiny-llama"), "cuda:0", torch.bfloat16, pc, seed=5, init_mode="full_slice")
            eng = LLMEngine(cfg, pc, model=model)
            torch.cuda.synchronize()
            dist.barrier()
            if rank > 0:
                eng.serve_worker()
            else:
                outs = {}
                for i in range(3):
                    sid = eng.new_sequence()
                    toks = eng.tok.system_prefix("sys") + eng.tok.message("user", "message %d " % i * (3 + 4 * i)) \
                        + eng.tok.header("assistant")
                    eng.submit(sid, toks, None, 20, temperature=0.0, seed=3,
                               on_done=lambda g, st, i=i: outs.__setitem__(i, g))
                eng.run_until_idle()
                eng.stop_workers()
                ex = model._exec
                res[(two_shot, push)] = {"outs": outs, "graph_steps": eng.stats["graph_steps"],
                                         "ar_push": int(ex.st.ar_push) if ex is not None else -1,
                                         "ar_mode": int(ex.st.ar_mode) if ex is not None else -1}
            torch.cuda.synchronize()
            dist.barrier()
            del eng, model
    xgmi.ONE_SHOT_MAX = one_shot_max
    status = pc.custom_ar.status()
    pc.custom_ar.close()
    if rank == 0:
        res["status"] = status
        torch.save(res, os.path.join(out_dir, "eng.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_push_epilogue_tp2_engine_matches_staged_path():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_engine_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "eng.pt"), weights_only=True)
    assert res["status"] == 0
    for two_shot in (False, True):
        pull, push = res[(two_shot, False)], res[(two_shot, True)]
        assert pull["ar_push"] == 0 and push["ar_push"] == 1, (pull, push)
        assert push["ar_mode"] == (2 if two_shot else 1)
        assert push["graph_steps"] > 0
        assert all(v is not None and len(v) == 20 for v in push["outs"].values())
        assert push["outs"] == pull["outs"]
