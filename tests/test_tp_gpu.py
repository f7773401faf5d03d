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

# two ranks share cuda:0: cap the xGMI collectives' grids so a rank's blocks spinning
# for its peer never hold every CU the peer's next kernel needs (XgmiAllReduce max_blocks)
SHARED_GPU_AR_BLOCKS = 32


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
    # generous: inside a long GPU suite a rank's first step (lazy code-object and library
    # initialisation) can lag its peer's by seconds; the stall tests below use 1 s on purpose
    pc.custom_ar = XgmiAllReduce(dist.group.WORLD, max_bytes=8 << 20, timeout_s=60.0, max_blocks=SHARED_GPU_AR_BLOCKS)
    res = {}
    for graphs in (False, True):
        cfg = EngineConfig(model="tiny-llama", device="cuda:0", num_blocks=64, block_size=64, max_batch_tokens=256,
                           temperature=0.0, use_graphs=graphs)
        model = LlamaModel(get_config("tiny-llama"), "cuda:0", torch.bfloat16, pc, seed=5, init_mode="full_slice")
        eng = LLMEngine(cfg, pc, model=model)
        torch.cuda.synchronize()
        dist.barrier()  # both engines built before rank 0's first collective starts its clock
        # pass 0 captures every decode bucket; pass 1 replays the same work and, on
        # the worker, runs under torch's sync checker: a worker step never waits
        # for its own GPU (its sampling winners travel over the xGMI all-to-all)
        for p in range(2 if graphs else 1):
            if rank > 0:
                if p == 1:
                    torch.cuda.set_sync_debug_mode("error")
                eng.serve_worker()
                torch.cuda.set_sync_debug_mode(0)
            else:
                outs = {}
                for i in range(5):
                    sid = eng.new_sequence()
                    toks = eng.tok.system_prefix("sys") + eng.tok.message("user", "message %d " % i * (3 + 4 * i)) \
                        + eng.tok.header("assistant")
                    eng.submit(sid, toks, None, 24, temperature=0.0 if i % 2 == 0 else 0.8, seed=3,
                               on_done=lambda g, st, i=i: outs.__setitem__(i, g))
                eng.run_until_idle()
                eng.stop_workers()
                res[(graphs, p)] = {"outs": outs, "graph_steps": eng.stats["graph_steps"],
                                    "exec": model._exec is not None}
            dist.barrier()
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
    eager, graph, again = res[(False, 0)], res[(True, 0)], res[(True, 1)]
    assert eager["graph_steps"] == 0 and graph["graph_steps"] > 0
    assert graph["exec"] and eager["exec"]
    assert eager["outs"] == graph["outs"] and all(v is not None and len(v) == 24 for v in graph["outs"].values())
    # the sync-checked pass: same greedy tokens (sampled rows differ: the noise is
    # keyed by the new sequences' ids), every run complete
    assert all(again["outs"][i] == graph["outs"][i] for i in (0, 2, 4))
    assert all(v is not None and len(v) == 24 for v in again["outs"].values())


def _stall_worker(rank, world, port, out_dir, push=False):
    """Rank 1 stops arriving at the collectives after the first request: rank
    0's all-reduce waits time out, STATUS is set, and the engine fails the
    runs in flight (and every later one) instead of returning wrong tokens.
    ``push``: o / down on the stream GEMM with the push epilogue, so the waits
    that time out include the push consumer's per-strip flag waits."""
    import time
    import torch.distributed as dist
    if push:
        from k8s_llm_rca_amd.ops import layer_exec as LE
        LE._tp_push = LE._tp_push_force = True
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    from k8s_llm_rca_amd.parallel.xgmi import CommFault, XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD)
    pc.custom_ar = XgmiAllReduce(dist.group.WORLD, max_bytes=8 << 20, timeout_s=1.0, max_blocks=SHARED_GPU_AR_BLOCKS)
    cfg = EngineConfig(model="tiny-llama", device="cuda:0", num_blocks=64, block_size=64, max_batch_tokens=256,
                       temperature=0.0, use_graphs=True)
    model = LlamaModel(get_config("tiny-llama"), "cuda:0", torch.bfloat16, pc, seed=5, init_mode="full_slice")
    eng = LLMEngine(cfg, pc, model=model)
    res = {}
    if rank > 0:
        eng.serve_worker()       # the healthy request
        eng._test_stall = True
        eng.serve_worker()       # receives every later step, executes none
    else:
        def run(n, tag):
            done = {}
            for i in range(n):
                sid = eng.new_sequence()
                toks = eng.tok.system_prefix("sys") + eng.tok.message("user", f"{tag} {i} " * 6) + \
                    eng.tok.header("assistant")
                eng.submit(sid, toks, None, 16, seed=3, on_done=lambda g, st, i=i: done.__setitem__(i, (g, st)))
            t0 = time.time()
            while len(done) < n and time.time() - t0 < 120:
                time.sleep(0.05)
            return done
        eng.start()
        ok = run(1, "healthy")
        eng.stop()
        eng.stop_workers()       # the worker now stalls
        eng.start()
        bad = run(3, "stalled")
        late = run(1, "late")
        eng.stop()
        eng.stop_workers()
        res = {"ok": [g is not None and len(g) == 16 for g, _ in ok.values()],
               "bad": [(g is None, st.get("error", "")) for g, st in bad.values()] if len(bad) == 3 else None,
               "late": [(g is None, st.get("error", "")) for g, st in late.values()],
               "fault": isinstance(eng.error, CommFault), "status": pc.custom_ar.status(),
               "ar_push": int(model._exec.st.ar_push) if model._exec is not None else -1}
        torch.save(res, os.path.join(out_dir, "stall.pt"))
    torch.cuda.synchronize()
    dist.barrier()
    pc.custom_ar.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("push", [False, True], ids=["staged", "push"])
def test_tp2_stalled_peer_fails_runs(push):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_stall_worker, args=(2, _free_port(), d, push), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "stall.pt"), weights_only=True)
    assert res["ok"] == [True]
    assert res["ar_push"] == int(push)
    assert res["fault"] and res["status"] == 1
    assert res["bad"] is not None and all(failed for failed, _ in res["bad"]), res["bad"]
    assert all(failed and "timed out" in err for failed, err in res["late"]), res["late"]


def _host_stall_worker(rank, world, port, out_dir):
    """rank 0's host stalls between sending an eager step
    and launching its own half, so the WORKER's collective is the one that
    times out.  The worker must notice its own STATUS and stop executing (so
    rank 0's next collective times out too) instead of skipping every later
    wait while still publishing flags -- which would let rank 0 mix
    unsynchronized partials into its outputs for good."""
    import time
    import torch.distributed as dist
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    from k8s_llm_rca_amd.parallel.xgmi import CommFault, XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD)
    pc.custom_ar = XgmiAllReduce(dist.group.WORLD, max_bytes=8 << 20, timeout_s=1.0, max_blocks=SHARED_GPU_AR_BLOCKS)
    cfg = EngineConfig(model="tiny-llama", device="cuda:0", num_blocks=64, block_size=64, max_batch_tokens=256,
                       temperature=0.0, use_graphs=True)
    model = LlamaModel(get_config("tiny-llama"), "cuda:0", torch.bfloat16, pc, seed=5, init_mode="full_slice")
    eng = LLMEngine(cfg, pc, model=model)
    if rank > 0:
        eng.serve_worker()       # the healthy request
        eng.serve_worker()       # the stalled ones: this rank's wait times out
        torch.cuda.synchronize()
        torch.save({"dead": eng.comm_dead, "status": pc.custom_ar.status()}, os.path.join(out_dir, "w.pt"))
    else:
        def run(n, tag):
            done = {}
            for i in range(n):
                sid = eng.new_sequence()
                toks = eng.tok.system_prefix("sys") + eng.tok.message("user", f"{tag} {i} " * 6) + \
                    eng.tok.header("assistant")
                eng.submit(sid, toks, None, 24, seed=3, on_done=lambda g, st, i=i: done.__setitem__(i, (g, st)))
            t0 = time.time()
            while len(done) < n and time.time() - t0 < 120:
                time.sleep(0.05)
            return done
        eng.start()
        ok = run(1, "healthy")
        eng.stop()
        eng.stop_workers()
        eng._test_host_stall_s = 3.0  # 3x the workers' timeout, before rank 0 launches its half
        eng.start()
        bad = run(2, "stalled")
        eng.stop()
        eng.stop_workers()
        res = {"ok": [g is not None and len(g) == 24 for g, _ in ok.values()],
               "bad": [(g is None, st.get("error", "")) for g, st in bad.values()] if len(bad) == 2 else None,
               "fault": isinstance(eng.error, CommFault), "status": pc.custom_ar.status()}
        torch.save(res, os.path.join(out_dir, "stall.pt"))
    torch.cuda.synchronize()
    dist.barrier()
    pc.custom_ar.close()
    dist.destroy_process_group()


def test_tp2_worker_timeout_stops_worker_and_fails_runs():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_host_stall_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "stall.pt"), weights_only=True)
        wres = torch.load(os.path.join(d, "w.pt"), weights_only=True)
    assert res["ok"] == [True]
    assert wres["dead"] and wres["status"] == 1
    assert res["fault"] and res["status"] == 1
    assert res["bad"] is not None and all(failed for failed, _ in res["bad"]), res["bad"]


def test_tp_sim_rank0_runs_real_kernels_with_standin_collectives():
    """bench --tp-sim: rank 0 of a TP=4 engine on one GPU (shard shapes, the
    native executor, HIP graphs, the xGMI kernels on a loopback communicator)
    generates complete runs, and the projection prices every forward's
    collectives both as stood in and as modelled."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.parallel.tpsim import project, sim_context
    pc = sim_context(4)
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda:0", num_blocks=64, block_size=64,
                                 max_batch_tokens=256, temperature=0.8), pc)
    assert eng.model.nq == 2 and eng.model.inter == 256 and eng._chan is None and not eng._dist_sample
    outs = {}
    for i in range(4):
        sid = eng.new_sequence()
        toks = eng.tok.system_prefix("sys") + eng.tok.message("user", "sim %d " % i * 9) + eng.tok.header("assistant")
        eng.submit(sid, toks, None, 20, seed=1, on_done=lambda g, st, i=i: outs.__setitem__(i, g))
    eng.run_until_idle()
    assert len(outs) == 4 and all(g is not None and len(g) == 20 for g in outs.values())
    assert eng.model._exec is not None and eng.stats["graph_steps"] > 0 and sum(eng.sim_rows.values()) > 0
    pr = project(eng.sim_rows, pc, eng.mc.hidden, eng.mc.n_layers, "cuda:0")
    assert pr["standin_s"] > 0 and pr["modelled_s"] > 0
    hops = pr["modelled_s_by_hop"]  # hop-latency sensitivity: monotone, the default hop reproduces modelled_s
    assert hops[2.5] == pytest.approx(pr["modelled_s"]) and hops[2.5] < hops[5.0] < hops[10.0]
    assert pc.custom_ar.status() == 0
    pc.custom_ar.close()


def test_tp_sim_moe_ep_runs_full_length():
    """bench --tp-sim on a MoE model (VERDICT r3 missing #2): rank 0 of a
    TP=4 / EP=4 tiny-mixtral -- attention shards, E/4 local experts, the
    fixed-capacity dispatch / combine / row all-gather over the loopback xGMI
    all-to-all -- produces finite logits and full-length runs (the r3 run
    sampled ~2 tokens per run: the row all-gather handed back never-written
    loopback slots), decode steps replay HIP graphs, and the projection prices
    the MoE collectives."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.parallel.tpsim import project, sim_context
    pc = sim_context(4, ep=4)
    eng = LLMEngine(EngineConfig(model="tiny-mixtral", device="cuda:0", num_blocks=128, block_size=64,
                                 max_batch_tokens=1024, temperature=0.8), pc)
    assert eng.model.moe is not None and eng.model.moe.E_local * 4 == eng.model.moe.E
    finite = []
    fwd = eng.model.forward

    def rec(*a, **k):
        out = fwd(*a, **k)
        if not torch.cuda.is_current_stream_capturing():
            finite.append(bool(torch.isfinite(out.float()).all()))
        return out
    eng.model.forward = rec
    outs = {}
    for i in range(6):
        sid = eng.new_sequence()
        toks = eng.tok.system_prefix("sys") + eng.tok.message("user", "moe %d " % i * (40 + 60 * i)) \
            + eng.tok.header("assistant")
        eng.submit(sid, toks, None, 24, seed=2, on_done=lambda g, st, i=i: outs.__setitem__(i, g))
    eng.run_until_idle()
    assert finite and all(finite)
    lens = {i: (None if g is None else len(g)) for i, g in outs.items()}
    assert len(outs) == 6 and all(v == 24 for v in lens.values()), (lens, eng.stats)
    assert eng.stats["graph_steps"] > 0
    pr = project(eng.sim_rows, pc, eng.mc.hidden, eng.mc.n_layers, "cuda:0", moe_k=eng.model.moe.k)
    assert pr["standin_s"] > 0 and pr["modelled_s"] > 0
    assert pc.custom_ar.status() == 0
    pc.custom_ar.close()


# ------------------------------------------------------------------ round 5
# Every TP / EP data collective on the xGMI kernels (xgmi_only): larger-than-
# buffer all-reduces and all-gathers in buffer-sized chunks, so the TP path that
# the 8-GPU node runs is the one these tests run (two ranks sharing cuda:0).

def _chunked_ar_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import ParallelContext, SHARED_GPU_AR_BLOCKS as CAP
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = XgmiAllReduce(dist.group.WORLD, max_bytes=16 << 20, timeout_s=60.0, max_blocks=CAP)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, custom_ar=car, xgmi_only=True)
    res = {}
    for mib in (32, 64, 128):
        n = (mib << 20) // 2
        # every rank draws every rank's input (same seeds): the fp32 sum of the bf16 inputs is the reference
        xs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1000 * mib + r))
              .bfloat16() for r in range(world)]
        ref = xs[0].float()
        for x in xs[1:]:
            ref += x.float()
        mine = xs[rank].clone()
        pc.all_reduce(mine)                       # 2-8 chunks of the 16 MiB buffer
        torch.cuda.synchronize()
        err = (mine.float() - ref).abs()
        res[mib] = {"max_err": err.max().item(), "bound": (ref.abs() * 2 ** -7 + 1e-6).sub(err).min().item(),
                    "chunks": -(-n // car.chunk_elems())}
        del xs, ref, mine
    # a larger-than-buffer all-gather (vocab-parallel logits rows)
    rows = torch.randn(300, 40000, device="cuda", generator=torch.Generator(device="cuda").manual_seed(77 + rank))
    g = pc.all_gather_last(rows)
    want0 = torch.randn(300, 40000, device="cuda", generator=torch.Generator(device="cuda").manual_seed(77))
    want1 = torch.randn(300, 40000, device="cuda", generator=torch.Generator(device="cuda").manual_seed(78))
    res["gather_ok"] = bool(torch.equal(g, torch.cat([want0, want1], 1)))
    res["status"] = car.status()
    car.close()
    if rank == 0:
        torch.save(res, os.path.join(out_dir, "ar.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_xgmi_chunked_allreduce_32_to_128_mib_vs_fp32():
    """the chunked large-message xGMI all-reduce (prefill-size
    TP messages, no RCCL on the data path) against the fp32 sum at 32 / 64 /
    128 MiB through a 16 MiB buffer, plus a 96 MB vocab-row all-gather."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_chunked_ar_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "ar.pt"), weights_only=True)
    assert res["status"] == 0 and res["gather_ok"]
    for mib in (32, 64, 128):
        r = res[mib]
        assert r["chunks"] >= 2 and r["bound"] >= 0, (mib, r)   # |err| <= |ref| 2^-7 (bf16 rounding of the sum)


def _prefill_inputs(m, T, seed=5):
    """StepInputs of one fresh sequence's T-token prefill (pages 0.., block 64)."""
    from k8s_llm_rca_amd.models.llama import StepInputs
    from k8s_llm_rca_amd.ops import attention as A
    BS = 64
    nb = -(-T // BS)
    ids = torch.randint(0, min(100000, m.cfg.vocab_size), (T,), generator=torch.Generator().manual_seed(seed),
                        dtype=torch.int32)
    meta = A.AttnMeta(block_tables=torch.arange(nb, dtype=torch.int32).view(1, -1).cuda(),
                      ctx_lens=torch.tensor([T], dtype=torch.int32).cuda(),
                      q_start=torch.tensor([0, T], dtype=torch.int32).cuda(), num_seqs=1, decode=False,
                      ctx_lens_host=[T], q_start_host=[0, T])
    A.attach_plan(meta, A.plan_prefill([0, T], m.nq // m.nkv, BS, [T], nkv=m.nkv), "cuda")
    inp = StepInputs(ids.cuda(), torch.arange(T, dtype=torch.int32).cuda(), torch.arange(T, dtype=torch.int32).cuda(),
                     0, None, meta, torch.tensor([T - 1], dtype=torch.int64).cuda())
    L = m.cfg.n_layers
    kc = torch.zeros(L, nb, m.nkv, BS, m.D, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(L, nb, m.nkv, m.D, BS, dtype=torch.bfloat16, device="cuda")
    return inp, kc, vc


def _fp32_reference_logits(m, T, seed=5):
    """Plain-PyTorch fp32 forward of ``_prefill_inputs``'s sequence on the
    TP=1 model's weights (each layer's weights upcast on the fly): the anchor
    both the bf16 TP=1 and TP=2 engines are measured against."""
    import torch.nn.functional as F
    cfg = m.cfg
    eps, D, nq, nkv = cfg.rms_eps, m.D, m.nq, m.nkv
    ids = torch.randint(0, min(100000, cfg.vocab_size), (T,), generator=torch.Generator().manual_seed(seed),
                        dtype=torch.int32).cuda()
    half = D // 2
    cs = m.cos_sin[:T].float()
    cos, sin = cs[:, None, :half], cs[:, None, half:]

    def norm(x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()

    def rope(x):  # [T, h, D], rotation pairs (i, i + D/2)
        a, b = x[..., :half], x[..., half:]
        return torch.cat([a * cos - b * sin, b * cos + a * sin], dim=-1)

    h = m.embed[ids.long()].float()
    for L in m.layers:
        y = norm(h, L["in_norm"])
        qkv = y @ L["wqkv"].float().t()
        q = rope(qkv[:, :nq * D].view(T, nq, D))
        k = rope(qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D))
        v = qkv[:, (nq + nkv) * D:(nq + 2 * nkv) * D].view(T, nkv, D)
        k, v = (t.repeat_interleave(nq // nkv, dim=1) for t in (k, v))
        a = F.scaled_dot_product_attention(q.transpose(0, 1)[None], k.transpose(0, 1)[None], v.transpose(0, 1)[None],
                                           is_causal=True, scale=m.scale)[0].transpose(0, 1).reshape(T, nq * D)
        h = h + a @ L["wo"].float().t()
        y = norm(h, L["post_norm"])
        gu = y @ L["w_gu"].float().t()
        I = gu.shape[1] // 2
        h = h + (F.silu(gu[:, :I]) * gu[:, I:]) @ L["w_down"].float().t()
    y = norm(h[T - 1:], m.final_norm)
    return (y @ m.lm_head.float().t()).cpu()


def _tp_logits_worker(rank, world, port, out_dir, Ts, max_mb, layers=(1, 2, 32)):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    from k8s_llm_rca_amd.knobs import set_knob
    set_knob("ar_max_mb", max_mb)
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext, attach_custom_allreduce
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pc = attach_custom_allreduce(ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD),
                                     same_gpu=True)
        assert pc.custom_ar is not None and pc.xgmi_only
    else:
        pc = None
    out = {}
    for nl in layers:
        m = LlamaModel(get_config("llama3-8b", n_layers=nl), "cuda:0", torch.bfloat16, pc, seed=11,
                       init_mode="full_slice")
        for T in Ts:
            inp, kc, vc = _prefill_inputs(m, T)
            out[f"{nl}/{T}"] = {"logits": m.forward(inp, kc, vc).float().cpu(),
                                "exec": m._exec is not None and m._exec.fits(T)}
            if world == 1:
                out[f"{nl}/{T}"]["fp32"] = _fp32_reference_logits(m, T)
        del m
        torch.cuda.empty_cache()
    if world > 1:
        out["status"] = pc.custom_ar.status()
    if rank == 0:
        torch.save(out, os.path.join(out_dir, f"tp{world}.pt"))
    if world > 1:
        dist.barrier()
        pc.custom_ar.close()
        dist.destroy_process_group()


def test_tp2_llama3_8b_logits_match_tp1_one_gpu():
    """Llama-3-8B at TP=2 as two processes on one MI355X
    (gloo host group, every collective on the xGMI kernels) at T=300 through
    the native executor's fused all-reduce + add + RMSNorm, and at T=1100
    (past the 4 MiB buffer) through the Python layer path's chunked
    all-reduce -- both measured against an fp32 PyTorch forward of the same
    weights (:func:`_fp32_reference_logits`) at 1, 2 and 32 layers.  The TP=2
    engine must be as close to fp32 as the TP=1 engine is:
    err(TP2) <= 1.25 err(TP1) + 1e-3.  (Round 5 bounded TP2 vs TP1 directly,
    loosened to 10 % at 32 layers; bf16 drift through a random-init stack is
    real -- profiles/r5/tp_check.txt -- but a bound on the difference cannot
    tell it from a few % of a wrong shard or a stale chunk, the anchor can.)"""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    Ts = (300, 1100)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_tp_logits_worker, args=(2, _free_port(), d, Ts, 4), nprocs=2, join=True)
        mp.spawn(_tp_logits_worker, args=(1, _free_port(), d, Ts, 4), nprocs=1, join=True)
        a = torch.load(os.path.join(d, "tp2.pt"), weights_only=True)
        b = torch.load(os.path.join(d, "tp1.pt"), weights_only=True)
    assert a["status"] == 0
    assert a["2/300"]["exec"] and not a["2/1100"]["exec"]
    rec = {}
    for nl in (1, 2, 32):
        for T in Ts:
            x, y = a[f"{nl}/{T}"]["logits"][:, :128256], b[f"{nl}/{T}"]["logits"][:, :128256]
            ref = b[f"{nl}/{T}"]["fp32"][:, :128256]
            assert torch.isfinite(x).all()
            e2 = ((x - ref).norm() / ref.norm()).item()
            e1 = ((y - ref).norm() / ref.norm()).item()
            rec[f"{nl}/{T}"] = {"tp2_vs_fp32": e2, "tp1_vs_fp32": e1, "tp2_vs_tp1": ((x - y).norm() / y.norm()).item()}
            assert e2 <= 1.25 * e1 + 1e-3, (nl, T, e2, e1)
            # the top token of each engine is among the fp32 forward's top 5
            top = set(ref.topk(5, -1).indices.view(-1).tolist())
            assert int(x.argmax(-1)) in top and int(y.argmax(-1)) in top, (nl, T)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        import json
        with open(os.path.join(out, "tp_fp32_anchor.json"), "w") as f:
            json.dump(rec, f, indent=1)


def _tune_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import SHARED_GPU_AR_BLOCKS as CAP
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    car = XgmiAllReduce(dist.group.WORLD, max_bytes=16 << 20, timeout_s=60.0, max_blocks=CAP)
    g = torch.Generator(device="cuda").manual_seed(3)
    H = 4096
    wo = (torch.randn(H, 2048, device="cuda", generator=g) * 0.02).bfloat16()
    wd = (torch.randn(H, 7168, device="cuda", generator=g) * 0.02).bfloat16()
    nw = torch.ones(H, device="cuda").bfloat16()
    rep = car.tune([("o", wo), ("down", wd)], nw, 1e-5, (16, 64, 256, 4096), iters=3, rounds=2)
    # the prefill-size GEMM / all-reduce overlap depth (steps past the executor's buffer:
    # row chunks, each chunk's xGMI all-reduce on the comm stream beside the next GEMM)
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, custom_ar=car, xgmi_only=True)
    ov = pc.tune_overlap([("o", wo), ("down", wd)], [4096], iters=2, rounds=1)
    res = {"plan": {int(k): list(v) for k, v in car.plan.items()}, "rep": {int(k): v for k, v in rep.items()},
           "for_40": list(car.plan_for(40, H)), "for_5000": list(car.plan_for(5000, H)), "status": car.status(),
           "ov": {int(k): v["pick"] for k, v in ov.items()}}
    car.close()
    torch.save(res, os.path.join(out_dir, f"tune{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_xgmi_epilogue_tuning_same_plan_on_every_rank():
    """the init-time fabric tuning times one-/two-shot (and
    push where the GEMM allows it) per bucket and every rank gets the SAME plan
    (a rank-dependent mode would deadlock the collective); buckets past the
    buffer are skipped and T above the largest bucket falls back to the size
    rule."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_tune_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        a = torch.load(os.path.join(d, "tune0.pt"), weights_only=True)
        b = torch.load(os.path.join(d, "tune1.pt"), weights_only=True)
    assert a["status"] == 0 and b["status"] == 0
    assert a["plan"] == b["plan"] and set(a["plan"]) == {16, 64, 256}   # 4096 x 4096 x 2 B > 16 MiB
    assert a["for_40"] == a["plan"][64]
    assert a["for_5000"] == [2, False]
    assert a["ov"] == b["ov"] and set(a["ov"]) == {4096} and a["ov"][4096] in (1, 2, 4)
    for T, r in a["rep"].items():
        assert "one_shot" in r and "two_shot" in r and all(v > 0 for k, v in r.items() if k != "pick")
