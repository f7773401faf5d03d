"""Tensor / expert parallelism on CPU with gloo (world_size 2), checked against the unsharded model."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(cfg, device="cpu"):
    """A mixed step: 2 decode rows + a 7-token prefill chunk over a paged cache."""
    from k8s_llm_rca_amd.models.llama import StepInputs
    from k8s_llm_rca_amd.ops import attention as A
    torch.manual_seed(0)
    BS = 32
    ids = torch.randint(0, 500, (9,), dtype=torch.int32)
    # seq0: ctx 40 (decode), seq1: ctx 3 (decode), seq2: 7 new tokens at positions 5..11
    pos = torch.tensor([39, 2, 5, 6, 7, 8, 9, 10, 11], dtype=torch.int32)
    bt_d = torch.tensor([[0, 1], [2, 0]], dtype=torch.int32)
    slots = torch.tensor([1 * BS + 7, 2 * BS + 2, 3 * BS + 5, 3 * BS + 6, 3 * BS + 7, 3 * BS + 8, 3 * BS + 9,
                          3 * BS + 10, 3 * BS + 11], dtype=torch.int32)
    md = A.AttnMeta(block_tables=bt_d, ctx_lens=torch.tensor([40, 3], dtype=torch.int32),
                    q_start=torch.tensor([0, 1, 2], dtype=torch.int32), num_seqs=2, decode=True,
                    ctx_lens_host=[40, 3], q_start_host=[0, 1, 2])
    mp_ = A.AttnMeta(block_tables=torch.tensor([[3]], dtype=torch.int32), ctx_lens=torch.tensor([12], dtype=torch.int32),
                     q_start=torch.tensor([0, 7], dtype=torch.int32), num_seqs=1, decode=False,
                     ctx_lens_host=[12], q_start_host=[0, 7])
    return StepInputs(ids, pos, slots, 2, md, mp_, torch.tensor([0, 1, 8])), BS


def _run_model(rank, world, port, name, out_path):
    import torch.distributed as dist
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, ep_size=world, ep_rank=rank,
                         ep_group=dist.group.WORLD)
    cfg = get_config(name)
    m = LlamaModel(cfg, "cpu", torch.float32, pc, seed=3, init_mode="full_slice")
    inp, BS = _inputs(cfg)
    torch.manual_seed(1)
    k = torch.randn(cfg.n_layers, 6, m.nkv, BS, 128) * 0.5
    v = torch.randn(cfg.n_layers, 6, m.nkv, 128, BS)
    # each rank holds its own kv heads: slice the shared random cache consistently
    kf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, BS, 128, generator=torch.Generator().manual_seed(7)) * 0.5
    vf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, 128, BS, generator=torch.Generator().manual_seed(8))
    h0 = (rank * cfg.n_kv_heads) // world if cfg.n_kv_heads < world else rank * m.nkv
    k.copy_(kf[:, :, h0:h0 + m.nkv])
    v.copy_(vf[:, :, h0:h0 + m.nkv])
    logits = m.forward(inp, k, v)
    if rank == 0:
        torch.save(logits[:, : cfg.vocab_size], out_path)
    dist.barrier()
    dist.destroy_process_group()


def _reference(name):
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    cfg = get_config(name)
    m = LlamaModel(cfg, "cpu", torch.float32, None, seed=3, init_mode="full_slice")
    inp, BS = _inputs(cfg)
    kf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, BS, 128, generator=torch.Generator().manual_seed(7)) * 0.5
    vf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, 128, BS, generator=torch.Generator().manual_seed(8))
    return m.forward(inp, kf, vf)[:, : cfg.vocab_size]


@pytest.mark.parametrize("name,world", [("tiny-llama", 2), ("tiny-mixtral", 2), ("tiny-llama", 4), ("tiny-llama", 8),
                                        ("tiny-llama-g8", 4), ("tiny-mixtral", 4)])
def test_tp2_matches_tp1(name, world):
    """Sharded forward (column / row / vocab parallel, kv heads replicated when
    n_kv < tp) == the unsharded model at world 2 / 4 / 8."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "logits.pt")
        mp.spawn(_run_model, args=(world, port, name, out), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    ref = _reference(name)
    torch.testing.assert_close(got, ref, atol=2e-4, rtol=2e-4)


def _run_engine(rank, world, port, out_path, temperature=0.0, grammar=False, name="tiny-llama", top_k=0, top_p=1.0):
    import torch.distributed as dist
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD)
    else:
        pc = None
    cfg = EngineConfig(model=name, device="cpu", dtype=torch.float32, num_blocks=32, block_size=32,
                       max_batch_tokens=64, temperature=temperature)
    model = LlamaModel(get_config(name), "cpu", torch.float32, pc, seed=5, init_mode="full_slice")
    eng = LLMEngine(cfg, pc, model=model)
    if rank > 0:
        eng.serve_worker()
    else:
        outs = {}
        for i in range(3):
            sid = eng.new_sequence()
            toks = eng.tok.system_prefix("sys") + eng.tok.message("user", "message %d " % i * (5 + 9 * i)) + \
                eng.tok.header("assistant")
            g = None
            if grammar:  # exercises list and bitmap masks in the distributed sampler
                from k8s_llm_rca_amd.engine.grammar import Choice, Free, Grammar, Lit
                g = Grammar([Lit('{"k": '), Choice(['"alpha"', '"beta"', '"gamma"'], "c"), Lit(', "t": "'),
                             Free(6, name="t"), Lit('"}')])
            eng.submit(sid, toks, g, 12, temperature=temperature, seed=7,
                       on_done=lambda g, st, i=i: outs.__setitem__(i, g), top_k=top_k, top_p=top_p)
        eng.run_until_idle()
        eng.stop_workers()
        outs["_msgs"] = eng._chan.sent if eng._chan is not None else 0
        torch.save(outs, out_path)
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "tiny-llama"), (4, "tiny-llama"), (8, "tiny-llama"),
                                        (2, "tiny-llama-g8"), (4, "tiny-llama-g8")])
def test_tp_engine_generation_matches_tp1(world, name):
    """TP engine (host step channel, async overlapped steps, vocab-parallel
    sampling) == the unsharded engine, token for token.  World 4 / 8 on
    tiny-llama (2 kv heads) and tiny-llama-g8 (1 kv head) run with kv heads
    replicated across ranks (n_kv < tp)."""
    with tempfile.TemporaryDirectory() as d:
        o2, o1 = os.path.join(d, "tpn.pt"), os.path.join(d, "tp1.pt")
        mp.spawn(_run_engine, args=(world, _free_port(), o2, 0.0, False, name), nprocs=world, join=True)
        _run_engine(0, 1, _free_port(), o1, 0.0, False, name)
        a = torch.load(o2, weights_only=True)
        b = torch.load(o1, weights_only=True)
    assert a.pop("_msgs") > 0 and b.pop("_msgs") == 0
    assert a == b and all(len(v) == 12 for v in a.values())


@pytest.mark.parametrize("top_k,top_p", [(0, 1.0), (5, 1.0), (20, 0.8), (64, 0.95), (0, 0.9), (100, 1.0), (100, 0.8)])
def test_tp2_distributed_sampling_with_grammar_matches_tp1(top_k, top_p):
    """Vocab-parallel Gumbel-max sampling (masks keyed by global id; top-k /
    top-p through the per-rank candidate lists, exact for k <= CAND_K) must pick the same tokens as
    single-device sampling of the gathered logits."""
    with tempfile.TemporaryDirectory() as d:
        o2, o1 = os.path.join(d, "tp2.pt"), os.path.join(d, "tp1.pt")
        mp.spawn(_run_engine, args=(2, _free_port(), o2, 0.9, True, "tiny-llama", top_k, top_p), nprocs=2,
                 join=True)
        _run_engine(0, 1, _free_port(), o1, 0.9, True, "tiny-llama", top_k, top_p)
        a = torch.load(o2, weights_only=True)
        b = torch.load(o1, weights_only=True)
    a.pop("_msgs"), b.pop("_msgs")
    assert a == b and len(a) == 3


def _run_overlap(rank, world, port, out_path):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, ar_chunks=3, overlap_min_bytes=64)
    g = torch.Generator().manual_seed(100 + rank)
    res = {}
    for M, N, K in ((7, 300, 64), (40, 64, 32), (600, 96, 48)):  # column path (M <= 256) and row path
        x = torch.randn(M, K, generator=g)
        w = torch.randn(N, K, generator=g)
        got = pc.linear_all_reduce(x, w)
        want = x @ w.t()
        dist.all_reduce(want)
        res[(M, N)] = (got - want).abs().max().item()
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_linear_all_reduce_overlap_chunks_exact():
    """Chunked GEMM + async all-reduce pipeline == GEMM then all-reduce."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_run_overlap, args=(2, _free_port(), out), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    assert all(v < 1e-4 for v in res.values()), res


def _run_tune_overlap(rank, world, port, out_path):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, overlap_min_bytes=64)
    g = torch.Generator().manual_seed(7 + rank)
    shapes = [("o", torch.randn(96, 48, generator=g)), ("down", torch.randn(96, 80, generator=g))]
    rep = pc.tune_overlap(shapes, [300, 600], iters=2, rounds=2)
    picks = torch.tensor([rep[300]["pick"], rep[600]["pick"]])
    allp = [torch.zeros_like(picks) for _ in range(world)]
    dist.all_gather(allp, picks)
    # the tuned depth is what linear_all_reduce then runs, and it is still exact
    x = torch.randn(450, 48, generator=g)
    got = pc.linear_all_reduce(x, shapes[0][1])
    want = x @ shapes[0][1].t()
    dist.all_reduce(want)
    if rank == 0:
        torch.save({"plan": pc.chunk_plan, "picks": [p.tolist() for p in allp], "k450": pc.chunks_for(450),
                    "err": (got - want).abs().max().item(), "keys": sorted(rep[300])}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_tune_overlap_same_plan_on_every_rank():
    """The GEMM / all-reduce pipeline depth timed per bucket at init
    (ParallelContext.tune_overlap): max-reduced timings give every rank the
    same plan, linear_all_reduce takes the bucket at or above M, exactly."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_run_tune_overlap, args=(2, _free_port(), out), nprocs=2, join=True)
        r = torch.load(out, weights_only=True)
    assert r["picks"][0] == r["picks"][1]
    assert set(r["plan"]) == {300, 600} and r["k450"] == r["plan"][600]
    # on a gloo group the one transport is torch.distributed's own collective
    assert r["keys"] == ["pick", "rccl_k1", "rccl_k2", "rccl_k4", "transport"]
    assert r["err"] < 1e-4


def _run_tune_transport(rank, world, port, out_path):
    """RCCL vs xGMI per bucket with fake, rank-dependent timings: each rank
    alone would pick differently; the max-reduce must give one plan."""
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, overlap_min_bytes=64)
    # (bucket, transport, depth) -> us on this rank.  Bucket 1024: rank 0 alone prefers xGMI k2 (90),
    # rank 1 alone RCCL k1 (80); the per-candidate max is xgmi_k2 = 130 < rccl_k1 = 150 -> xGMI k2.
    # Bucket 8192: RCCL k4 is the slowest-rank winner on both.
    fake = {(1024, "xgmi", 2): (90, 130), (1024, "rccl", 1): (150, 80), (8192, "rccl", 4): (200, 210),
            (8192, "xgmi", 4): (230, 190)}
    seen = []

    def timer(shapes, x, k, rccl, iters):
        T = next(iter(x.values())).shape[0]
        tr = "rccl" if rccl else "xgmi"
        seen.append((T, tr, k, pc.rccl_for(T), pc.chunks_for(T)))
        return float(fake.get((T, tr, k), (500, 500))[rank])

    pc._time_candidate = timer
    shapes = [("o", torch.randn(96, 48)), ("down", torch.randn(96, 80))]
    rep = pc.tune_overlap(shapes, [1024, 8192], iters=1, rounds=1, transports=("xgmi", "rccl"))
    res = {"plan": pc.chunk_plan, "rplan": pc.rccl_plan, "rep": rep,
           "route": [pc.rccl_for(M) for M in (512, 1024, 2000, 8192, 20000)], "n": len(seen)}
    objs = [None] * world
    dist.all_gather_object(objs, res)
    if rank == 0:
        torch.save(objs, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_tune_overlap_rccl_vs_xgmi_same_plan_on_every_rank():
    """the init-time tuning times RCCL against the xGMI kernels
    per prefill-size bucket; the per-candidate max over ranks decides, so
    every rank holds the same (depth, transport) plan, and steps route by it."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_run_tune_transport, args=(2, _free_port(), out), nprocs=2, join=True)
        a, b = torch.load(out, weights_only=True)
    assert a["plan"] == b["plan"] == {1024: 2, 8192: 4}
    assert a["rplan"] == b["rplan"] == {1024: False, 8192: True}
    assert a["rep"][1024]["transport"] == "xgmi" and a["rep"][8192]["transport"] == "rccl"
    assert a["rep"][1024]["k2"] == 130 and a["rep"][1024]["rccl_k1"] == 150   # the slowest rank's view
    # rows up to 1024 -> xGMI, 1025..8192 -> RCCL, past the last bucket -> the default (xGMI)
    assert a["route"] == [False, False, True, True, False]
    assert a["n"] == 2 * 6   # 2 buckets x (2 transports x 3 depths)


def _run_moe(rank, world, port, out_path):
    import torch.distributed as dist
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.moe import MoELayerSet
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, ep_size=world, ep_rank=rank,
                             ep_group=dist.group.WORLD)
    else:
        pc = ParallelContext()
    cfg = get_config("tiny-mixtral", n_experts=8, init_std=0.05)
    moe = MoELayerSet(cfg, "cpu", torch.float32, pc, torch.Generator().manual_seed(11), 0.02, full_slice=True)
    res = {}
    for T in (1, 9, 64, 300):  # 300 > FIXED_MAX_T: the variable-size path
        y = torch.randn(T, cfg.hidden, generator=torch.Generator().manual_seed(T))
        res[T] = moe.forward(1, y)
    if rank == 0:
        torch.save(res, out_path)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ep_moe_matches_ep1(world):
    """Expert parallelism (static-size dispatch for decode batches, exact
    variable-size all-to-alls for prefill) == all experts on one rank."""
    with tempfile.TemporaryDirectory() as d:
        o, o1 = os.path.join(d, "ep.pt"), os.path.join(d, "ep1.pt")
        mp.spawn(_run_moe, args=(world, _free_port(), o), nprocs=world, join=True)
        _run_moe(0, 1, _free_port(), o1)
        a = torch.load(o, weights_only=True)
        b = torch.load(o1, weights_only=True)
    for T in b:
        torch.testing.assert_close(a[T], b[T], atol=1e-5, rtol=1e-5)


def _run_channel(rank, world, port, out_path):
    import numpy as np
    import torch.distributed as dist

    from k8s_llm_rca_amd.parallel.channel import FWD_GRAPH, SAMPLE, STOP, StepChannel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ch = StepChannel(dist.group.WORLD, 0)
    msgs = [(FWD_GRAPH, [np.arange(5, dtype=np.int32), np.array([1, -2, 3 << 40], dtype=np.int64),
                         np.array([0.5, -1.25], dtype=np.float32)]),
            (SAMPLE, [np.zeros(0, np.int32), np.arange(3, dtype=np.int64)]),
            (STOP, [])]
    got = []
    if rank == 0:
        for kind, arrs in msgs:
            ch.send(kind, arrs)
    else:
        for _ in msgs:
            kind, arrs = ch.recv()
            got.append((kind, [(a.dtype.str, a.tolist()) for a in arrs]))
        want = [(k, [(a.dtype.str, a.tolist()) for a in arrs]) for k, arrs in msgs]
        assert got == want, (got, want)
        with open(f"{out_path}.{rank}", "w") as f:
            f.write("ok")
    dist.destroy_process_group()


def test_step_channel_roundtrip():
    """The TP host step channel (parallel/channel.py) delivers every message's
    kind and int32 / int64 / float32 arrays bit-exactly to every worker, in
    order, including empty arrays and payload-free messages."""
    world = 3
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "ch")
        mp.spawn(_run_channel, args=(world, _free_port(), out), nprocs=world, join=True)
        assert all(open(f"{out}.{r}").read() == "ok" for r in range(1, world))


def test_xgmi_plan_for_buckets_and_size_rule():
    """XgmiAllReduce.plan_for: the tuned bucket at or above T, else the size
    rule (one-shot up to ONE_SHOT_MAX bytes, never push) -- the executor's
    per-step (mode, push) choice (ops/layer_exec.py)."""
    import types
    from k8s_llm_rca_amd.parallel.xgmi import ONE_SHOT_MAX, XgmiAllReduce
    tuned = types.SimpleNamespace(plan={16: (1, False), 64: (2, True), 256: (1, True)})
    assert XgmiAllReduce.plan_for(tuned, 1, 8192) == (1, False)
    assert XgmiAllReduce.plan_for(tuned, 17, 8192) == (2, True)
    assert XgmiAllReduce.plan_for(tuned, 256, 8192) == (1, True)
    big = 300                                                          # > the largest bucket, > ONE_SHOT_MAX bytes
    assert big * 8192 * 2 > ONE_SHOT_MAX
    assert XgmiAllReduce.plan_for(tuned, big, 8192) == (2, False)       # past the largest bucket: size rule
    untuned = types.SimpleNamespace(plan=None)
    assert XgmiAllReduce.plan_for(untuned, 4, 8192) == (1, False)
    assert XgmiAllReduce.plan_for(untuned, big, 8192) == (2, False)
