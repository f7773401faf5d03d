"""Model-level numerics: HIP kernel path (bf16, MI355X) vs the fp32 PyTorch reference path (CPU)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _clone_to(model, device, dtype):
    import copy
    m = copy.copy(model)
    m.device = torch.device(device)
    m.dtype = dtype
    m.layers = [{k: v.to(device, dtype) for k, v in L.items()} for L in model.layers]
    m.embed = model.embed.to(device, dtype)
    m.lm_head = model.lm_head.to(device, dtype)
    m.final_norm = model.final_norm.to(device, dtype)
    m.cos_sin = model.cos_sin.to(device)
    if model.moe is not None:
        mo = copy.copy(model.moe)
        mo.router = [t.to(device, dtype) for t in model.moe.router]
        mo.w13 = [t.to(device, dtype) for t in model.moe.w13]
        mo.w2 = [t.to(device, dtype) for t in model.moe.w2]
        m.moe = mo
    return m


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama-g8", "tiny-mixtral"])
def test_forward_gpu_matches_cpu(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from tests.test_parallel import _inputs
    cfg = get_config(name, init_std=0.08)  # peaked logits: the argmax is stable under bf16 rounding
    ref_m = LlamaModel(cfg, "cpu", torch.float32, None, seed=3, init_mode="full_slice")
    inp, BS = _inputs(cfg)
    kf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, BS, 128, generator=torch.Generator().manual_seed(7)) * 0.5
    vf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, 128, BS, generator=torch.Generator().manual_seed(8))
    ref = ref_m.forward(inp, kf.clone(), vf.clone())[:, : cfg.vocab_size]
    gm = _clone_to(ref_m, "cuda", torch.bfloat16)
    dev = lambda t: None if t is None else t.cuda()
    for meta in (inp.meta_decode, inp.meta_prefill):
        for f in ("block_tables", "ctx_lens", "q_start"):
            setattr(meta, f, dev(getattr(meta, f)))
    import k8s_llm_rca_amd.ops.attention as A
    md = inp.meta_decode
    md.n_parts, md.part_size = 1, 256
    mp_ = inp.meta_prefill
    A.attach_plan(mp_, A.plan_prefill(mp_.q_start_host, cfg.n_heads // cfg.n_kv_heads, BS, mp_.ctx_lens_host,
                                      nkv=cfg.n_kv_heads), "cuda")
    inp.input_ids, inp.positions, inp.slots, inp.logits_idx = (inp.input_ids.cuda(), inp.positions.cuda(),
                                                               inp.slots.cuda(), inp.logits_idx.cuda())
    out = gm.forward(inp, kf.cuda().bfloat16(), vf.cuda().bfloat16())[:, : cfg.vocab_size].float().cpu()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item()
    rel = ((out - ref).norm() / ref.norm()).item()
    # bf16 weights / activations with fp32 accumulation and fp32 logits vs the fp32 reference
    # (MoE: a near-tie router score may pick the other expert for a token under bf16)
    assert rel <= 0.03 and err <= (0.05 if cfg.n_experts else 0.03) * scale, (rel, err, scale)
    assert torch.equal(out.argmax(-1), ref.argmax(-1))


def test_moe_prefill_no_host_sync():
    """a Mixtral prefill-sized MoE layer (tiny-mixtral, 1,100
    tokens x top-2 = 2,200 routed rows > GROUPED_MAX_ROWS) runs routing,
    permutation, the grouped SwiGLU gate_up + down (gemm_big.hip grouped form)
    and the combine with no host sync (torch's sync checker in error mode), and
    matches the per-expert hipBLASLt path it replaced."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    cfg = get_config("tiny-mixtral")
    m = LlamaModel(cfg, "cuda", torch.bfloat16, None, seed=4)
    moe = m.moe
    y = (torch.randn(1100, cfg.hidden, device="cuda") * 0.5).bfloat16()
    torch.cuda.synchronize()
    assert 1100 * moe.k > moe.GROUPED_MAX_ROWS
    torch.cuda.set_sync_debug_mode("error")
    try:
        out = moe.forward(0, y)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    moe.BIG_PREFILL = False
    try:
        ref = moe.forward(0, y)
    finally:
        moe.BIG_PREFILL = True
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_engine_graph_vs_eager_decode():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    outs = []
    for graphs in (False, True):
        eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", num_blocks=256, use_graphs=graphs,
                                     temperature=0.0, graph_batch_sizes=(1, 2, 4, 8)))
        res = {}
        for i in range(5):
            sid = eng.new_sequence()
            p = eng.tok.system_prefix("s") + eng.tok.message("user", "q%d " % i * (3 + 7 * i)) + eng.tok.header("assistant")
            eng.submit(sid, p, None, 16, temperature=0.0, on_done=lambda g, st, i=i: res.__setitem__(i, g))
        eng.run_until_idle()
        outs.append(res)
        if graphs:
            assert eng.stats["graph_steps"] > 0
    assert outs[0] == outs[1]


def test_mixtral_engine_graphs_match_eager():
    """MoE decode steps run inside HIP graphs (grouped GEMM reads device-side
    expert offsets: nothing syncs to the host) and match eager execution."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.engine.grammar import Choice, Free, Grammar, Lit
    outs = []
    for graphs in (True, False):
        eng = LLMEngine(EngineConfig(model="tiny-mixtral", device="cuda", dtype=torch.bfloat16, num_blocks=256,
                                     block_size=64, temperature=0.0, use_graphs=graphs))
        res = {}
        for i in range(5):
            sid = eng.new_sequence()
            g = Grammar([Lit('{"k": '), Choice(['"a"', '"bb"', '"ccc"'], "c"), Lit(', "t": "'), Free(12, name="t"),
                         Lit('"}')])
            p = eng.tok.system_prefix("s") + eng.tok.message("user", "mixtral %d " % i * (4 + 3 * i)) + \
                eng.tok.header("assistant")
            eng.submit(sid, p, g, 24, temperature=0.0, on_done=lambda gen, st, i=i: res.__setitem__(i, gen))
        eng.run_until_idle()
        assert len(res) == 5
        if graphs:
            assert eng.stats["graph_steps"] > 0
        outs.append(res)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("graphs,splitk", [(False, False), (True, False), (False, True), (True, True),
                                           (False, "stream"), (True, "stream"), (False, "big"), (True, "big"),
                                           (False, "bigsplit")])
def test_layer_executor_bit_identical(graphs, splitk):
    """The native layer executor (one C call per forward) issues the same
    kernels in the same order as the Python layer loop: every step's logits
    are bit-identical, for mixed prefill+decode steps and graph decode steps.
    ``splitk``: a dispatch table that sends the o / down projections to the
    split-K kernels (gemm_mid, grouped), whose partials the executor reduces
    inside the following residual add + RMSNorm instead of a reduce kernel.
    ``"big"``: every projection above 256 rows on gemm_big (gate_up with its
    SwiGLU epilogue) and the decode-size gate_up on the stream kernel's
    SwiGLU epilogue.  ``"bigsplit"``: gemm_big with K split over 2 / 4
    workgroups for qkv / o / down above 256 rows: the executor leaves the fp32
    partials to the RoPE / KV write and the residual add + RMSNorm, the Python
    path reduces them with gemm_big's reduce kernel -- same sums, same order."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.ops import layer_exec as LX
    from k8s_llm_rca_amd.ops import linear as LIN
    split_rows = [(32, "mid", 0, 2), (64, "mid", 2, 4), (256, "grp", -1, 2)]  # tiny-llama o and down: [512, 1024]
    if splitk == "stream":  # the register-ring and LDS-DMA stream kernels (dispatch kind 4)
        split_rows = [(16, "stream", 4, 2), (64, "stream", 14, 2), (256, "stream", 14, 4)]
    runs = []
    try:
        for on in (False, True):
            LX.set_enabled(on)
            eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", num_blocks=512, use_graphs=graphs,
                                         temperature=0.0, max_batch_tokens=1024 if splitk == "big" else 256,
                                         graph_batch_sizes=(1, 2, 4, 8)))
            if splitk == "big":
                LIN.set_big("all")
                LIN._dispatch[(2048, 512)] = [(16, "stream", 4, 1), (64, "stream", 13, 1), (256, "stream", 24, 1)]
                assert LIN.swiglu_choice(300, 2048, 512)[0] == LIN.KIND_BIG
                assert LIN.swiglu_choice(5, 2048, 512) == (LIN.KIND_STREAM, 4, 1)
                assert LIN.select_gemm(300, 512, 1024)[0] == LIN.KIND_BIG
            elif splitk == "bigsplit":
                LIN.set_big("1")
                LIN._big_ranges[(512, 1024)] = [(257, 1 << 20, 4)]   # o and down
                LIN._big_ranges[(1536, 512)] = [(257, 1 << 20, 2)]   # qkv
                assert LIN.select_gemm(300, 512, 1024) == (LIN.KIND_BIG, LIN.BIG_PIPE, 4)
                assert LIN.select_gemm(300, 1536, 512) == (LIN.KIND_BIG, LIN.BIG_PIPE, 2)
            elif splitk:  # after the engine's own (absent) dispatch table was loaded
                LIN._dispatch[(512, 1024)] = split_rows
                if splitk == "stream":
                    assert LIN.select_gemm(6, 512, 1024)[0] == LIN.KIND_STREAM
                    assert LIN.select_gemm(100, 512, 1024) == (LIN.KIND_STREAM, 14, 4)
                else:
                    assert LIN.select_gemm(6, 512, 1024)[0] == LIN.KIND_MID
                    assert LIN.select_gemm(100, 512, 1024)[0] == LIN.KIND_GRP
            logs = []
            fwd = eng.model.forward

            def rec(*a, **k):
                out = fwd(*a, **k)
                if not torch.cuda.is_current_stream_capturing():  # graph steps: covered by the tokens
                    logs.append(out.float().cpu())
                return out
            eng.model.forward = rec
            res = {}
            for i in range(6):
                sid = eng.new_sequence()
                p = eng.tok.system_prefix("s") + eng.tok.message("user", "w%d " % i * (20 + 40 * i)) + \
                    eng.tok.header("assistant")
                eng.submit(sid, p, None, 12, temperature=0.0, on_done=lambda g, st, i=i: res.__setitem__(i, g))
            eng.run_until_idle()
            assert (eng.model._exec is not None) == on
            runs.append((res, logs))
    finally:
        LX.set_enabled(True)
        LIN._dispatch.pop((512, 1024), None)
        LIN._dispatch.pop((2048, 512), None)
        LIN._big_ranges.pop((512, 1024), None)
        LIN._big_ranges.pop((1536, 512), None)
        LIN.set_big(os.environ.get("K8SRCA_BIG_GEMM", "1"))
    (r0, l0), (r1, l1) = runs
    assert r0 == r1
    assert len(l0) == len(l1) and len(l0) > 2
    for a, b in zip(l0, l1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("graphs", [False, True])
def test_tiny_chunk_decode_rows_match_prefill_logits(graphs):
    """A short prefill chunk run as decode-attention rows (one row per token,
    each with its own causal key count; the HIP-graph decode path when the
    step has no other chunk) gives the logits of the prefill-attention path."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", num_blocks=64, use_graphs=graphs,
                                 temperature=0.0, graph_batch_sizes=(1, 2, 4, 8, 16)))
    g = torch.Generator().manual_seed(3)
    outs = []
    gmax = eng._dec_gmax
    assert gmax > 1
    # chunks inside a page / across a page boundary / across a decode partition boundary
    for n0, q in ((40, 6), (63, 5), (64, 8), (254, 6), (1000, 7)):
        s = eng.seqs[eng.new_sequence()]
        s.tokens = torch.randint(5, 1000, (n0 + q,), generator=g).tolist()
        assert eng.kvm.ensure_blocks(s, n0 + q, set())
        eng._forward([], [(s, n0)], [n0 - 1])
        s.n_cached = n0
        big = eng._forward([], [(s, q)], list(range(q))).float()
        rows = eng._forward([(s, j) for j in range(q)], [], list(range(q))).float()
        eng._dec_gmax = 1  # one decode item per row: the multi-token items are bit-identical
        rows1 = eng._forward([(s, j) for j in range(q)], [], list(range(q))).float()
        eng._dec_gmax = gmax
        torch.cuda.synchronize()
        assert torch.equal(rows, rows1), (n0, q)
        err = (big - rows).abs().max().item() / big.abs().max().item()
        assert err < 3e-2, (n0, q, err)
        assert (big.argmax(-1) == rows.argmax(-1)).float().mean().item() >= 0.8
        outs.append(err)
    if graphs:
        assert eng.stats["graph_steps"] == 10


@pytest.mark.parametrize("deferred", [True, False])
@pytest.mark.parametrize("nl", [1, 2, 3])
def test_layer_executor_norm_fuse_bit_identical(nl, deferred):
    """steps of <= 4 rows with the fused RMSNorm prologues ON
    (``st.norm_fuse == 3``: the input norm in the skinny RoPE qkv GEMM, the
    post-attention norm in the SwiGLU stream gate_up GEMM) give the same
    (prev, residual) and logits, bit for bit, as the executor with the fusion
    off and as the Python layer loop -- for 1 / 2 / 3 layers (the residual
    ping-pong between ``residual`` and ``res2`` ends on either buffer) and with
    the o / down projections either split-K with their partials deferred into
    the next norm, or not split."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.nn.functional as F
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.ops import layer_exec as LX
    from k8s_llm_rca_amd.ops import linear as LIN
    from tests.test_tp_gpu import _prefill_inputs
    keys = [(1536, 512), (2048, 512), (512, 1024)]
    saved = {k: LIN._dispatch.get(k) for k in keys}
    fuse0 = LX._norm_fuse
    try:
        LIN._dispatch[(1536, 512)] = [(16, "skinny", -1, 1)]      # qkv: skinny + RoPE / KV-write epilogue
        LIN._dispatch[(2048, 512)] = [(16, "stream", 4, 1)]       # gate_up: stream kernel's SwiGLU form
        LIN._dispatch[(512, 1024)] = ([(16, "stream", 4, 2)] if deferred   # o / down: split-K, partials deferred
                                      else [(16, "skinny", -1, 1)])
        m = LlamaModel(get_config("tiny-llama", n_layers=nl, init_std=0.08), "cuda:0", torch.bfloat16, None, seed=4)
        for T in (1, 2, 3, 4):
            outs = {}
            for mode in ("fused", "unfused", "python"):
                LX._norm_fuse = mode == "fused"
                LX.set_enabled(mode != "python")
                inp, kc, vc = _prefill_inputs(m, T, seed=T)
                logits = m.forward(inp, kc, vc).float().cpu()
                rec = {"logits": logits, "kc": kc.float().cpu()}
                if mode != "python":
                    assert m._exec is not None
                    assert m._exec.st.norm_fuse == (3 if mode == "fused" else 0), (mode, T)
                    inp, kc, vc = _prefill_inputs(m, T, seed=T)
                    res = F.embedding(inp.input_ids.long(), m.embed)
                    prev, r = m._exec.run(inp, res, kc, vc)
                    rec["prev"], rec["res"] = prev.float().cpu(), r.float().cpu()
                outs[mode] = rec
            a, b, c = outs["fused"], outs["unfused"], outs["python"]
            assert torch.equal(a["prev"], b["prev"]) and torch.equal(a["res"], b["res"]), (nl, T, deferred)
            assert torch.equal(a["logits"], b["logits"]) and torch.equal(a["logits"], c["logits"]), (nl, T, deferred)
            assert torch.equal(a["kc"], b["kc"]) and torch.equal(a["kc"], c["kc"])
    finally:
        LX._norm_fuse = fuse0
        LX.set_enabled(True)
        for k, v in saved.items():
            if v is None:
                LIN._dispatch.pop(k, None)
            else:
                LIN._dispatch[k] = v


def _mixed_step_8b(m, nd=40, npf=640, cached=128, seed=0):
    """A mixed step on Llama-3-8B shapes: ``nd`` decode rows (300-800 cached keys
    each, scattered pages of random K/V) + one ``npf``-token prefill chunk after
    ``cached`` keys.  Returns (StepInputs, k_cache, v_cache)."""
    import numpy as np
    from k8s_llm_rca_amd.models.llama import StepInputs
    from k8s_llm_rca_amd.ops import attention as A
    BS, dev = 64, "cuda"
    g = np.random.default_rng(seed)
    ctx = [int(c) for c in g.integers(300, 800, nd)]   # decode row i: key ctx-1 is its new token
    nbs = [-(-c // BS) for c in ctx] + [-(-(cached + npf) // BS)]
    perm = g.permutation(sum(nbs))
    bts, u = [], 0
    for n in nbs:
        bts.append(perm[u:u + n].tolist())
        u += n
    L = m.cfg.n_layers
    kc = (torch.randn(L, sum(nbs), m.nkv, BS, m.D, generator=torch.Generator().manual_seed(seed)) * 0.5).bfloat16().to(dev)
    vc = torch.randn(L, sum(nbs), m.nkv, m.D, BS, generator=torch.Generator().manual_seed(seed + 1)).bfloat16().to(dev)
    mb = max(nbs[:nd])
    bt_d = torch.zeros(nd, mb, dtype=torch.int32)
    for i in range(nd):
        bt_d[i, :nbs[i]] = torch.tensor(bts[i], dtype=torch.int32)
    md = A.AttnMeta(block_tables=bt_d.to(dev), ctx_lens=torch.tensor(ctx, dtype=torch.int32, device=dev),
                    q_start=torch.arange(nd + 1, dtype=torch.int32, device=dev), num_seqs=nd, decode=True,
                    ctx_lens_host=ctx, q_start_host=list(range(nd + 1)))
    A.attach_decode_plan(md, ctx, m.nq, m.nkv, BS, dev)
    tot = cached + npf
    mp_ = A.AttnMeta(block_tables=torch.tensor([bts[nd]], dtype=torch.int32, device=dev),
                     ctx_lens=torch.tensor([tot], dtype=torch.int32, device=dev),
                     q_start=torch.tensor([0, npf], dtype=torch.int32, device=dev), num_seqs=1, decode=False,
                     ctx_lens_host=[tot], q_start_host=[0, npf])
    A.attach_plan(mp_, A.plan_prefill([0, npf], m.nq // m.nkv, BS, [tot], nkv=m.nkv), dev)
    pos = ctx_pos = [c - 1 for c in ctx] + list(range(cached, tot))
    slots = [bts[i][p // BS] * BS + p % BS for i, p in enumerate(ctx_pos[:nd])] + \
        [bts[nd][p // BS] * BS + p % BS for p in range(cached, tot)]
    T = nd + npf
    ids = torch.tensor(g.integers(0, 100000, T), dtype=torch.int32, device=dev)
    inp = StepInputs(ids, torch.tensor(pos, dtype=torch.int32, device=dev),
                     torch.tensor(slots, dtype=torch.int32, device=dev), nd, md, mp_,
                     torch.tensor(list(range(nd)) + [T - 1], dtype=torch.int64, device=dev))
    return inp, kc, vc


def test_nano_batch_two_streams_bit_identical_to_serial():
    """a mixed step as two nano-batch layer stacks (decode rows on
    a high-priority side stream beside the prefill rows on the compute stream,
    ops/layer_exec.py ``_run_nano``) gives bit-identically the logits and KV of
    the same two stacks run one after the other, and agrees with the single
    combined stack to bf16 tolerance (the stacks pick their GEMM kernels for
    their own M)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.ops import layer_exec as LX
    from k8s_llm_rca_amd.ops import linear as LIN
    saved = (dict(LIN._dispatch), dict(LIN._big_ranges), LX._nano, LX._nano_serial)
    try:
        dev = torch.device("cuda:0")
        LIN.reserve_lib_workspace(dev)
        assert LIN.load_dispatch(LIN.dispatch_path("llama3-8b"))
        LIN.load_big(LIN.big_path("llama3-8b"))
        LIN.reserve_dispatch_scratch(dev)
        m = LlamaModel(get_config("llama3-8b", n_layers=2), "cuda:0", torch.bfloat16, None, seed=2)
        outs = {}
        for mode in ("single", "serial", "streams"):
            LX._nano, LX._nano_serial = mode != "single", mode == "serial"
            inp, kc, vc = _mixed_step_8b(m)
            n0 = m._exec.nano_steps if m._exec is not None else 0
            logits = m.forward(inp, kc, vc).float()
            torch.cuda.synchronize()
            assert m._exec.nano_steps == n0 + (mode != "single"), mode
            outs[mode] = (logits.cpu(), kc.float().cpu(), vc.float().cpu())
        a, b, c = outs["streams"], outs["serial"], outs["single"]
        assert all(torch.equal(x, y) for x, y in zip(a, b))
        assert torch.isfinite(a[0]).all()
        rel = ((a[0] - c[0]).norm() / c[0].norm()).item()
        assert rel < 0.02, rel
        assert (a[0].argmax(-1) == c[0].argmax(-1)).float().mean().item() >= 0.9
    finally:
        LIN._dispatch.clear()
        LIN._dispatch.update(saved[0])
        LIN._big_ranges.clear()
        LIN._big_ranges.update(saved[1])
        LX._nano, LX._nano_serial = saved[2], saved[3]


def test_token_flag_wait_same_tokens():
    """Knob token_flag: the engine waits for each step's tokens by
    polling a pinned-host flag that a one-wave kernel raises after their copy,
    instead of hipEventSynchronize; the generations are the same as with the
    event wait, and the flag ran (its sequence advanced)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd import knobs as K
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.engine import sampler as SM
    outs = []
    min_rows = SM.TOKEN_FLAG_MIN_ROWS
    SM.TOKEN_FLAG_MIN_ROWS = 1  # every step polls (the default keeps the event wait below 16 rows)
    for on in (False, True):
        with K.override(token_flag=on):
            eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", num_blocks=256, temperature=0.0,
                                         graph_batch_sizes=(1, 2, 4, 8)))
            res = {}
            for i in range(5):
                sid = eng.new_sequence()
                p = eng.tok.system_prefix("s") + eng.tok.message("user", "flag %d " % i * (10 + 7 * i)) + \
                    eng.tok.header("assistant")
                eng.submit(sid, p, None, 16, temperature=0.0, on_done=lambda g, st, i=i: res.__setitem__(i, g))
            eng.run_until_idle()
            assert (eng._tflag_seq > 0) == on
            outs.append(res)
    SM.TOKEN_FLAG_MIN_ROWS = min_rows
    assert outs[0] == outs[1] and all(len(v) == 16 for v in outs[0].values())


def test_kv_stage_round_trip_kernel():
    """k8s_kv_stage + the DMA copies of the KV host tier (engine/kv_offload.py):
    pages swapped out and back into other pool pages are bit-identical, across
    staging chunks and runs of consecutive host slots."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.kv_cache import KVPool
    from k8s_llm_rca_amd.engine.kv_offload import KVHostTier
    pool = KVPool(3, 8, 128, 40, 64, "cuda", torch.bfloat16)
    g = torch.Generator(device="cuda").manual_seed(3)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g, device="cuda"))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g, device="cuda"))
    blocks = pool.alloc(12)
    src = [blocks[i] for i in (0, 1, 2, 5, 7, 8, 11)]
    ref_k, ref_v = pool.k[:, src].clone(), pool.v[:, src].clone()
    per = KVPool.bytes_per_block(3, 8, 128, 64)
    t = KVHostTier(pool, 16, staging_bytes=3 * per)  # 3 blocks per staging chunk
    assert t.chunk == 3
    slots = t.swap_out(src)
    t.drain()
    assert pool.free_blocks == 40 - 12 + len(src)
    pool.k.zero_()
    pool.v.zero_()
    dst = pool.alloc(len(src))[::-1]
    ev = t.swap_in(slots, dst)
    ev.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(pool.k[:, dst], ref_k) and torch.equal(pool.v[:, dst], ref_v)
    t.close()


def test_kv_host_tier_same_tokens():
    """An engine whose pool is too small for its idle threads swaps them to the
    host tier and back: the generations (greedy) are the same as with a pool
    that never runs short, nothing is dropped or re-prefilled."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.engine.kv_cache import KVPool

    def run(**kw):
        eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", temperature=0.0,
                                     graph_batch_sizes=(1, 2, 4, 8), **kw))
        outs = {}
        sids = [eng.new_sequence() for _ in range(4)]
        for r in range(3):
            for i, sid in enumerate(sids):
                base = eng.seqs[sid].tokens if r else eng.tok.system_prefix("s")
                p = base + eng.tok.message("user", ("t%d r%d " % (i, r)) * 12) + eng.tok.header("assistant")
                eng.submit(sid, p, None, 12, temperature=0.0, on_done=lambda g, st, k=(r, i): outs.__setitem__(k, g))
                eng.run_until_idle()
        eng.stop()
        return eng, outs

    ref, want = run(num_blocks=256)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 64)
    eng, got = run(num_blocks=10, kv_host_gb=64 * per / (1 << 30), kv_host_watermark=2)
    assert got == want and all(v is not None for v in got.values())
    assert eng.stats["evictions"] == 0 and eng.stats["swap_outs"] > 0 and eng.stats["swap_ins"] > 0
    assert eng.stats["prefill_tokens"] == ref.stats["prefill_tokens"]
    eng.kv_host.close()


def test_kv_host_tier_concurrent_runs_same_tokens():
    """Every thread's next run submitted at once while the pool holds only a few
    threads: swap-ins run on the copy stream while other rows decode, and a run
    is scheduled only once its pages have landed -- the same greedy tokens as a
    pool that never runs short."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    from k8s_llm_rca_amd.engine.kv_cache import KVPool

    def run(**kw):
        eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", temperature=0.0,
                                     graph_batch_sizes=(1, 2, 4, 8), **kw))
        outs = {}
        sids = [eng.new_sequence() for _ in range(6)]
        for r in range(3):
            for half in (sids[:3], sids[3:]):  # three threads run together, the other three idle
                for sid in half:
                    i = sids.index(sid)
                    base = eng.seqs[sid].tokens if r else eng.tok.system_prefix("s")
                    p = base + eng.tok.message("user", ("c%d r%d " % (i, r)) * (8 + 3 * i)) + \
                        eng.tok.header("assistant")
                    eng.submit(sid, p, None, 10, temperature=0.0,
                               on_done=lambda g, st, k=(r, i): outs.__setitem__(k, g))
                eng.run_until_idle()
        eng.stop()
        return eng, outs

    ref, want = run(num_blocks=512)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 64)
    eng, got = run(num_blocks=20, kv_host_gb=128 * per / (1 << 30), kv_host_watermark=2)
    assert got == want and all(v is not None for v in got.values())
    assert eng.stats["swap_ins"] > 0 and eng.stats["evictions"] == 0
    eng.kv_host.close()
