"""KV host tier (engine/kv_offload.py) on CPU: page round trip, and an engine
that swaps idle threads to the host instead of dropping them generates the
same tokens as one whose pool never runs short (GPU form:
tests/test_model_gpu.py::test_kv_host_tier_same_tokens).

Reference: the threads being kept are the assistants' conversations that
``/root/reference/common/openai_generic_assistant.py:45-51`` re-sends on every run."""
import torch

from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
from k8s_llm_rca_amd.engine.kv_cache import KVPool
from k8s_llm_rca_amd.engine.kv_offload import KVHostTier, _runs


def test_runs():
    assert _runs([3, 4, 5, 9, 10, 2]) == [(0, 3, 3), (3, 9, 2), (5, 2, 1)]
    assert _runs([]) == []


def test_host_tier_round_trip_cpu():
    pool = KVPool(3, 2, 16, 12, 32, "cpu", torch.float32)
    g = torch.Generator().manual_seed(0)
    pool.k.copy_(torch.randn(pool.k.shape, generator=g))
    pool.v.copy_(torch.randn(pool.v.shape, generator=g))
    blocks = pool.alloc(5)
    src = [blocks[0], blocks[2], blocks[4]]
    ref_k, ref_v = pool.k[:, src].clone(), pool.v[:, src].clone()
    t = KVHostTier(pool, 8)
    slots = t.swap_out(src)
    assert len(slots) == 3 and t.free_slots == 5
    assert pool.free_blocks == 12 - 2  # the swapped pages went back (CPU: copy is synchronous)
    pool.k.zero_()
    pool.v.zero_()
    dst = pool.alloc(3)
    assert t.swap_in(slots, dst) is None and t.free_slots == 8
    assert torch.equal(pool.k[:, dst], ref_k) and torch.equal(pool.v[:, dst], ref_v)
    r = t.report()
    assert r["out_blocks"] == 3 and r["in_blocks"] == 3 and r["peak_host_blocks"] == 3


def _engine(**kw):
    cfg = dict(model="tiny-llama", device="cpu", dtype=torch.float32, block_size=32, max_batch_tokens=128,
               temperature=0.0)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg))


def _rounds(eng, n_threads=4, rounds=2):
    outs = {}
    sids = [eng.new_sequence() for _ in range(n_threads)]
    for r in range(rounds):
        for i, sid in enumerate(sids):
            base = eng.seqs[sid].tokens if r else eng.tok.system_prefix("s")
            p = base + eng.tok.message("user", ("x%d r%d " % (i, r)) * 12) + eng.tok.header("assistant")
            eng.submit(sid, p, None, 6, on_done=lambda g, st, k=(r, i): outs.__setitem__(k, g))
            eng.run_until_idle()
    return outs


def test_engine_swaps_idle_threads_instead_of_dropping():
    ref = _engine(num_blocks=256)
    want = _rounds(ref)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 32, elem=4)
    eng = _engine(num_blocks=12, kv_host_gb=64 * per / (1 << 30), kv_host_watermark=2)
    assert eng.kv_host is not None and eng.kv_host.host_blocks == 64
    got = _rounds(eng)
    assert got == want
    assert eng.stats["evictions"] == 0 and eng.stats["swap_outs"] > 0 and eng.stats["swap_ins"] > 0
    # every run after the first re-prefills only its new message, as with the big pool
    assert eng.stats["prefill_tokens"] == ref.stats["prefill_tokens"]
    assert eng.stats["recompute_tokens"] == ref.stats["recompute_tokens"]


def test_full_host_tier_falls_back_to_dropping():
    per = None
    ref = _engine(num_blocks=256)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 32, elem=4)
    eng = _engine(num_blocks=12, kv_host_gb=3 * per / (1 << 30), kv_host_watermark=2)
    got = _rounds(eng)
    assert len(got) == 8  # every run completes
    assert eng.stats["evictions"] + eng.kv_host.stats["host_dropped_blocks"] > 0


def test_release_frees_host_slots():
    ref = _engine(num_blocks=256)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 32, elem=4)
    eng = _engine(num_blocks=12, kv_host_gb=64 * per / (1 << 30), kv_host_watermark=2)
    _rounds(eng, rounds=1)
    held = [s.id for s in eng.seqs.values() if s.host]
    assert held
    for sid in list(eng.seqs):
        eng.release_sequence(sid)
    assert eng.kv_host.free_slots == 64 and eng.kv.free_blocks == 12


def test_prometheus_reports_host_tier():
    from k8s_llm_rca_amd.api.http import prometheus_text
    from k8s_llm_rca_amd.api.service import AssistantService
    from k8s_llm_rca_amd.engine.backend import EngineBackend
    ref = _engine(num_blocks=256)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 32, elem=4)
    eng = _engine(num_blocks=12, kv_host_gb=16 * per / (1 << 30), kv_host_watermark=2)
    _rounds(eng, rounds=1)
    txt = prometheus_text(AssistantService(EngineBackend(eng)), eng)
    assert "k8srca_kv_host_free_blocks" in txt and "k8srca_engine_swap_outs" in txt


class _Ev:
    """A copy-completion event stand-in (CPU): done once ``done`` is set."""
    def __init__(self):
        self.done = False

    def query(self):
        return self.done

    def synchronize(self):
        self.done = True


def test_pages_under_a_swap_in_are_released_only_after_it_lands():
    """A thread dropped while its swap-in copy is still on the copy stream (a
    cancelled run, a released thread) gives its pages back only once the copy
    has landed, and it is never chosen for eviction or preemption meanwhile."""
    from k8s_llm_rca_amd.engine.types import Sequence
    ref = _engine(num_blocks=256)
    per = KVPool.bytes_per_block(ref.mc.n_layers, ref.model.nkv, ref.model.D, 32, elem=4)
    eng = _engine(num_blocks=12, kv_host_gb=8 * per / (1 << 30), kv_host_watermark=0)
    kvm = eng.kvm
    s = Sequence(eng.new_sequence())
    eng.seqs[s.id] = s
    s.blocks = eng.kv.alloc(3)
    ev = _Ev()
    s.loading = ev
    assert kvm.loading(s)
    kvm.evict(12, set())            # an idle thread under a swap-in is not evicted
    assert len(s.blocks) == 3
    free0 = eng.kv.free_blocks
    kvm.drop(s)                     # e.g. its run was cancelled mid-copy
    assert s.blocks == [] and s.loading is None and eng.kv.free_blocks == free0
    assert eng.kv_host.poll() == 0 and eng.kv.free_blocks == free0   # still being written
    ev.done = True
    assert eng.kv_host.poll() == 3 and eng.kv.free_blocks == free0 + 3
