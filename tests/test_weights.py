"""HF-format safetensors checkpoints <-> the engine's (TP-sharded) layout."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from k8s_llm_rca_amd.models.config import get_config
from k8s_llm_rca_amd.models.llama import LlamaModel
from k8s_llm_rca_amd.models.weights import config_from_hf, load_safetensors, save_safetensors


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _caches(cfg, BS):
    kf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, BS, 128, generator=torch.Generator().manual_seed(7)) * 0.5
    vf = torch.randn(cfg.n_layers, 6, cfg.n_kv_heads, 128, BS, generator=torch.Generator().manual_seed(8))
    return kf, vf


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_save_load_roundtrip_exact(name):
    from tests.test_parallel import _inputs as mk
    cfg = get_config(name)
    ref = LlamaModel(cfg, "cpu", torch.float32, None, seed=4, init_mode="full_slice")
    with tempfile.TemporaryDirectory() as d:
        save_safetensors(ref, d)
        cfg2 = config_from_hf(d, name)
        assert (cfg2.hidden, cfg2.n_layers, cfg2.n_heads, cfg2.n_kv_heads, cfg2.n_experts) == \
            (cfg.hidden, cfg.n_layers, cfg.n_heads, cfg.n_kv_heads, cfg.n_experts)
        m = LlamaModel(cfg2, "cpu", torch.float32, None, init=False)
        load_safetensors(m, d)
    inp, BS = mk(cfg)
    kf, vf = _caches(cfg, BS)
    a = ref.forward(inp, kf.clone(), vf.clone())
    inp, _ = mk(cfg)
    b = m.forward(inp, kf.clone(), vf.clone())
    assert torch.equal(a, b)


def _tp_load(rank, world, port, ckpt, out):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import ParallelContext
    from tests.test_parallel import _inputs as mk
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, ep_size=world, ep_rank=rank,
                         ep_group=dist.group.WORLD)
    cfg = config_from_hf(ckpt)
    m = LlamaModel(cfg, "cpu", torch.float32, pc, init=False)
    load_safetensors(m, ckpt)
    inp, BS = mk(cfg)
    kf, vf = _caches(cfg, BS)
    h0 = (rank * cfg.n_kv_heads) // world if cfg.n_kv_heads < world else rank * m.nkv
    logits = m.forward(inp, kf[:, :, h0:h0 + m.nkv].contiguous(), vf[:, :, h0:h0 + m.nkv].contiguous())
    if rank == 0:
        torch.save(logits[:, : cfg.vocab_size], out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_tp2_loads_its_shards(name):
    from tests.test_parallel import _inputs as mk
    cfg = get_config(name)
    ref = LlamaModel(cfg, "cpu", torch.float32, None, seed=4, init_mode="full_slice")
    with tempfile.TemporaryDirectory() as d:
        save_safetensors(ref, d)
        out = os.path.join(d, "logits.pt")
        mp.spawn(_tp_load, args=(2, _free_port(), d, out), nprocs=2, join=True)
        got = torch.load(out, weights_only=True)
    inp, BS = mk(cfg)
    kf, vf = _caches(cfg, BS)
    want = ref.forward(inp, kf, vf)[:, : cfg.vocab_size]
    torch.testing.assert_close(got, want, atol=2e-4, rtol=2e-4)


def test_engine_runs_from_checkpoint_dir():
    from k8s_llm_rca_amd.engine.engine import EngineConfig, LLMEngine
    cfg = get_config("tiny-llama")
    ref = LlamaModel(cfg, "cpu", torch.float32, None, seed=4, init_mode="full_slice")
    with tempfile.TemporaryDirectory() as d:
        save_safetensors(ref, d)
        eng = LLMEngine(EngineConfig(weights=d, device="cpu", dtype=torch.float32, num_blocks=32, block_size=32,
                                     max_batch_tokens=64, temperature=0.0))
    sid = eng.new_sequence()
    out = {}
    eng.submit(sid, eng.tok.system_prefix("s") + eng.tok.header("assistant"), None, 6,
               on_done=lambda g, st: out.setdefault("g", g))
    eng.run_until_idle()
    assert len(out["g"]) == 6
