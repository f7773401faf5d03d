"""TP / EP across DISTINCT GPUs (VERDICT r5 #4a; SURVEY.md §4.5's "guarded
real test that runs only when >= 2 GPUs are visible").

Every other multi-rank GPU test puts its ranks on cuda:0 (a one-GPU box), with
a gloo host group and the xGMI collectives' grids capped at 32 blocks.  These
run the deployment's own configuration instead: one process per device, a
"nccl" (RCCL) group, the communicator built by ``attach_custom_allreduce``
(uncapped grids, cross-device ``hipIpcOpenMemHandle`` mappings, the cross-XCD
and cross-device flag protocol), world 2 and world ``min(8, device_count)``.
They skip cleanly on a box with fewer than two GPUs (the driver's 1-GPU test
tier) and are what the first multi-GPU node runs.

Reference: the sequential loops these engines replace,
``/root/reference/test_with_file.py:64,111,159``.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _n_gpus() -> int:
    # device_count() does not initialise the GPU on this image
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


N_GPUS = _n_gpus()
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(N_GPUS < 2, reason="needs >= 2 GPUs (one process per device)")]
WORLDS = sorted({2, min(8, max(N_GPUS, 2))})


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    """One process per device, an RCCL group, the xGMI communicator on top."""
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.groups import ParallelContext, attach_custom_allreduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    pc = attach_custom_allreduce(ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD,
                                                 ep_size=world, ep_rank=rank, ep_group=dist.group.WORLD))
    assert pc.custom_ar is not None and pc.xgmi_only and pc.rccl_ok()
    return pc


def _done(pc, out_dir, rank, res):
    import torch.distributed as dist
    torch.cuda.synchronize()
    res["status"] = pc.custom_ar.status()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    pc.custom_ar.close()
    dist.destroy_process_group()


def _collectives_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from tests.test_allreduce_gpu import _inp
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    pc = _init(rank, world, port)
    car = pc.custom_ar
    res = {"exact_bad": [], "a2a_ok": True}
    # one- and two-shot: bit-identical to the fixed-order fp32 sum rounded to bf16, on every rank
    for mode in (1, 2):
        for n in (8 * world, 4096, 65536 + 8 * 13 * world, 1 << 20):
            for it in range(4):   # > 2 epochs per block: the parity double buffer is reused
                x = _inp(rank, n, it, mode).cuda()
                car(x, mode=mode)
                ref = sum(_inp(r, n, it, mode).float() for r in range(world)).bfloat16()
                if not torch.equal(x.cpu(), ref):
                    res["exact_bad"].append((mode, n, it))
    # larger than the buffer (a 16 MiB communicator): chunked two-shot, and RCCL on the same data
    small = XgmiAllReduce(dist.group.WORLD, max_bytes=16 << 20, timeout_s=30.0)
    for mib in (32, 128):
        n = (mib << 20) // 2
        xs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1000 * mib + r))
              .bfloat16() for r in range(world)]
        ref, mag = xs[0].float(), xs[0].float().abs()
        for x in xs[1:]:
            ref += x.float()
            mag += x.float().abs()
        a, b = xs[rank].clone(), xs[rank].clone()
        small(a)
        dist.all_reduce(b)
        torch.cuda.synchronize()
        for tag, got in (("xgmi", a), ("rccl", b)):
            err = (got.float() - ref).abs()
            # RCCL rounds every partial sum of its ring to bf16: <= world roundings of <= sum |x| each
            res[f"{tag}_{mib}"] = (mag * world * 2 ** -8 + 1e-6).sub(err).min().item()   # >= 0: within bound
        del xs, ref, mag, a, b
    res["small_status"] = small.status()
    small.close()
    # fused all-reduce + residual add + RMSNorm (the executor's row-parallel epilogue)
    T, H = 64, 4096
    g = torch.Generator().manual_seed(5)
    res0 = torch.randn(T, H, generator=g).bfloat16()
    nw = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
    parts = [torch.randn(T, H, generator=torch.Generator().manual_seed(50 + r)).bfloat16() for r in range(world)]
    for mode in (1, 2):
        r_ = res0.cuda().clone()
        y = torch.empty(T, H, dtype=torch.bfloat16, device="cuda")
        car.addnorm(parts[rank].cuda(), r_, nw.cuda(), y, 1e-5, mode)
        torch.cuda.synchronize()
        tot = sum(p.float() for p in parts) + res0.float()
        yr = tot * torch.rsqrt(tot.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
        res[f"addnorm_{mode}"] = (float((r_.float().cpu() - tot).abs().max() / tot.abs().max()),
                                  float((y.float().cpu() - yr).abs().max() / yr.abs().max()))
    # EP all-to-all: recv[r] = rank r's send[this rank], exactly
    chunk = 4096
    send = torch.stack([torch.full((chunk,), float(100 * rank + d), dtype=torch.bfloat16) for d in range(world)]).cuda()
    recv = torch.empty_like(send)
    car.all_to_all(send, recv)
    torch.cuda.synchronize()
    for r in range(world):
        if not bool((recv[r].float() == float(100 * r + rank)).all()):
            res["a2a_ok"] = False
    _done(pc, out_dir, rank, res)


@pytest.mark.parametrize("world", WORLDS)
def test_xgmi_collectives_across_devices(world):
    """One- / two-shot all-reduce (bit-exact), the chunked 32 / 128 MiB form and
    RCCL's all-reduce on the same data (fp32-sum bound), the fused add + RMSNorm,
    and the EP all-to-all -- with uncapped grids over real peer mappings."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_collectives_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        rs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in rs:
        assert r["status"] == 0 and r["small_status"] == 0
        assert r["exact_bad"] == [], r["exact_bad"]
        for k in ("xgmi_32", "xgmi_128", "rccl_32", "rccl_128"):
            assert r[k] >= 0, (k, r[k])
        for mode in (1, 2):
            er, ey = r[f"addnorm_{mode}"]
            assert er < 1e-2 and ey < 2e-2, (mode, er, ey)
        assert r["a2a_ok"]


def _push_worker(rank, world, port, out_dir):
    from tests.test_tp_push_gpu import _run_cases
    pc = _init(rank, world, port)
    rows = _run_cases(pc.custom_ar, rank, world)
    _done(pc, out_dir, rank, {"rows": rows})


@pytest.mark.parametrize("world", WORLDS)
def test_push_epilogue_across_devices(world):
    """The o / down GEMM's push epilogue (posted remote writes into the peers'
    slots + per-strip flags) is bit-identical to the staged path across devices."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_push_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        rs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in rs:
        assert r["status"] == 0
        for row in r["rows"]:
            assert row["same"] and row["same_parity"], row
            assert row["err_res"] < 1e-2 and row["err_y"] < 2e-2, row


def _logits_worker(rank, world, port, out_dir, Ts):
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from tests.test_tp_gpu import _fp32_reference_logits, _prefill_inputs
    pc = _init(rank, world, port)
    res = {}
    for nl in (2, 32):
        m = LlamaModel(get_config("llama3-8b", n_layers=nl), f"cuda:{rank}", torch.bfloat16, pc, seed=11,
                       init_mode="full_slice")
        for T in Ts:
            inp, kc, vc = _prefill_inputs(m, T)
            res[f"{nl}/{T}"] = {"logits": m.forward(inp, kc, vc).float().cpu(),
                                "exec": m._exec is not None and m._exec.fits(T)}
        del m
        torch.cuda.empty_cache()
    _done(pc, out_dir, rank, res)


def _logits_ref_worker(out_dir, Ts):
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from tests.test_tp_gpu import _fp32_reference_logits, _prefill_inputs
    torch.cuda.set_device(0)
    res = {}
    for nl in (2, 32):
        m = LlamaModel(get_config("llama3-8b", n_layers=nl), "cuda:0", torch.bfloat16, None, seed=11,
                       init_mode="full_slice")
        for T in Ts:
            inp, kc, vc = _prefill_inputs(m, T)
            res[f"{nl}/{T}"] = {"logits": m.forward(inp, kc, vc).float().cpu(), "fp32": _fp32_reference_logits(m, T)}
        del m
        torch.cuda.empty_cache()
    torch.save(res, os.path.join(out_dir, "tp1.pt"))


@pytest.mark.parametrize("world", WORLDS)
def test_llama3_8b_tp_logits_across_devices(world):
    """Llama-3-8B at TP = world over distinct devices (nccl group, uncapped xGMI
    epilogues; T = 300 through the native executor, T = 8,300 past the 64 MiB
    buffer through the Python path's chunked / RCCL-or-xGMI all-reduce): as close
    to an fp32 forward of the same weights as the TP=1 engine is."""
    Ts = (300, 8300)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_logits_worker, args=(world, _free_port(), d, Ts), nprocs=world, join=True)
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=_logits_ref_worker, args=(d, Ts))
        p.start()
        p.join()
        assert p.exitcode == 0
        a = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        b = torch.load(os.path.join(d, "tp1.pt"), weights_only=True)
    assert a["status"] == 0 and a["2/300"]["exec"] and not a["2/8300"]["exec"]
    for nl in (2, 32):
        for T in Ts:
            x, y = a[f"{nl}/{T}"]["logits"][:, :128256], b[f"{nl}/{T}"]["logits"][:, :128256]
            ref = b[f"{nl}/{T}"]["fp32"][:, :128256]
            e2 = ((x - ref).norm() / ref.norm()).item()
            e1 = ((y - ref).norm() / ref.norm()).item()
            assert e2 <= 1.25 * e1 + 1e-3, (world, nl, T, e2, e1)
            assert int(x.argmax(-1)) in set(ref.topk(5, -1).indices.view(-1).tolist()), (world, nl, T)
