"""Custom xGMI all-reduce (B14): IPC buffers, flag protocol, one-/two-shot.

The box has one GPU, so the ranks are processes sharing cuda:0: the IPC
export/open, the cross-process release/acquire flags and the parity double
buffering are exercised for real; only the xGMI link itself is not.  Results
must be bit-identical to a fixed-order fp32 sum rounded to bf16 on every rank.
"""
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


def _inp(rank, n, it, mode):
    g = torch.Generator().manual_seed(rank * 1_000_003 + n * 31 + it * 7 + mode)
    return torch.randn(n, generator=g).bfloat16()


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ar = XgmiAllReduce(dist.group.WORLD, max_bytes=4 << 20, timeout_s=20.0)
    bad = []
    for mode in (1, 2):
        for n in (8, 4096, 65536 + 8 * 13, 1 << 20):
            for it in range(6):  # > 2 epochs per block: exercises parity reuse
                x = _inp(rank, n, it, mode).cuda()
                ar(x, mode=mode)
                ref = sum(_inp(r, n, it, mode).float() for r in range(world)).bfloat16()
                if not torch.equal(x.cpu(), ref):
                    bad.append((mode, n, it, (x.cpu().float() - ref.float()).abs().max().item()))
    # sizes alternating large / small back to back with no host sync between
    # calls: the block count changes every call (per-block epochs raced)
    xs, refs = [], []
    for it, n in enumerate([1 << 20, 4096, 1 << 19, 8, 65536, 1 << 20, 2048, 300008, 16, 1 << 20] * 2):
        mode = 1 + it % 2
        x = _inp(rank, n, 100 + it, mode).cuda()
        ar(x, mode=mode)
        xs.append(x)
        refs.append(sum(_inp(r, n, 100 + it, mode).float() for r in range(world)).bfloat16())
    torch.cuda.synchronize()
    for it, (x, ref) in enumerate(zip(xs, refs)):
        if not torch.equal(x.cpu(), ref):
            bad.append(("alt", x.numel(), it, (x.cpu().float() - ref.float()).abs().max().item()))
    status = ar.status()
    ar.close()
    torch.save({"bad": bad, "status": status}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_processes_sharing_one_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r, v in enumerate(res):
        assert v["status"] == 0, f"rank {r}: a flag wait timed out"
        assert not v["bad"], (r, v["bad"][:4])


def _an_worker(rank, world, port, out_dir):
    """Fused all-reduce + residual add + RMSNorm vs all-reduce, then the rmsnorm
    kernel: one-shot bit-identical, two-shot within a bf16 ulp of it and the
    same on every rank (the inverse norm comes from the same partial sums)."""
    import torch.distributed as dist
    from k8s_llm_rca_amd.ops import norm as N
    from k8s_llm_rca_amd.parallel.xgmi import XgmiAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ar = XgmiAllReduce(dist.group.WORLD, max_bytes=4 << 20, timeout_s=20.0)
    res_out = {}
    for T, H, mode in ((1, 4096, 1), (8, 8192, 1), (33, 1024, 1), (128, 8192, 2), (300, 1024, 2), (37, 4096, 2)):
        for it in range(3):
            g = torch.Generator().manual_seed(T * 131 + H + it)
            resid0 = torch.randn(T, H, generator=g).bfloat16().cuda()
            w = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16().cuda()
            x = _inp(rank, T * H, it, mode).view(T, H).cuda()
            r_f, y_f = resid0.clone(), torch.empty_like(resid0)
            ar.addnorm(x.clone(), r_f, w, y_f, 1e-5, mode=mode)
            xa = x.clone()
            ar(xa.view(-1), mode=mode)
            r_u, y_u = resid0.clone(), torch.empty_like(resid0)
            N.rmsnorm(xa, w, 1e-5, residual=r_u, out=y_u)
            torch.cuda.synchronize()
            res_out[(T, H, mode, it)] = (r_f.cpu(), y_f.cpu(), r_u.cpu(), y_u.cpu())
    status = ar.status()
    ar.close()
    torch.save({"res": res_out, "status": status}, os.path.join(out_dir, f"an{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_fused_addnorm_processes_sharing_one_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_an_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"an{r}.pt"), weights_only=True) for r in range(world)]
    for r, v in enumerate(res):
        assert v["status"] == 0
        for (T, H, mode, it), (r_f, y_f, r_u, y_u) in v["res"].items():
            assert torch.equal(r_f, r_u), (r, T, H, mode)  # the residual update is exact in both forms
            if mode == 1:
                assert torch.equal(y_f, y_u), (r, T, H)
            else:
                torch.testing.assert_close(y_f.float(), y_u.float(), atol=0, rtol=2.0 ** -7)
            # every rank holds the same normed rows
            assert torch.equal(y_f, res[0]["res"][(T, H, mode, it)][1])
