"""Can two ranks share one MI355X over RCCL (backend "nccl")?

The TP engine sends messages above the xGMI communicator's buffer (prefill
all-reduces, the EP prefill all-to-alls) through RCCL; on a one-GPU box the
only way to execute that branch for real is two ranks on the same device.
Prints one JSON line per rank: whether init, all_reduce and all_to_all_single
ran and matched the expected values.

usage (GPU box): python tools/rccl_same_gpu.py
"""
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _rank(r, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world))
    out = {"rank": r}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=r, world_size=world, device_id=torch.device("cuda:0"))
        out["init"] = True
        x = torch.full((1 << 20,), float(r + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["all_reduce_ok"] = bool(torch.all(x == world * (world + 1) / 2).item())
        send = torch.arange(world * 4, device="cuda:0", dtype=torch.float32) + 100 * r
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send)
        torch.cuda.synchronize()
        exp = torch.cat([torch.arange(4, device="cuda:0", dtype=torch.float32) + 4 * r + 100 * p for p in range(world)])
        out["all_to_all_ok"] = bool(torch.equal(recv, exp))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- report, do not hang the peer
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    q.put(out)


def main():
    world, port = 2, 29613
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = []
    for _ in range(world):
        try:
            res.append(q.get(timeout=120))
        except Exception:  # noqa: BLE001
            res.append({"error": "timeout"})
    for p in ps:
        p.join(30)
        if p.is_alive():
            p.kill()
    for r in sorted(res, key=lambda d: d.get("rank", 9)):
        print(json.dumps(r), flush=True)
    return 0 if all(r.get("all_reduce_ok") and r.get("all_to_all_ok") for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
