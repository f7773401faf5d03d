"""TP=N vs TP=1 logits of one prefill on ONE GPU (N processes sharing cuda:0,
gloo host group, every collective on the xGMI kernels), per layer count.

Separates a TP bug from bf16 drift: a correct TP engine differs from TP=1
only by the rounding of its partial sums (each rank's row-parallel output is
rounded to bf16 before the all-reduce), which starts at ~2^-9 relative after
one layer and grows through a random-init stack; a wrong collective or shard
is already O(1) after one layer.

    python tools/tp_check.py --layers 1,2,8,32 --tokens 300,1100 --tp 2
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _worker(rank, world, port, out_dir, layers, Ts, max_mb, model):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    from k8s_llm_rca_amd.knobs import set_knob
    set_knob("ar_max_mb", max_mb)
    from k8s_llm_rca_amd.models.config import get_config
    from k8s_llm_rca_amd.models.llama import LlamaModel
    from k8s_llm_rca_amd.parallel.groups import ParallelContext, attach_custom_allreduce
    from test_tp_gpu import _prefill_inputs
    pc = None
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pc = attach_custom_allreduce(ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD),
                                     same_gpu=True)
    out = {}
    for nl in layers:
        m = LlamaModel(get_config(model, n_layers=nl), "cuda:0", torch.bfloat16, pc, seed=11, init_mode="full_slice")
        for T in Ts:
            inp, kc, vc = _prefill_inputs(m, T)
            out[(nl, T)] = {"logits": m.forward(inp, kc, vc).float().cpu(),
                            "exec": m._exec is not None and m._exec.fits(T)}
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="1,2,8,32")
    ap.add_argument("--tokens", default="300,1100")
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--max-mb", type=int, default=4)
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()
    layers = [int(x) for x in a.layers.split(",")]
    Ts = [int(x) for x in a.tokens.split(",")]
    import socket
    res = []
    with tempfile.TemporaryDirectory() as d:
        for world in (a.tp, 1):
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            mp.spawn(_worker, args=(world, port, d, layers, Ts, a.max_mb, a.model), nprocs=world, join=True)
        x = torch.load(os.path.join(d, f"tp{a.tp}.pt"), weights_only=True)
        y = torch.load(os.path.join(d, "tp1.pt"), weights_only=True)
    for nl in layers:
        for T in Ts:
            lx, ly = x[(nl, T)]["logits"], y[(nl, T)]["logits"]
            rel = ((lx - ly).norm() / ly.norm()).item()
            top = int(lx.argmax(-1)) in set(ly.topk(5, -1).indices.view(-1).tolist())
            r = {"layers": nl, "T": T, "rel": round(rel, 5), "argmax_in_top5": top, "exec": x[(nl, T)]["exec"],
                 "finite": bool(torch.isfinite(lx).all())}
            res.append(r)
            print(json.dumps(r), flush=True)
    print(json.dumps({"status": x.get("status")}))


if __name__ == "__main__":
    main()
