"""Offline GEMM tuning for the decode buckets (PyTorch TunableOp over hipBLASLt).

    python tools/tune_gemms.py --out k8s_llm_rca_amd/data/tunableop_mi355x.csv [--model llama3-8b]

Pure-decode steps run in HIP graphs whose batch sizes are bucketed
(EngineConfig.graph_batch_sizes), so their projection GEMMs have a small,
known set of (M, N, K) shapes.  hipBLASLt's default heuristic picks a poor
solution for several of them (o_proj at 1.8 TB/s for every M); TunableOp
times every hipBLASLt solution per shape and records the winner.  The engine
loads the table read-only (no online tuning): other shapes keep the default.
Prints default vs tuned time per shape.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.models.config import get_config  # noqa: E402


def shapes_for(model: str, tp: int = 1):
    mc = get_config(model)
    H, I = mc.hidden, mc.intermediate
    qkv = (mc.n_heads + 2 * mc.n_kv_heads) * mc.head_dim // tp
    out = [(qkv, H), (H, mc.n_heads * mc.head_dim // tp)]
    if not mc.n_experts:
        out += [(H, I // tp), (2 * I // tp, H)]
    out.append((mc.vocab_size // tp, H))  # lm_head over the sampled rows
    return out


def write_table(path):
    """TunableOp's results file format (validators, then one line per tuned GEMM)."""
    T = torch.cuda.tunable
    with open(path, "w") as f:
        for k, v in T.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for op, params, sol, t in T.get_results():
            f.write(f"{op},{params},{sol},{t}\n")


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None, help="default: the engine's table path for --model/--tp")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ms", default="1,2,4,8,16,24,32,48,64,96,128,160,192,224,256")
    ap.add_argument("--tp", type=int, default=1)
    a = ap.parse_args()
    if a.out is None:
        from k8s_llm_rca_amd.ops.gemm_tuning import table_path
        a.out = table_path(a.model, a.tp)
    dev = torch.device("cuda")
    ms = [int(m) for m in a.ms.split(",")]
    shapes = shapes_for(a.model, a.tp)
    ws = {s: torch.randn(s, dtype=torch.bfloat16, device=dev) * 0.02 for s in shapes}
    xs = {m: {k: torch.randn(m, k, dtype=torch.bfloat16, device=dev) for (_, k) in shapes} for m in ms}
    base = {}
    for m in ms:
        for (n, k) in shapes:
            base[(m, n, k)] = bench(lambda: torch.matmul(xs[m][k], ws[(n, k)].t()))
    T = torch.cuda.tunable
    T.enable(True)
    T.tuning_enable(True)
    T.set_filename(os.path.abspath(a.out) + ".autosave", insert_device_ordinal=False)
    T.set_max_tuning_iterations(30)
    T.set_max_tuning_duration(60)
    for m in ms:
        for (n, k) in shapes:
            torch.matmul(xs[m][k], ws[(n, k)].t())
    torch.cuda.synchronize()
    T.tuning_enable(False)
    write_table(a.out)
    tot_b = tot_t = 0.0
    for m in ms:
        for (n, k) in shapes:
            t = bench(lambda: torch.matmul(xs[m][k], ws[(n, k)].t()))
            b = base[(m, n, k)]
            tot_b += b
            tot_t += t
            gb = n * k * 2 / 1e9
            print(f"M{m:4d} N{n:6d} K{k:6d}  default {b:7.1f}us ({gb / b * 1e3:4.2f} TB/s)  "
                  f"tuned {t:7.1f}us ({gb / t * 1e3:4.2f} TB/s)", flush=True)
    print(f"total default {tot_b:.1f}us tuned {tot_t:.1f}us")


if __name__ == "__main__":
    main()
