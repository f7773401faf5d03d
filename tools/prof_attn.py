"""Run one paged-attention configuration repeatedly (for rocprofv3 PMC passes).

    python tools/prof_attn.py --mode prefill --S 8 --q 512 --ctx 3000 --iters 20
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402
from tools.bench_kernels import make_meta  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["prefill", "decode"], default="prefill")
    ap.add_argument("--S", type=int, default=8)
    ap.add_argument("--q", type=int, default=512)
    ap.add_argument("--ctx", type=int, default=3000)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    nq, nkv, BS, dev = 32, 8, 64, "cuda"
    torch.manual_seed(0)
    q_len = 1 if args.mode == "decode" else args.q
    meta, nb = make_meta([args.ctx] * args.S, [q_len] * args.S, nq, nkv, BS, dev, args.mode == "decode")
    kc = torch.randn(nb, nkv, BS, 128, device=dev).bfloat16()
    vc = torch.randn(nb, nkv, 128, BS, device=dev).bfloat16()
    q = torch.randn(q_len * args.S, (nq + 2 * nkv) * 128, device=dev).bfloat16()
    out = torch.empty(q_len * args.S, nq * 128, device=dev).bfloat16()
    for _ in range(args.iters):
        A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128), out=out)
    torch.cuda.synchronize()
    print("ok", args)


if __name__ == "__main__":
    main()
