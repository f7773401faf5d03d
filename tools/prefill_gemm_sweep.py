"""Prefill-regime projection GEMMs (M = 320..2048): hipBLASLt vs the 64x128-tile
grouped kernel (single expert, split-K 1/2/4) on the Llama-3-8B shapes.

    python tools/prefill_gemm_sweep.py [--ms 320,512,...]

At these M hipBLASLt's large-tile solutions leave CUs idle (M=512, N=4096
has 32 256x256 tiles for 256 CUs); the grouped kernel's 64x128 tiles give
(N/128)(M/64) workgroups.  Cold weights (rotated copies), checked vs hipBLASLt.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_rca_amd.ops import linear as L  # noqa: E402
from tools.gemm_mid_sweep import bench  # noqa: E402

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="320,384,512,640,768,1024,1536,2048")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ws = {}
    for s in SHAPES:
        n = max(2, (768 << 20) // (s[0] * s[1] * 2))
        ws[s] = [torch.randn(s, dtype=torch.bfloat16, device=dev) * 0.02 for _ in range(n)]
    for M in [int(m) for m in a.ms.split(",")]:
        tot = {"lib": 0.0, "best": 0.0}
        for (N, K) in SHAPES:
            x = torch.randn(M, K, dtype=torch.bfloat16, device=dev)
            cyc = ws[(N, K)]
            it = [0]

            def rot():
                it[0] = (it[0] + 1) % len(cyc)
                return cyc[it[0]]
            ref = L.lib_gemm(x, cyc[0]).float()
            res = {"lib": bench(lambda: L.lib_gemm(x, rot()))}
            for s in (1, 2, 4):
                if K % (64 * s):
                    continue
                y = L.gemm_grp(x, cyc[0], s).float()
                err = (y - ref).abs().max().item() / max(1e-6, ref.abs().max().item())
                assert err < 2e-2, (M, N, K, s, err)
                res[f"grp:x{s}"] = bench(lambda s=s: L.gemm_grp(x, rot(), s))
            fl = 2.0 * M * N * K
            best = min(res, key=res.get)
            tot["lib"] += res["lib"]
            tot["best"] += res[best]
            print(f"M {M:5d} N {N:6d} K {K:6d}  " + "  ".join(f"{k} {v:7.1f}us {fl / v / 1e6:6.0f}TF" for k, v in res.items())
                  + f"  -> {best}", flush=True)
        print(f"M {M:5d} per-layer: lib {tot['lib']:.1f}us best {tot['best']:.1f}us ({tot['lib'] / tot['best']:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
