"""Mid-M projections (8B shapes): library GEMM vs K-split batched library
GEMM (fp32-accumulated partials summed afterwards) -- is the chip under-filled
at M = 256..1024?  Cold weights (rotated, > MALL)."""
import sys

import torch


def bench(fn, iters=30):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = "cuda"
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    for M in (256, 384, 512, 640, 768, 1024, 1536):
        line = f"M {M:5d}"
        tot = {}
        for N, K in shapes:
            nw = max(2, int(2e9 // (N * K * 2)))
            ws = [torch.randn(N, K, device=dev).bfloat16() for _ in range(nw)]
            x = torch.randn(M, K, device=dev).bfloat16()
            res = {"lib": bench(lambda i: torch.matmul(x, ws[i % nw].t()))}
            for S in (2, 4):
                Ks = K // S
                xs = x.view(M, S, Ks).transpose(0, 1)
                wss = [w.view(N, S, Ks).permute(1, 2, 0) for w in ws]
                res[f"sk{S}"] = bench(lambda i: torch.bmm(xs, wss[i % nw]))
            best = min(res, key=res.get)
            for k, v in res.items():
                tot[k] = tot.get(k, 0.0) + v
            fl = 2 * M * N * K
            line += f" | N{N} K{K} " + " ".join(f"{k} {v:6.1f}" for k, v in res.items()) + \
                f" -> {best} {fl / res[best] / 1e6:5.0f}TF"
        print(line + " | layer " + " ".join(f"{k} {v:6.1f}" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    sys.exit(main())
