"""Diagnose: is the decode attention output deterministic call to call, and does the reduce's
register-prefetch form (K8SRCA_DECODE_REDUCE_PRE=1) change bits?  (test_paged_decode shapes)"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402
from k8s_llm_rca_amd.knobs import KNOBS, set_knob  # noqa: E402

import test_kernels_gpu as T  # noqa: E402
from k8s_llm_rca_amd.ops import attention as A  # noqa: E402

for ctx, BS, (nq, nkv) in (([1000, 3, 2500, 128], 64, (32, 8)), ([5000], 64, (32, 8)), ([1000, 3, 2500, 128], 32, (32, 8))):
    torch.manual_seed(1)
    NB = sum((c + BS - 1) // BS for c in ctx) + 4
    kc, vc = T._setup_cache(nkv, BS, NB, T.dev)
    meta = T._meta(ctx, [1] * len(ctx), nq, nkv, BS, NB, T.dev, decode=True)
    q = torch.randn(len(ctx), (nq + 2 * nkv) * 128, device=T.dev).bfloat16()
    outs = []
    for pre in ("0", "0", "1", "1", "0"):
        set_knob("decode_reduce_pre", pre)
        outs.append(A.paged_attention(q, kc, vc, meta, nq, nkv, 1 / math.sqrt(128)).clone())
    torch.cuda.synchronize()
    eq = [[bool(torch.equal(a, b)) for b in outs] for a in outs]
    print(ctx, BS, "n_parts", getattr(meta, "n_parts", None), "part_size", getattr(meta, "part_size", None))
    print("  equal matrix (runs 0,0,1,1,0):", eq[0], eq[2])
    print("  max |0 - 1|:", float((outs[0].float() - outs[2].float()).abs().max()),
          "rows differing:", (outs[0] != outs[2]).any(-1).nonzero().flatten().tolist())
