#!/bin/bash
# hipBLASLt solution tuning at prefill M: GPU test, then headline bench A/B
# (tuned vs heuristic-only), interleaved.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tune_ab; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "blaslt or linear" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -c "
import torch
from k8s_llm_rca_amd.models.config import get_config
from k8s_llm_rca_amd.ops import linear as L
rep = L.tune_lib_gemms(torch.device('cuda'), L.projection_shapes(get_config('llama3-8b')))
for M, N, K, h, t, r in rep:
    print(f'M {M:5d} N {N:6d} K {K:6d}  heuristic {h:8.1f}us  tuned {t:8.1f}us  ({h / t:.2f}x, rank {r})')
print('total heuristic %.1f us tuned %.1f us' % (sum(x[3] for x in rep), sum(x[4] for x in rep)))
" > $O/tune_8b.txt 2>&1 || { tail -20 $O/tune_8b.txt; exit 1; }
tail -1 $O/tune_8b.txt
for t in 1 0 1 0; do
  K8SRCA_BLASLT_TUNE=$t timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 > $O/b_$t.log 2>&1 || { tail -20 $O/b_$t.log; exit 1; }
  echo "tune=$t $(grep '^{' $O/b_$t.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_s"], d["setup_s"], d.get("blaslt_tune"))')"
done
