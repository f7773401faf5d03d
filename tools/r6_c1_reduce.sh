#!/bin/bash
# Concurrency 1: the decode split-KV reduce's 32-partition prefetch form (27 partitions at one
# row x 5k keys used to take the LDS form) vs the LDS form (knob decode_reduce_pre=0), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/r6/c1_reduce; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "paged_decode" -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
c1() {
  env $2 timeout -k 10 300 python3 $R/bench.py --incidents 1 --quantum 1 --steps 10 --warmup 2 --no-hints-steps 0 \
    > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); t=d['throughput']; print('$1', d['value'], 'p50', d['p50_latency_s'], 'decode tok/s', t['decode_tok_per_s'])"
}
c1 pre32_a "" && c1 lds_a "K8SRCA_DECODE_REDUCE_PRE=0" && c1 pre32_b "" && c1 lds_b "K8SRCA_DECODE_REDUCE_PRE=0"
