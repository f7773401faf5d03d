#!/bin/bash
# Concurrency-1 latency A/B (the headline config, thread regime): default dispatch vs a variant table.
# usage (GPU box): tools/c1_ab.sh TAG VARIANT_TABLE.json -> gpurun_out/TAG/{base,var}.json
R=${GRAFT_REPO_ROOT:-.}; tag=$1; var=$2; O=$R/gpurun_out/$tag; mkdir -p $O
run() {  # name, extra env
  env $2 timeout -k 10 400 python3 $R/bench.py --incidents 1 --quantum 1 --steps 10 --warmup 2 --no-hints-steps 0 \
    > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -3 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d['p50_latency_s'], 'p90', d['p90_latency_s'])"
}
run base "K8SRCA_STREAM_SILU=0" && run silu "K8SRCA_STREAM_SILU=1" && run var "K8SRCA_GEMM_DISPATCH_FILE=$var"
