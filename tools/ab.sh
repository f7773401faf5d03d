#!/bin/bash
# Interleaved A/B of environment settings on the driver's bench (one process per run, same box).
# usage (GPU box): tools/ab.sh TAG ROUNDS "ENV_A" "ENV_B" [-- bench args]
#   e.g. tools/ab.sh prio 2 "K8SRCA_PF_W8=1" "K8SRCA_PF_W8=0" -- --steps 20 --warmup 5
# -> gpurun_out/ab_TAG/{a,b}<round>.json; prints value / p50 / work per analysis per run.
R=${GRAFT_REPO_ROOT:-.}; tag=$1; rounds=$2; A=$3; B=$4; shift 4; [ "$1" = "--" ] && shift
O=$R/gpurun_out/ab_$tag; mkdir -p $O
for i in $(seq 1 $rounds); do
  for arm in a b; do
    envs=$A; [ $arm = b ] && envs=$B
    env $envs timeout -k 10 600 python3 $R/bench.py "$@" > $O/$arm$i.json 2> $O/$arm$i.err || { tail -5 $O/$arm$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$arm$i.json').read().strip().splitlines()[-1]); \
print('$arm$i [$envs]', d['value'], 'p50', d['p50_latency_s'], 'work', d['work_per_analysis'])"
  done
done
