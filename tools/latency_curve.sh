#!/bin/bash
# Latency-throughput curve of the headline config under the driver's thread regime
# (pre-aged threads, per-pipeline warm-up): one bench run per concurrency.
# usage (GPU box): tools/latency_curve.sh [concurrencies...]   -> gpurun_out/curve/c<N>.json
R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/curve; mkdir -p $O
for c in ${@:-1 8 32 64 128}; do
  q=$(( c >= 16 ? c / 8 : 1 )); s=$(( c >= 16 ? 20 : 10 ))
  timeout -k 10 600 python3 $R/bench.py --incidents $c --quantum $q --steps $s --warmup 2 --no-hints-steps 0 \
    > $O/c$c.json 2> $O/c$c.err || { echo "c=$c failed"; tail -3 $O/c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c$c.json').read().strip().splitlines()[-1]); \
print('c=$c', d['value'], 'p50', d['p50_latency_s'], 'p90', d['p90_latency_s'], 'age', d['thread_regime']['incidents_at_t0'])"
done
