#!/bin/bash
# Interleaved A/B of tiny prefill chunks as decode-attention rows on the headline.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_tiny; mkdir -p $O
for i in 1 2; do
  for t in 0 8 32; do
    K8S_TINY_CHUNK_TOKENS=$t timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 \
      --no-hints-steps 0 > $O/t$t.$i.log 2>&1 || { tail -5 $O/t$t.$i.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/t$t.$i.log') if l.startswith('{')][-1]); e=d['engine']; print('tiny=$t run$i', d['value'], d['p50_latency_s'], e.get('steps'), e.get('graph_steps'))"
  done
done
