#!/bin/bash
# Interleaved A/B of tiny prefill chunks as decode-attention rows on the headline.
# Config "T:G" = K8S_TINY_CHUNK_TOKENS=T, K8S_DECODE_GROUP=G (multi-token decode items).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_tiny; mkdir -p $O
CFGS=${CFGS:-"0:1 8:1 8:0 32:1"}
for i in 1 2; do
  for c in $CFGS; do
    t=${c%:*}; g=${c#*:}
    K8S_TINY_CHUNK_TOKENS=$t K8S_DECODE_GROUP=$g timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 \
      --no-hints-steps 0 > $O/t$t.g$g.$i.log 2>&1 || { tail -5 $O/t$t.g$g.$i.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/t$t.g$g.$i.log') if l.startswith('{')][-1]); e=d['engine']; print('tiny=$t group=$g run$i', d['value'], d['p50_latency_s'], e.get('steps'), e.get('graph_steps'))"
  done
done
