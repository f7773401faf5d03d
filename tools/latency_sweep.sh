#!/bin/bash
# p50/p90 end-to-end latency of one analysis at low concurrency (headline config:
# Llama-3-8B, 10k-node graph, 1 GPU).  usage: tools/latency_sweep.sh (via gpurun)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/latency; mkdir -p $O
for c in 1 8; do
  q=$(( c < 4 ? 1 : 4 ))
  timeout -k 10 300 python3 $R/bench.py --incidents $c --quantum $q --steps 10 --warmup 2 --no-hints-steps 0 \
    > $O/c$c.json 2> $O/c$c.err || { tail -5 $O/c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c$c.json').read().strip().splitlines()[-1]); print('concurrency', $c, 'value', d['value'], 'p50', d['p50_latency_s'], 'p90', d['p90_latency_s'], 'ttft_p50', d['throughput']['ttft_p50_s'])"
done
