#!/bin/bash
# Interleaved A/B (grouped kernel vs LDS-DMA gate_up) on the Mixtral preset.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_moe; mkdir -p $O
for i in 1 2; do
  for t in 0 384; do
    K8S_MOE_GLDS_MAX_ROWS=$t timeout -k 10 300 python3 $R/bench.py --preset mixtral-10k --steps 8 --warmup 2 \
      --no-hints-steps 0 > $O/g$t.$i.log 2>&1 || { tail -5 $O/g$t.$i.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/g$t.$i.log') if l.startswith('{')][-1]); print('glds_max_rows=$t run$i', d['value'], d['p50_latency_s'])"
  done
done
