#!/bin/bash
# Interleaved A/B of two GEMM dispatch tables on the headline bench (old/new/old/new).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O
A=${1:-profiles/r2_dispatch_pre_glds.json}; B=${2:-k8s_llm_rca_amd/data/gemm_dispatch_llama3-8b.json}
for i in 1 2; do
  for t in A B; do
    f=$A; [ $t = B ] && f=$B
    K8SRCA_GEMM_DISPATCH_FILE=$R/$f timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-hints-steps 0 \
      > $O/$t$i.log 2>&1 || { tail -5 $O/$t$i.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$t$i.log') if l.startswith('{')][-1]); print('$t$i', d['value'], d['p50_latency_s'])"
  done
done
