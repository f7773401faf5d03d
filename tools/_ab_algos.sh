#!/bin/bash
# Sweep every hipBLASLt solution (8B shapes), emit the table, then an interleaved
# headline A/B with the table on / off.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_algos; mkdir -p $O
timeout -k 10 300 python3 $R/tools/blaslt_sweep.py --emit > $O/sweep.txt 2>&1 || { tail -5 $O/sweep.txt; exit 1; }
tail -3 $O/sweep.txt
cp $R/k8s_llm_rca_amd/data/blaslt_algos_llama3-8b.json $O/
for i in 1 2; do
  for t in 0 1; do
    K8S_BLASLT_ALGOS=$t timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 --no-hints-steps 0 \
      > $O/a$t.$i.log 2>&1 || { tail -5 $O/a$t.$i.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/a$t.$i.log') if l.startswith('{')][-1]); e=d['engine']; print('algos=$t run$i', d['value'], d['p50_latency_s'], e.get('steps'))"
  done
done
