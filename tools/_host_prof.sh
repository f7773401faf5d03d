#!/bin/bash
# Headline with the engine thread under cProfile + step timing + per-thread CPU.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/hostprof; mkdir -p $O
K8S_RCA_STEP_TIMING=1 K8S_RCA_PROFILE_ENGINE=$O/eng.prof timeout -k 10 300 python3 $R/bench.py --steps 8 --warmup 2 \
  --no-hints-steps 0 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print(d['value'], d['host_cpu_s'], d['engine'])"
python3 -c "
import pstats; p=pstats.Stats('$O/eng.prof'); p.sort_stats('tottime').print_stats(30); p.sort_stats('cumulative').print_stats(40)" > $O/eng_prof.txt
head -60 $O/eng_prof.txt
