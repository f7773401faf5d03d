#!/bin/bash
# Round-2 closing measurements: smoke, the driver's headline contract twice, latency at concurrency 1 and 8.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 400 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { tail -5 $O/bench$i.log; exit 1; }
  grep '^{' $O/bench$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench$i', d['value'], d['p50_latency_s'], d['p90_latency_s'], d['wall_s'], d['no_hints'])"
done
bash $R/tools/latency_sweep.sh
