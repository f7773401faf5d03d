#!/bin/bash
# round 4: decode split-KV reduce with one round of register loads -- decode tests, then an interleaved
# A/B over the steady-state decode replay (REDUCE_PRE=1 vs 0) under rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4al; mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
for pre in 1 0; do
  K8SRCA_DECODE_REDUCE_PRE=$pre timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/red$pre -o run -- \
    python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl --variants plan_makespan \
    --pf-ab 0 --samples 60 > $O/replay_pre$pre.txt 2>&1 || { tail -10 $O/replay_pre$pre.txt; exit 1; }
  f=$(find /tmp/red$pre -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_pre$pre.csv
  python3 - $O/kernel_stats_pre$pre.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "attn_reduce" in r["Name"] or "attn_decode" in r["Name"]:
        print(sys.argv[1].split("/")[-1], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
