#!/bin/bash
# round 4: kernel split of the replayed prefill attention (VAR 6 + makespan planner): main kernel vs split-KV merge
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4ae; mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 6 --samples 60 > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -3
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4ae/kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(round(float(r["TotalDurationNs"]) / 1e6, 2), "ms", r["Calls"], round(float(r["TotalDurationNs"]) / tot * 100, 1), "%", r["Name"][:90])
PY
