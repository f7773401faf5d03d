#!/bin/bash
# round 4: 16-B-per-lane bf16 prefill merge -- prefill kernel tests, replay A/B (VAR 6 with the new vs old merge)
# and the kernel split of the new arm under rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4af; mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 500 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 6,6m --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | grep replay
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 6 --samples 60 > $O/replay_prof.txt 2>&1 || { tail -10 $O/replay_prof.txt; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4af/kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:4]:
    print(round(float(r["TotalDurationNs"]) / 1e6, 2), "ms", r["Calls"], round(float(r["TotalDurationNs"]) / tot * 100, 1), "%", r["Name"][:80])
PY
