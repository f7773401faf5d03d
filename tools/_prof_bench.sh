#!/bin/bash
# Kernel-trace profile of the headline bench (1 warmup + 1 timed step).
# usage: tools/_prof_bench.sh TAG [bench args...]
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; tag=$1; shift
O=$R/gpurun_out/prof_$tag; mkdir -p $O
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-400
f=$(find $O -name "*kernel_stats.csv" | head -1); t=$(find $O -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kernel_summary.py $f > $O/summary.txt && cat $O/summary.txt
python3 $R/tools/trace_gaps.py $t 0.55 > $O/gaps.json && head -c 1500 $O/gaps.json
cp $f $O/kernel_stats.csv; rm -f $t
