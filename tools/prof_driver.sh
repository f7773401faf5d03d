#!/bin/bash
# Kernel-trace profile of the driver's bench contract (default --steps 20 --warmup 5).
# usage: tools/prof_driver.sh TAG [bench args...]   (run on the GPU box via gpurun)
# window_summary.txt = the timed window alone (tools/window_summary.py).
# Leaves only small summaries under gpurun_out/prof_TAG (gpurun copies back <= 64 MiB).
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; tag=$1; shift
O=$R/gpurun_out/prof_$tag; mkdir -p $O; T=/tmp/prof_$tag; rm -rf $T; mkdir -p $T
cd /tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-hints-steps 0 "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-600
f=$(find $T -name "*kernel_stats.csv" | head -1); t=$(find $T -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kernel_summary.py $f > $O/summary.txt && cat $O/summary.txt
python3 $R/tools/trace_gaps.py $t 0.55 > $O/gaps.json && head -c 1500 $O/gaps.json
# the timed window only (between bench.py's window_mark kernels), priced against each family's ceiling
python3 $R/tools/window_summary.py $t $O/bench.log > $O/window_summary.txt && cat $O/window_summary.txt
cp $f $O/kernel_stats.csv
rm -rf $T
