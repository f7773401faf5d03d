#!/bin/bash
# Kernel-trace profile of the concurrency-1 decode loop (tools/decode_latency.py, one variant).
# usage (GPU box): tools/prof_decode.sh TAG [decode_latency args...] -> gpurun_out/prof_TAG/{summary.txt,kernel_stats.csv}
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; tag=$1; shift
O=$R/gpurun_out/prof_$tag; mkdir -p $O; T=/tmp/prof_$tag; rm -rf $T; mkdir -p $T
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- \
  python3 $R/tools/decode_latency.py "$@" > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
tail -2 $O/run.log
f=$(find $T -name "*kernel_stats.csv" | head -1)
python3 $R/tools/kernel_summary.py $f --top 25 > $O/summary.txt && cat $O/summary.txt
cp $f $O/kernel_stats.csv
rm -rf $T
