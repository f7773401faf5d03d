#!/bin/bash
# Kernel + HIP API trace of a short headline-config run; host calls during GPU idle gaps.
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=$R/gpurun_out/gapapi; mkdir -p $O
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O -o run -- \
  python3 $R/bench.py --steps 1 --warmup 0 --incidents 64 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
k=$(find $O -name "*kernel_trace.csv" | head -1); h=$(find $O -name "*hip_api_trace.csv" | head -1)
head -2 $h > $O/api_head.txt
python3 $R/tools/gap_api.py $k $h --min-us 150 > $O/gap_api.txt 2>&1; cat $O/gap_api.txt
rm -f $k $h
