#!/bin/bash
# Kernel trace of the headline bench (1 warmup + 1 timed step): idle gaps by preceding step kind.
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=$R/gpurun_out/gapsteps; mkdir -p $O
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
k=$(find $O -name "*kernel_trace.csv" | head -1)
python3 $R/tools/gap_steps.py $k --from-frac 0.55 > $O/gap_steps.txt 2>&1; cat $O/gap_steps.txt
rm -f $k
