#!/bin/bash
# Kernel trace of a short headline-config run (128 concurrent, 4 steps): small kernels split by grid size.
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=$R/gpurun_out/small2; mkdir -p $O; T=/tmp/small2; rm -rf $T
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $T -o run -- \
  python3 $R/bench.py --steps 4 --warmup 2 --no-hints-steps 0 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
t=$(find $T -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py $t --match "rmsnorm|rope|silu|reduce" --top 40 > $O/small.txt && cat $O/small.txt
python3 $R/tools/trace_by_grid.py $t --match "Cijk|gemm|grouped" --top 60 > $O/gemms.txt
rm -rf $T
