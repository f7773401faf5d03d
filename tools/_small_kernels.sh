#!/bin/bash
# Kernel trace of a shorter headline-config run; small kernels split by grid size.
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=$R/gpurun_out/small; mkdir -p $O
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
  python3 $R/bench.py --steps 1 --warmup 0 --incidents 64 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
t=$(find $O -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py $t > $O/small.txt && cat $O/small.txt
python3 $R/tools/trace_by_grid.py $t --match "Cijk|gemm|grouped" --top 60 > $O/gemms.txt
python3 $R/tools/trace_by_grid.py $t --match "attn" --top 30 > $O/attn.txt
rm -f $t
