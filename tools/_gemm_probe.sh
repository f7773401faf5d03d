R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=$R/gpurun_out/probe; mkdir -p $O; rm -rf /tmp/pp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/pp -o run -- python3 $R/tools/gemm_probe.py --m 128 > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
cd $R && t=$(find /tmp/pp -name "*kernel_trace.csv" | head -1) && python3 tools/trace_by_grid.py $t --match "gemm|reduce|Cijk" --top 60 > $O/by_grid.txt && cat $O/probe.txt | grep "^M" && cat $O/by_grid.txt
