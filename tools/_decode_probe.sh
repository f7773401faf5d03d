# decode attention probe under a kernel trace (per-kernel split of decode vs reduce)
export TMPDIR=/tmp; O=$GRAFT_REPO_ROOT/gpurun_out/decode_probe; mkdir -p $O; T=/tmp/dprobe; rm -rf $T
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- python3 $GRAFT_REPO_ROOT/tools/decode_probe.py > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
cat $O/probe.txt | grep -v amdgpu.ids
f=$(find $T -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 $GRAFT_REPO_ROOT/tools/trace_by_grid.py $(find $T -name "*kernel_trace.csv" | head -1) --match attn > $O/by_grid.txt 2>&1; cat $O/by_grid.txt
