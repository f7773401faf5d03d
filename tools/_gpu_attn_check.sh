R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "prefill or spike" > gpurun_out/t_attn.log 2>&1 || { tail -20 gpurun_out/t_attn.log; exit 1; }
tail -2 gpurun_out/t_attn.log
timeout -k 10 300 python tools/bench_kernels.py --what attn > gpurun_out/bk_attn.log 2>&1 && tail -6 gpurun_out/bk_attn.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ktm -o run -- python3 $R/tools/prof_attn.py --S 1 --q 600 --ctx 3500 > /dev/null 2>&1; cut -d, -f1-4 $R/gpurun_out/ktm/run_kernel_stats.csv; rm -f $R/gpurun_out/ktm/run_kernel_trace.csv
