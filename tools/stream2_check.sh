#!/bin/bash
# Decoupled-ring stream kernels (cfg 32 / 33): their GPU tests, then the decode-size dispatch sweep
# (tools/gemm_mid_sweep.py) into a candidate table.  usage (GPU box): tools/stream2_check.sh TAG [ms]
R=${GRAFT_REPO_ROOT:-.}; tag=$1; ms=${2:-48,64,96,128,160,192,224,256}; O=$R/gpurun_out/$tag; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -k "gemm_stream" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u tools/gemm_mid_sweep.py --ms $ms --emit --out $O/dispatch.json > $O/sweep.txt 2>&1
rc=$?; grep -E "^M " $O/sweep.txt | cut -c1-220 | tail -40; exit $rc
