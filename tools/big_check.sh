#!/bin/bash
# gemm_big on one GPU box: its GPU tests, then the A/B against hipBLASLt (tools/big_gemm_ab.py).
# usage (GPU box): tools/big_check.sh TAG [ab args...]  -> gpurun_out/TAG/{tests.log,ab.log,ab.jsonl}
R=${GRAFT_REPO_ROOT:-.}; tag=$1; shift; O=$R/gpurun_out/$tag; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 200 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm_big or stream_silu or executor or graph_vs_eager" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc   # a fault / abort / timeout: nothing more on the GPU
timeout -k 10 400 python3 -u tools/big_gemm_ab.py --out $O/ab.jsonl "$@" > $O/ab.log 2>&1
rc2=$?; tail -45 $O/ab.log; exit $(( rc > rc2 ? rc : rc2 ))
