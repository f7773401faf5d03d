#!/bin/bash
# gemm_mid variants with padding-free M tiles (MT = 3/6/10/12/14): correctness on
# every variant, re-sweep the Llama-3-8B dispatch, then A/B the headline bench
# old table vs new table (interleaved).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/mt; mkdir -p $O; cd $R
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-8b.json $O/disp_old.json
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_mid" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 tools/gemm_mid_sweep.py --model llama3-8b --emit > $O/sweep_8b.txt 2>&1 || { tail -5 $O/sweep_8b.txt; exit 1; }
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-8b.json $O/disp_new.json
grep "per-layer sum" $O/sweep_8b.txt
for t in new old new old; do
  K8SRCA_GEMM_DISPATCH_FILE=$O/disp_$t.json timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 > $O/b_$t.log 2>&1 || { tail -5 $O/b_$t.log; exit 1; }
  echo "$t $(grep '^{' $O/b_$t.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_s"])')"
done
