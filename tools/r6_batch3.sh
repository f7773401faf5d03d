#!/bin/bash
# The GPU suite on the current tree (KV manager refactor, host tier), then decode-GEMM
# re-sweeps of the 70B TP=8 shard and Mixtral tables with the current candidates.
set -o pipefail
O=gpurun_out/r6/batch3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > $O/gpu_tests.log 2>&1 \
  || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for spec in "llama3-70b 8" "mixtral-8x7b 1"; do
  set -- $spec
  timeout -k 10 400 python -u tools/gemm_mid_sweep.py --model $1 --tp $2 --ms 16,24,32,48,64,96,128,160,192,224,256 \
    --emit --out $O/dispatch_$1_tp$2.json > $O/sweep_$1_tp$2.log 2>&1 || { tail -5 $O/sweep_$1_tp$2.log; exit 1; }
  grep "per-layer" $O/sweep_$1_tp$2.log | tail -4
done
