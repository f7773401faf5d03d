#!/bin/bash
# Round-6 GPU batch 2: token-flag test + interleaved contract A/B token_flag on / off.
R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/r6; mkdir -p $O
cd $R
timeout -k 10 200 python3 -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "token_flag or nano" > $O/flag_tests.log 2>&1 || exit 12
for i in 1 2; do
  K8SRCA_TOKEN_FLAG=1 timeout -k 10 330 python3 -u bench.py --steps 20 --warmup 5 --no-hints-steps 0 > $O/flag_on_$i.log 2>&1 || exit 13
  timeout -k 10 330 python3 -u bench.py --steps 20 --warmup 5 --no-hints-steps 0 > $O/flag_off_$i.log 2>&1 || exit 14
done
exit 0
