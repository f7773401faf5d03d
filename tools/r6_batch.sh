#!/bin/bash
# Round-6 GPU batch (one gpurun call; the pool is congested): co-execution probe,
# nano-batch bit-identity test, interleaved contract A/B nano_batch on/off, step trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/r6; mkdir -p $O
cd $R
timeout -k 10 240 python3 -u tools/coexec_cumask.py --out $O/coexec2.json > $O/coexec2.log 2>&1 || exit 11
timeout -k 10 200 python3 -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread \
  -k "nano or norm_fuse or executor_bit" > $O/nano_tests.log 2>&1 || exit 12
for i in 1 2; do
  K8SRCA_NANO_BATCH=1 timeout -k 10 330 python3 -u bench.py --steps 20 --warmup 5 --no-hints-steps 0 > $O/nano_on_$i.log 2>&1 || exit 13
  timeout -k 10 330 python3 -u bench.py --steps 20 --warmup 5 --no-hints-steps 0 > $O/nano_off_$i.log 2>&1 || exit 14
done
exit 0
