#!/bin/bash
# Round-6 closing check (one gpurun call): GPU test suite, smoke, the driver's contract
# bench twice, and the window profile under rocprofv3 (kernel trace only).
R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/r6/${TAG:-final}; mkdir -p $O
cd $R
timeout -k 10 420 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rs > $O/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
for i in 1 2; do
  timeout -k 10 330 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit 13
done
[ -n "$NOPROF" ] || timeout -k 10 720 tools/prof_driver.sh r6final > $O/prof.log 2>&1 || exit 14
exit 0
