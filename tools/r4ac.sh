#!/bin/bash
# round 4: collectives with world-templated peer loads -- push + TP/EP GPU tests, then the loopback push A/B
set -o pipefail
O=gpurun_out/push2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_tp_push_gpu.py > $O/tests_push.log 2>&1 || { tail -40 $O/tests_push.log; exit 1; }
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_tp_gpu.py tests/test_ep_gpu.py tests/test_model_gpu.py > $O/tests_tp.log 2>&1 || { tail -40 $O/tests_tp.log; exit 1; }
tail -n 3 $O/tests_push.log
tail -n 3 $O/tests_tp.log
timeout -k 10 300 python3 -u tools/push_ab.py --ms 32,64,128,256 > $O/push_ab.log 2>&1 || { tail -20 $O/push_ab.log; exit 1; }
grep -v amdgpu.ids $O/push_ab.log
