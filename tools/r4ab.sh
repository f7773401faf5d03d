#!/bin/bash
# round 4: TP push epilogue -- GPU tests (push bit-identity: 2 processes, loopback, engine;
# the TP / EP shared-GPU suite; the executor tests), then the loopback push A/B
set -o pipefail
O=gpurun_out/push
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_tp_push_gpu.py > $O/tests_push.log 2>&1 || { tail -40 $O/tests_push.log; exit 1; }
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_tp_gpu.py tests/test_ep_gpu.py tests/test_model_gpu.py > $O/tests_tp.log 2>&1 || { tail -40 $O/tests_tp.log; exit 1; }
tail -3 $O/tests_push.log $O/tests_tp.log
timeout -k 10 300 python3 -u tools/push_ab.py > $O/push_ab.log 2>&1 || { tail -20 $O/push_ab.log; exit 1; }
cat $O/push_ab.log
