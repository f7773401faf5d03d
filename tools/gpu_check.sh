#!/bin/bash
# Round-end rehearsal on one GPU box: the GPU test suite, smoke(), and the driver's bench contract.
# usage (GPU box): tools/gpu_check.sh [TAG]   -> gpurun_out/check_TAG/{tests.log,smoke.log,bench.json}
R=${GRAFT_REPO_ROOT:-.}; tag=${1:-check}; O=$R/gpurun_out/check_$tag; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
grep "smoke ok" $O/smoke.log | cut -c1-200
if [ "${NO_BENCH:-0}" != "1" ]; then
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['p50_latency_s'], d['p90_latency_s'], d['wall_s'], d['thread_regime']['incidents_at_t0'])"
fi
