#!/bin/bash
# round 4: non-finite-logit guard in the sampler -- sampling / model GPU tests, smoke, a 10-step bench
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4ai; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_sampling.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
grep "smoke ok" $O/smoke.log | cut -c1-120
timeout -k 10 500 python3 bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['p50_latency_s'], d['work_per_analysis'], d['engine']['nonfinite_rows'], d['errors'])"
