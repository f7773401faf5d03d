# HIP-runtime thread probe (engine-like operations), prefill tests on the new default, headline contract run
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 300 python3 -u tools/hip_thread_probe.py > $O/probe.txt 2>&1 || { tail -10 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/head.json 2> $O/head.err || { tail -5 $O/head.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/head.json').read().strip().splitlines()[-1]); print(d['value'], d['p50_latency_s'], d['native_threads'], d['host_cpu_s'], d['work_per_analysis'])"
