# the busy HIP-runtime thread in the real bench: graph packet capture on (default) / off; then the GPU tests
# that plan prefill (makespan planner default)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4s; mkdir -p $O
nt() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d['p50_latency_s'], json.dumps(d['native_threads']['top_cpu_s']), d['host_cpu_s'], d['engine'].get('graph_steps'), d['work_per_analysis'])"; }
for arm in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  env $arm timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 3 --no-hints-steps 0 > $O/nt_$arm.json 2> $O/nt_$arm.err || { tail -5 $O/nt_$arm.err; exit 1; }
  nt $O/nt_$arm.json
done
timeout -k 10 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill or chunk or executor or extend" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
