# which HIP-runtime setting quiets the native thread that graph replays and hipBLASLt calls keep busy;
# then the prefill planner default under the GPU tests that plan prefill, and the headline
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4r; mkdir -p $O
for arm in "X=0" "DEBUG_CLR_MAX_BATCH_SIZE=1024" "DEBUG_HIP_GRAPH_BATCH_SIZE=1024" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" \
           "DEBUG_CLR_BATCH_CPU_SYNC_SIZE=1024" "DEBUG_HIP_FORCE_GRAPH_QUEUES=0" "DEBUG_HIP_BLOCK_SYNC=0"; do
  echo "== $arm"
  env $arm timeout -k 10 120 python3 -u tools/hip_thread_probe.py --n 100000 --phases graph_replays,big_graph,torch_matmul,eager_kernels > $O/probe_$arm.txt 2>&1 || { tail -5 $O/probe_$arm.txt; exit 1; }
  grep -v amdgpu.ids $O/probe_$arm.txt
done
timeout -k 10 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill or chunk or executor or extend" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/head.json 2> $O/head.err || { tail -5 $O/head.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/head.json').read().strip().splitlines()[-1]); print(d['value'], d['p50_latency_s'], d['native_threads']['top_cpu_s'], d['work_per_analysis'])"
