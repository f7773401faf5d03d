export TMPDIR=/tmp; mkdir -p gpurun_out/lx
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lx/gpu_tests.log 2>&1 || { tail -30 gpurun_out/lx/gpu_tests.log; exit 1; }
tail -1 gpurun_out/lx/gpu_tests.log
for m in "exec:" "noexec:"; do
  n=${m%%:*}
  if [ $n = noexec ]; then export K8SRCA_LAYER_EXEC=0; fi
  timeout -k 10 400 python bench.py > gpurun_out/lx/$n.log 2>&1 || { tail -5 gpurun_out/lx/$n.log; exit 1; }
  echo "== $n"; grep '^{"metric"' gpurun_out/lx/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], t['avg_decode_batch'], e['forward_s'], e['wait_s'])"
done
