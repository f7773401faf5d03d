export TMPDIR=/tmp; mkdir -p gpurun_out/blaslt
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "blaslt" > gpurun_out/blaslt/t.log 2>&1 || { tail -30 gpurun_out/blaslt/t.log; exit 1; }
tail -1 gpurun_out/blaslt/t.log
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/blaslt/gpu_tests.log 2>&1 || { tail -20 gpurun_out/blaslt/gpu_tests.log; exit 1; }
tail -1 gpurun_out/blaslt/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/blaslt/bench.log 2>&1 || { tail -5 gpurun_out/blaslt/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/blaslt/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], t['avg_decode_batch'], e['wait_s'], e['host_s'], e['forward_s'])"
