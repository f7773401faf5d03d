export TMPDIR=/tmp; mkdir -p gpurun_out/moe
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "grouped or mixtral or moe" > gpurun_out/moe/t.log 2>&1 || { tail -30 gpurun_out/moe/t.log; exit 1; }
tail -1 gpurun_out/moe/t.log
timeout -k 10 200 python tools/bench_kernels.py --what moe_split > gpurun_out/moe/split.txt 2>&1 || exit 1
grep moe_split gpurun_out/moe/split.txt
timeout -k 10 500 python bench.py --preset mixtral-10k > gpurun_out/moe/bench.log 2>&1 || { tail -5 gpurun_out/moe/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/moe/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], t['avg_decode_batch'], e['evictions'], t['kv_peak_util'])"
