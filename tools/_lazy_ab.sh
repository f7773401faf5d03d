export TMPDIR=/tmp; mkdir -p gpurun_out/lazy
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lazy/gpu_tests.log 2>&1 || { tail -20 gpurun_out/lazy/gpu_tests.log; exit 1; }
tail -1 gpurun_out/lazy/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/lazy/bench.log 2>&1 || { tail -5 gpurun_out/lazy/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/lazy/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], t['avg_decode_batch'], e['wait_s'], e['host_s'], e['forward_s'])"
bash tools/_prof_bench.sh lazy > gpurun_out/lazy/prof.txt 2>&1 || { tail -5 gpurun_out/lazy/prof.txt; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/prof_lazy/gaps.json')); print({k:v for k,v in d.items() if k not in ('top_pairs','window_us')}); [print(p) for p in d['top_pairs'][:8]]"
