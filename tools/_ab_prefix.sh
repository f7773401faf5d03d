export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/gpu_tests.log 2>&1 || { tail -20 gpurun_out/ab/gpu_tests.log; exit 1; }
tail -1 gpurun_out/ab/gpu_tests.log
for cfg in "10k:" "1k:--preset llama3-8b-1k" "10k-noshare:--no-prefix-sharing"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 400 python bench.py $a > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab/$n.log; exit 1; }
  echo "== $n"; grep '^{"metric"' gpurun_out/ab/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; print(d['value'], d['p50_latency_s'], e['prefill_tokens'], e['prefix_hit_tokens'], e['decode_ctx_tokens'], e['evictions'], d['throughput'])"
done
