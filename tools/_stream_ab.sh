export TMPDIR=/tmp; mkdir -p gpurun_out/stream
for m in "stream:" "sync:--sync-steps" "stream4:--steps 4"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 500 python bench.py $a > gpurun_out/stream/$n.log 2>&1 || { tail -5 gpurun_out/stream/$n.log; exit 1; }
  echo "== $n"; grep '^{"metric"' gpurun_out/stream/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['ms_per_step'], d['p50_latency_s'], d['p90_latency_s'], t['avg_decode_batch'], t['kv_peak_util'], e['evictions'])"
done
