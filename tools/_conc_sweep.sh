export TMPDIR=/tmp; mkdir -p gpurun_out/conc
for n in "$@"; do
  timeout -k 10 500 python bench.py --incidents $n > gpurun_out/conc/c$n.log 2>&1 || { echo "c$n failed"; tail -5 gpurun_out/conc/c$n.log; exit 1; }
  echo "== $n"; grep '^{"metric"' gpurun_out/conc/c$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], d['p90_latency_s'], e['evictions'], t['avg_decode_batch'], t['kv_peak_util'])"
done
