export TMPDIR=/tmp; mkdir -p gpurun_out/gc
for m in "freeze:" "nofreeze:--no-gc-freeze"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 400 python bench.py $a > gpurun_out/gc/$n.log 2>&1 || { tail -5 gpurun_out/gc/$n.log; exit 1; }
  echo "== $n"; grep '^{"metric"' gpurun_out/gc/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], t['avg_decode_batch'], e['wait_s'])"
done
