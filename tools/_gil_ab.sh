export TMPDIR=/tmp; mkdir -p gpurun_out/gil
for si in 0.0005 0.002; do
  K8S_RCA_SWITCH_INTERVAL=$si timeout -k 10 400 python bench.py > gpurun_out/gil/si$si.log 2>&1 || { tail -5 gpurun_out/gil/si$si.log; exit 1; }
  echo "== $si"; grep '^{"metric"' gpurun_out/gil/si$si.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; print(d['value'], d['p50_latency_s'], e['wait_s'], e['host_s'], e['forward_s'], e['sample_s'])"
done
