R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/r5a; mkdir -p $O; cd $R
for c in 128 96 104; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --incidents $c > $O/c$c.json 2> $O/c$c.err || { tail -5 $O/c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c$c.json').read().strip().splitlines()[-1]); print('c=$c', d['value'], d['p50_latency_s'], d['p90_latency_s'], d['wall_s'], d['work_per_analysis'], d['native_threads']['top_cpu_s'])"
done
