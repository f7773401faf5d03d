# the busy HIP-runtime thread in the real bench: ROCclr's command batch size default vs 4096 (the probe's
# DEBUG_CLR_MAX_BATCH_SIZE=4096 arm kept the helper thread from polling after a launch flood), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4u; mkdir -p $O
nt() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d['p50_latency_s'], json.dumps(d['native_threads']['top_cpu_s']), d['host_cpu_s'], d['engine'].get('graph_steps'), d['work_per_analysis'])"; }
i=0
for arm in "X=0" "DEBUG_CLR_MAX_BATCH_SIZE=4096" "X=0" "DEBUG_CLR_MAX_BATCH_SIZE=4096"; do
  i=$((i+1))
  env $arm timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 3 --no-hints-steps 0 > $O/nt_$i.json 2> $O/nt_$i.err || { tail -5 $O/nt_$i.err; exit 1; }
  echo "$arm"; nt $O/nt_$i.json
done
