# per-step prefill-attention replay (w8 explicit schedule vs pg64), the c = 96 latency-curve point
# (with the busy native thread's syscall sample), and the Mixtral EP=8 per-rank projection
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4l; mkdir -p $O
show() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d.get('p50_latency_s'), json.dumps(d.get('native_threads')), json.dumps({k: v for k, v in (d.get('tp_sim') or {}).items() if k != 'per_T'}), d.get('work_per_analysis'), d['engine'].get('graph_steps'))"; }
timeout -k 10 500 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 4,0 --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -4
bash tools/latency_curve.sh 96 || exit 1
show gpurun_out/curve/c96.json
timeout -k 10 600 python3 -u bench.py --preset mixtral-10k --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim_mixtral.json 2> $O/tpsim_mixtral.err || { tail -5 $O/tpsim_mixtral.err; exit 1; }
show $O/tpsim_mixtral.json
