# headline (driver contract) with the native-thread report, then the two 8-GPU per-rank projections
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4j; mkdir -p $O
show() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d.get('p50_latency_s'), json.dumps(d.get('native_threads')), json.dumps({k: v for k, v in (d.get('tp_sim') or {}).items() if k != 'per_T'}), d.get('work_per_analysis'))"; }
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/head.json 2> $O/head.err || { tail -5 $O/head.err; exit 1; }
show $O/head.json
timeout -k 10 600 python3 -u bench.py --model llama3-70b --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim70b.json 2> $O/tpsim70b.err || { tail -5 $O/tpsim70b.err; exit 1; }
show $O/tpsim70b.json
timeout -k 10 600 python3 -u bench.py --preset mixtral-10k --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim_mixtral.json 2> $O/tpsim_mixtral.err || { tail -5 $O/tpsim_mixtral.err; exit 1; }
show $O/tpsim_mixtral.json
