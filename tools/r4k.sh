# prefill attention: the explicit-schedule w8 variant (tests, then replay A/B vs the compiler schedule),
# then the headline (driver contract, native-thread report) and the 70B TP=8 per-rank projection
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4k; mkdir -p $O
show() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d.get('p50_latency_s'), json.dumps(d.get('native_threads')), json.dumps({k: v for k, v in (d.get('tp_sim') or {}).items() if k != 'per_T'}), d.get('work_per_analysis'))"; }
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 2,4 --samples 60 > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -6
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/head.json 2> $O/head.err || { tail -5 $O/head.err; exit 1; }
show $O/head.json
timeout -k 10 600 python3 -u bench.py --model llama3-70b --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim70b.json 2> $O/tpsim70b.err || { tail -5 $O/tpsim70b.err; exit 1; }
show $O/tpsim70b.json
