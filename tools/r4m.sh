# w8 VAR 4 with the LDS-staged bf16 epilogue: prefill tests, replay vs the compiler-scheduled arm;
# then which env setting quiets the busy HIP-runtime thread (short bench runs, native-thread report)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4m; mkdir -p $O
nt() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], 'p50', d.get('p50_latency_s'), json.dumps(d.get('native_threads')), d['host_cpu_s'])"; }
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 4,2 --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -4
timeout -k 10 400 python3 -u bench.py --steps 6 --warmup 2 --no-hints-steps 0 > $O/nt_base.json 2> $O/nt_base.err || { tail -5 $O/nt_base.err; exit 1; }
nt $O/nt_base.json
ROC_ACTIVE_WAIT_TIMEOUT=0 timeout -k 10 400 python3 -u bench.py --steps 6 --warmup 2 --no-hints-steps 0 > $O/nt_awt0.json 2> $O/nt_awt0.err || { tail -5 $O/nt_awt0.err; exit 1; }
nt $O/nt_awt0.json
