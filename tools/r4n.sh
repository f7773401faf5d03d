# prefill attention epilogue A/B (4: per-lane fp32 partials / dwordx2 rows; 5: LDS-staged bf16 rows), then the
# HIP-runtime thread probe
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 4,5,2 --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -4
timeout -k 10 300 python3 -u tools/hip_thread_probe.py > $O/probe.txt 2>&1 || { tail -10 $O/probe.txt; exit 1; }
cat $O/probe.txt
