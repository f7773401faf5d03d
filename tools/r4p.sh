# HIP-runtime thread probe (library GEMM / norm / big graphs), then the prefill split planner arms on the replay
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 240 python3 -u tools/hip_thread_probe.py > $O/probe.txt 2>&1 || { tail -10 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 700 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 5,5@o2,5@o4,5@o8 --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -5
nt() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], json.dumps(d['native_threads']['top_cpu_s']), d['host_cpu_s'].get('engine'))"; }
for arm in "X=0" "ROC_SYSTEM_SCOPE_SIGNAL=0" "ROC_CPU_WAIT_FOR_SIGNAL=0"; do
  env $arm timeout -k 10 400 python3 -u bench.py --steps 6 --warmup 2 --no-hints-steps 0 > $O/nt_$arm.json 2> $O/nt_$arm.err || { tail -5 $O/nt_$arm.err; exit 1; }
  nt $O/nt_$arm.json
done
