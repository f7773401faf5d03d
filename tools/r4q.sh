# prefill split planner arms (makespan choice everywhere / only where the fixed rule splits), longer thread probe
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 800 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 5,5@o8,5@o12,5@o16,5@h8,5@h16 --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -7
timeout -k 10 400 python3 -u tools/hip_thread_probe.py --n 200000 > $O/probe.txt 2>&1 || { tail -10 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
