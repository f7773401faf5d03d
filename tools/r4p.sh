# HIP-runtime thread probe (library GEMM / norm / big graphs), then the prefill split planner arms on the replay
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 240 python3 -u tools/hip_thread_probe.py > $O/probe.txt 2>&1 || { tail -10 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 700 python3 -u tools/bench_kernels.py --what replay --trace profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 5,5@o2,5@o4,5@o8 --samples 60 --pf-steps-out $O/pf_steps.jsonl > $O/replay.txt 2>&1 || { tail -10 $O/replay.txt; exit 1; }
grep -v "^#" $O/replay.txt | tail -5
