# PMC passes over the prefill-attention replay (w8 VAR 5, makespan planner): where the main loop's cycles go
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; export PYTHONPATH=$GRAFT_REPO_ROOT
bash tools/pmc.sh pf5 python3 $GRAFT_REPO_ROOT/tools/bench_kernels.py --what replay --trace $GRAFT_REPO_ROOT/profiles/r3/shape_trace_steady.jsonl \
  --variants none --pf-ab 1 --pf-kinds 5 --samples 20 > gpurun_out/pmc_pf5.txt 2>&1; rc=$?
grep -E "attn_prefill|merge" gpurun_out/pmc_pf5.txt | cut -c1-700; exit $rc
