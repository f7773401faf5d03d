export TMPDIR=/tmp; mkdir -p gpurun_out/final
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || { tail -30 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench.log 2>&1 || { tail -5 gpurun_out/final/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/final/bench.log
bash tools/_prof_bench.sh final > gpurun_out/final/prof.txt 2>&1 || { tail -5 gpurun_out/final/prof.txt; exit 1; }
head -12 gpurun_out/prof_final/summary.txt
