export TMPDIR=/tmp; mkdir -p gpurun_out/tune
timeout -k 10 400 python tools/tune_gemms.py --model llama3-8b > gpurun_out/tune/8b.txt 2>&1 || { tail -5 gpurun_out/tune/8b.txt; exit 1; }
grep -v amdgpu gpurun_out/tune/8b.txt | tail -3
cp k8s_llm_rca_amd/data/gemm_tuned_llama3-8b.csv gpurun_out/tune/
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tune/gpu_tests.log 2>&1 || { tail -20 gpurun_out/tune/gpu_tests.log; exit 1; }
tail -1 gpurun_out/tune/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/tune/bench.log 2>&1 || { tail -5 gpurun_out/tune/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/tune/bench.log | cut -c1-330
