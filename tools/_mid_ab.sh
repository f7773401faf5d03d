export TMPDIR=/tmp; mkdir -p gpurun_out/mid
timeout -k 10 400 python tools/gemm_mid_sweep.py --model llama3-8b --emit > gpurun_out/mid/sweep.txt 2>&1 || { tail -5 gpurun_out/mid/sweep.txt; exit 1; }
grep -v amdgpu gpurun_out/mid/sweep.txt | tail -18
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-8b.json gpurun_out/mid/
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mid/gpu_tests.log 2>&1 || { tail -20 gpurun_out/mid/gpu_tests.log; exit 1; }
tail -1 gpurun_out/mid/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/mid/bench.log 2>&1 || { tail -5 gpurun_out/mid/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/mid/bench.log | cut -c1-330
