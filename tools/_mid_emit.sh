export TMPDIR=/tmp; mkdir -p gpurun_out/mid
timeout -k 10 300 python tools/gemm_mid_sweep.py --model llama3-8b --emit > gpurun_out/mid/sweep_8b.txt 2>&1 || { tail -5 gpurun_out/mid/sweep_8b.txt; exit 1; }
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-8b.json gpurun_out/mid/
timeout -k 10 300 python tools/gemm_mid_sweep.py --model llama3-70b --emit --ms 1,2,4,8,16,24,32,48,64,96,128 > gpurun_out/mid/sweep_70b.txt 2>&1 || { tail -5 gpurun_out/mid/sweep_70b.txt; exit 1; }
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-70b.json gpurun_out/mid/
timeout -k 10 300 python tools/gemm_mid_sweep.py --model llama3-70b --tp 8 --emit > gpurun_out/mid/sweep_70b_tp8.txt 2>&1 || { tail -5 gpurun_out/mid/sweep_70b_tp8.txt; exit 1; }
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-70b-tp8.json gpurun_out/mid/
grep "per-layer" gpurun_out/mid/sweep_*.txt
timeout -k 10 400 python bench.py > gpurun_out/mid/bench.log 2>&1 || { tail -5 gpurun_out/mid/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/mid/bench.log | cut -c1-330
