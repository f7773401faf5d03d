export TMPDIR=/tmp; mkdir -p gpurun_out/mid
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/mid/t_gemm.log 2>&1 || { tail -20 gpurun_out/mid/t_gemm.log; exit 1; }
tail -1 gpurun_out/mid/t_gemm.log
for m in "llama3-8b" "llama3-70b --tp 8"; do
  tag=$(echo $m | tr ' ' '_')
  timeout -k 10 300 python tools/gemm_mid_sweep.py --model $m --emit > gpurun_out/mid/sweep_$tag.txt 2>&1 || { tail -5 gpurun_out/mid/sweep_$tag.txt; exit 1; }
done
timeout -k 10 300 python tools/gemm_mid_sweep.py --model llama3-70b --emit --ms 1,2,4,8,16,24,32,48,64,96,128 > gpurun_out/mid/sweep_llama3-70b_tp1.txt 2>&1 || exit 1
cp k8s_llm_rca_amd/data/gemm_dispatch_*.json gpurun_out/mid/
grep -h "silu+down\|per-layer" gpurun_out/mid/sweep_llama3-8b.txt
timeout -k 10 400 python bench.py > gpurun_out/mid/bench2.log 2>&1 || { tail -5 gpurun_out/mid/bench2.log; exit 1; }
grep '^{"metric"' gpurun_out/mid/bench2.log | cut -c1-330
