# 128-column LDS-DMA strips: numerics, then the 8B decode-GEMM dispatch sweep (table to gpurun_out)
export TMPDIR=/tmp; O=gpurun_out/bn128; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_stream" > $O/test.log 2>&1; e=$?; tail -2 $O/test.log; [ $e -eq 0 ] || exit $e
timeout -k 10 300 python3 tools/gemm_mid_sweep.py --emit --out $O/gemm_dispatch_llama3-8b.json > $O/sweep.txt 2>&1 || { tail -5 $O/sweep.txt; exit 1; }
grep "per-layer" $O/sweep.txt | cut -c1-125
grep "^M 128\|^M  96\|^M 192" $O/sweep.txt | cut -c1-200
