# gemm_big variants: kernel tests (16x16 / 32x32, SwiGLU, RoPE epilogue, grouped, split) + A/B + emit
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r4g2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm_big or grouped_big or layer_executor or moe_prefill or rope or skinny" > $O/tests.log 2>&1 || { grep -E "^E |Error|passed|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python -u tools/big_gemm_ab.py --ms 512,1024,2048,3072,4096,6144,8192 --pipes 1,5 --rounds 3 --out $O/ab.jsonl --emit $O/gemm_big_llama3-8b.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cut -c1-330 $O/ab.log
