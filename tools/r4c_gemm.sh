# round-4 GEMM check: tests, A/B with K splits + dispatch emit, then the MoE tp-sim test
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r4e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm_big or layer_executor" > $O/tests.log 2>&1 || { grep -E "^E |Error|passed|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/big_gemm_ab.py --ms 512,768,1024,1536,2048,3072,4096,6144,8192 --pipes 1 --rounds 3 --out $O/ab.jsonl --emit $O/gemm_big_llama3-8b.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cut -c1-250 $O/ab.log
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_tp_gpu.py -k "moe" > $O/tests_moe.log 2>&1 || { grep -E "^E " $O/tests_moe.log | cut -c1-600 | head -20; exit 1; }
tail -2 $O/tests_moe.log
