set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r4b; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" > gpurun_out/r4b/tests.log 2>&1 || { tail -30 gpurun_out/r4b/tests.log; exit 1; }
tail -2 gpurun_out/r4b/tests.log
timeout -k 10 400 python -u tools/big_gemm_ab.py --ms 1024,2048,4096,8192 --pipes 3,1,2,0 --rounds 3 --out gpurun_out/r4b/ab.jsonl > gpurun_out/r4b/ab.log 2>&1 || { tail -20 gpurun_out/r4b/ab.log; exit 1; }
cat gpurun_out/r4b/ab.log
