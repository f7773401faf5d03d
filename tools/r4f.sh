# GPU suite + interleaved headline A/B: hipBLASLt prefill GEMMs vs gemm_big dispatch
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r4f
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4f/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/r4f/tests.log | head -20; exit 1; }
tail -1 gpurun_out/r4f/tests.log
bash tools/ab.sh big 2 "K8SRCA_BIG_GEMM=0" "K8SRCA_BIG_GEMM=1" -- --steps 20 --warmup 5
