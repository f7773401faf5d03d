# the decode GEMM hand-read bit-identity test, then the c = 112 latency-curve point on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4aa; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "glds_hand or gemm_stream or grouped_glds" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/latency_curve.sh 112 96 || exit 1
