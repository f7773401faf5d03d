set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r4h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "rope_kv_epilogue" > $O/tests.log 2>&1; grep -E "^E  .*qkv|^E  .*pages|passed|failed" $O/tests.log | head -30
