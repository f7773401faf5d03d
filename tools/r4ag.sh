# closing check of the round-4 tree (push epilogue, batched peer loads, merge16): GPU suite + smoke + driver-contract bench, then the kernel profile of the
# contract run (the first pass also ran tools/rccl_same_gpu.py last: RCCL refuses two ranks on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/gpu_check.sh r4final4 || exit 1
bash tools/prof_driver.sh r4final4 || exit 1
