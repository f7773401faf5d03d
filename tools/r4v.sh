# closing check of the round-4 tree: GPU suite + smoke + driver-contract bench, the kernel profile of the
# contract run, then whether RCCL runs with two ranks on one GPU (last: it may hang)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/gpu_check.sh r4final || exit 1
bash tools/prof_driver.sh r4final || exit 1
timeout -k 10 200 python3 -u tools/rccl_same_gpu.py > gpurun_out/rccl_same_gpu.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/rccl_same_gpu.txt | tail -4; exit $rc
