# after a flood of launches the HIP runtime's helper thread keeps polling while later GPU work runs:
# runtime settings vs that activation (probe phases: eager flood, then long hand-written GEMMs)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4t; mkdir -p $O
for arm in "X=0" "ROC_AQL_QUEUE_SIZE=65536" "HIP_FORCE_DEV_KERNARG=0" "ROC_USE_FGS_KERNARG=0" "DEBUG_CLR_MAX_BATCH_SIZE=4096" "AMD_DIRECT_DISPATCH=0"; do
  echo "== $arm"
  env $arm timeout -k 10 120 python3 -u tools/hip_thread_probe.py --n 100000 --phases big_gemm,eager_kernels,big_gemm#2,idle_2s,big_gemm#3 > $O/probe_$arm.txt 2>&1 || { tail -5 $O/probe_$arm.txt; exit 1; }
  grep -v amdgpu.ids $O/probe_$arm.txt
done
