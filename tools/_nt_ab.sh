# Weight-stream cache policy A/B: nt (default build) vs default policy (K8S_W_NT=0 build,
# k8s_llm_rca_amd/libk8srca_hip_wnt0.so), decode-GEMM sweep interleaved nt / off / nt / off
export TMPDIR=/tmp; O=gpurun_out/nt_ab; mkdir -p $O
for v in nt0 off0 nt1 off1; do
  case $v in off*) L=$GRAFT_REPO_ROOT/k8s_llm_rca_amd/libk8srca_hip_wnt0.so;; *) L=;; esac
  timeout -k 10 200 env K8SRCA_HIP_LIB=$L python3 tools/gemm_mid_sweep.py --ms 1,8,16,32,64,96,128,160,192,256 > $O/$v.txt 2>&1 || { tail -5 $O/$v.txt; exit 1; }
  grep "per-layer" $O/$v.txt | awk -v v=$v '{print v, $0}' | cut -c1-120
done
