#!/bin/bash
# Interleaved A/B between two builds of the HIP library (K8SRCA_HIP_LIB):
# decode attention at the headline shape (decode_probe.py) and the decode
# projections at one row (decode_gemm_probe.py --m 1: the skinny kernel), N rounds.
# usage (GPU box): tools/decode_ab.sh OLD_LIB [rounds]   -> stdout
R=${GRAFT_REPO_ROOT:-.}; old=$1; n=${2:-3}
for i in $(seq 1 $n); do
  for arm in old new; do
    if [ $arm = old ]; then export K8SRCA_HIP_LIB=$old; else unset K8SRCA_HIP_LIB; fi
    echo "== round $i $arm"
    timeout -k 10 120 python3 $R/tools/decode_probe.py || exit 1
    timeout -k 10 120 python3 $R/tools/decode_gemm_probe.py --m 1 --shapes qkv,o || exit 1
  done
done
