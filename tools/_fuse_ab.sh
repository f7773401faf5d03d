#!/bin/bash
# A/B: split-K reduce fused into the residual add + RMSNorm (executor) on vs off, headline config
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fuse_ab; mkdir -p $O; cd $R
for f in 1 0 1 0; do
  K8SRCA_FUSE_SPLITK=$f timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 > $O/b$f.log 2>&1 || { tail -5 $O/b$f.log; exit 1; }
  echo "fuse=$f $(grep '^{' $O/b$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_s"])')"
done
