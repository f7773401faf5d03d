#!/bin/bash
# round 4: 70B TP=8 tp-sim with the fused-collective stand-in in the projection
set -o pipefail
O=gpurun_out/tpsim_fused; mkdir -p $O
timeout -k 10 500 python3 -u bench.py --model llama3-70b --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim70b.json 2> $O/tpsim70b.err || { tail -5 $O/tpsim70b.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/tpsim_fused/tpsim70b.json").read().strip().splitlines()[-1])
t = d["tp_sim"]
print(d["value"], d["p50_latency_s"], t["standin_collectives_s"], t["modelled_xgmi_collectives_s"], t["projected_value"], t["projected_value_by_hop_us"], d["work_per_analysis"])
print({k: v for k, v in list(t["per_T"].items())[:3]})
PY
