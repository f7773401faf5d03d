#!/bin/bash
# round 4: Mixtral-8x7B EP=8 tp-sim on the final tree (batched peer loads in the all-reduce / all-to-all)
set -o pipefail
O=gpurun_out/tpsim_mix_final; mkdir -p $O
timeout -k 10 600 python3 -u bench.py --preset mixtral-10k --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim_mixtral.json 2> $O/tpsim_mixtral.err || { tail -5 $O/tpsim_mixtral.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/tpsim_mix_final/tpsim_mixtral.json").read().strip().splitlines()[-1])
t = d["tp_sim"]
print(d["value"], d["p50_latency_s"], t["standin_collectives_s"], t["modelled_xgmi_collectives_s"], t["projected_value"], t["projected_value_by_hop_us"], d["work_per_analysis"], d["engine"]["graph_steps"])
PY
