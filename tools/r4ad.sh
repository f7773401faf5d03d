#!/bin/bash
# round 4: tp-sim 70B TP=8 with the batched peer loads, staged (default) vs push epilogue
set -o pipefail
O=gpurun_out/tpsim_push
mkdir -p $O
timeout -k 10 500 python3 -u bench.py --model llama3-70b --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim70b.json 2> $O/tpsim70b.err || { tail -5 $O/tpsim70b.err; exit 1; }
K8SRCA_TP_PUSH=1 timeout -k 10 500 python3 -u bench.py --model llama3-70b --tp-sim 8 --steps 10 --warmup 3 > $O/tpsim70b_push.json 2> $O/tpsim70b_push.err || { tail -5 $O/tpsim70b_push.err; exit 1; }
python3 - <<'PY'
import json
for f in ("tpsim70b", "tpsim70b_push"):
    d = json.load(open(f"gpurun_out/tpsim_push/{f}.json"))
    t = d["tp_sim"]
    print(f, d["value"], d["p50_latency_s"], t["standin_collectives_s"], t["modelled_xgmi_collectives_s"], t["projected_value"], d["tokens"]["sampled"])
PY
