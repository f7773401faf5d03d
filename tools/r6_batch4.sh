#!/bin/bash
# After the table re-sweeps: the concurrent host-tier test, the 70B TP=8 projection (--tp-sim 8)
# and the Mixtral 8k preset, each against its round-4/5 number.
set -o pipefail
O=gpurun_out/r6/batch4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "kv_host" -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
show() { python -c "
import json; d=json.load(open('$O/$1.json')); e=d['engine']
print('$1', d['value'], d['p50_latency_s'], d['p90_latency_s'], d['errors'], d['sanity']['ok'], 'proj', (d.get('tp_sim') or {}).get('projected'), 'batch', d['throughput']['avg_decode_batch'], d['work_per_analysis'])"; }
timeout -k 10 560 python -u bench.py --model llama3-70b --tp-sim 8 --steps 10 --warmup 3 --no-hints-steps 0 \
  > $O/tpsim70b.json 2> $O/tpsim70b.err || { tail -12 $O/tpsim70b.err; exit 1; }
show tpsim70b
timeout -k 10 560 python -u bench.py --preset mixtral-10k-8k --no-hints-steps 0 > $O/mix8k64.json 2> $O/mix8k64.err \
  || { tail -12 $O/mix8k64.err; exit 1; }
show mix8k64
