#!/bin/bash
# KV host tier on the GPU: its tests, then Llama-3-70B TP=1 at 40 concurrent
# analyses with idle threads swapped to a 100 GB host tier.
set -o pipefail
O=gpurun_out/r6/kvhost
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -k "kv_stage or kv_host" -x -v --timeout 200 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 $O/tests.log
ARGS="--model llama3-70b --quantum 4 --steps 10 --warmup 2 --no-hints-steps 0 --time-budget ${TB:-700}"
timeout -k 10 ${BT:-820} python -u bench.py $ARGS --incidents ${INC:-40} ${EXTRA:---kv-host-gb 100} \
    > $O/${TAG:-b40_host}.json 2> $O/${TAG:-b40_host}.err || { tail -20 $O/${TAG:-b40_host}.err; exit 1; }
python -c "
import json,sys; d=json.load(open('$O/${TAG:-b40_host}.json'))
e=d['engine']; print(d['value'], d['p50_latency_s'], d['p90_latency_s'], d['errors'], d['sanity']['ok'], e['evictions'], e['preemptions'], e.get('swap_outs'), e.get('swap_ins'), e.get('kv_host'), d['throughput']['avg_decode_batch'], d['work_per_analysis'])"
