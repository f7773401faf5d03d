#!/bin/bash
# Mixtral-8x7B, 8k window, with the KV host tier at a higher concurrency than fits in HBM alone.
set -o pipefail
O=gpurun_out/r6/kvhost
mkdir -p $O
timeout -k 10 ${BT:-900} python -u bench.py --preset mixtral-10k-8k --incidents ${INC:-128} --quantum ${Q:-16} \
    --no-hints-steps 0 --time-budget ${TB:-780} ${EXTRA:---kv-host-gb 100} > $O/${TAG:-mix128_host}.json \
    2> $O/${TAG:-mix128_host}.err || { grep -av "message compat" $O/${TAG:-mix128_host}.err | tail -20; exit 1; }
python -c "
import json; d=json.load(open('$O/${TAG:-mix128_host}.json'))
e=d['engine']; print(d['value'], d['p50_latency_s'], d['p90_latency_s'], d['errors'], d['sanity']['ok'], e['evictions'], e['preemptions'], e.get('swap_outs'), e.get('swap_ins'), e.get('kv_host'), d['throughput'], d['work_per_analysis'])"
