#!/bin/bash
# Mixtral-8x7B with its 32k window (preset mixtral-10k) above the concurrency that fits in HBM,
# idle threads on the KV host tier; then the preset's own 48 for comparison on the same box.
set -o pipefail
O=gpurun_out/r6/kvhost; mkdir -p $O
run() {  # tag, args
  timeout -k 10 560 python -u bench.py --preset mixtral-10k --no-hints-steps 0 --time-budget 500 $2 > $O/$1.json 2> $O/$1.err \
    || { grep -av "message compat" $O/$1.err | tail -12; return 1; }
  python -c "
import json; d=json.load(open('$O/$1.json')); e=d['engine']
print('$1', d['value'], d['p50_latency_s'], d['p90_latency_s'], d['errors'], d['sanity']['ok'], 'evict', e['evictions'], 'preempt', e['preemptions'], 'swaps', e.get('swap_outs'), e.get('swap_ins'), 'batch', d['throughput']['avg_decode_batch'], 'kvutil', d['throughput']['kv_peak_util'], d['work_per_analysis'])"
}
run mix32k_96_host "--incidents 96 --quantum 12 --kv-host-gb 120" && run mix32k_48 ""
# the 70B TP=8 projection at round 4's 128 concurrent analyses (after the TP=8 table re-sweep)
[ -n "$TPSIM128" ] && { timeout -k 10 560 python -u bench.py --model llama3-70b --tp-sim 8 --incidents 128 --steps 10 --warmup 3 \
  --no-hints-steps 0 > $O/tpsim70b_128.json 2> $O/tpsim70b_128.err || { tail -12 $O/tpsim70b_128.err; exit 1; }
  python -c "import json; d=json.load(open('$O/tpsim70b_128.json')); print('tpsim70b_128', d['value'], d['p50_latency_s'], d['tp_sim']['projected_value'])"; }
exit 0
