#!/bin/bash
# The HIP runtime's busy thread: contract bench under runtime settings that
# change how it waits -- default, direct dispatch forced on, no active-wait spin.
set -o pipefail
O=gpurun_out/r6/rt_env; mkdir -p $O
run() {  # tag, env
  env $2 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-hints-steps 0 > $O/$1.json 2> $O/$1.err \
    || { echo "$1 failed"; tail -8 $O/$1.err; return 1; }
  python -c "
import json; d=json.load(open('$O/$1.json')); n=d['native_threads']
print('$1', d['value'], d['p50_latency_s'], 'top_cpu_s', n['top_cpu_s'][:3], 'busiest', [(b.get('wchan'), b.get('user_s'), b.get('sys_s')) for b in n['busiest'][:2]], 'engine', d['host_cpu_s'])"
}
run base "" && run direct "AMD_DIRECT_DISPATCH=1" && run nospin "ROC_ACTIVE_WAIT_TIMEOUT=0" && run base2 ""
