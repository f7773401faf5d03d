#!/bin/bash
# Evidence for the TP=2 one-GPU rehearsal's variance: the 8B TP=2 bench as two
# processes on ONE GPU, twice plainly, then once under a kernel trace -- the all-reduce kernels'
# duration spread (min vs mean vs max) shows how long a rank's collective waits for its peer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-.}; O=$R/gpurun_out/r6/tp2; mkdir -p $O; export TMPDIR=/tmp
ARGS="--gpus 2 --tp 2 --same-gpu --kv-gb 40 --incidents 24 --quantum 4 --steps 6 --warmup 2 --no-hints-steps 0 --time-budget 300"
for i in 1 2; do
  timeout -k 10 420 python3 -u $R/bench.py $ARGS > $O/run_$i.json 2> $O/run_$i.err || { tail -8 $O/run_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run_$i.json').read().strip().splitlines()[-1]); print('run $i', d['value'], d['p50_latency_s'], d['engine']['wait_s'], d['engine']['forward_s'])"
done
T=/tmp/tp2prof; rm -rf $T; mkdir -p $T
cd /tmp && timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- \
  python3 $R/bench.py $ARGS > $O/prof_run.json 2> $O/prof_run.err || { tail -8 $O/prof_run.err; exit 1; }
for f in $(find $T -name "*kernel_stats.csv"); do cp $f $O/$(basename $(dirname $f))_kernel_stats.csv 2>/dev/null || cp $f $O/; done
python3 - "$T" "$O" <<'PY'
import csv, glob, os, sys
T, O = sys.argv[1], sys.argv[2]
out = []
for f in glob.glob(os.path.join(T, "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "ar_" in n or "allreduce" in n.lower() or "push" in n.lower():
            out.append(f"{os.path.relpath(f, T)}  {int(r['Calls']):7d} calls  avg {float(r['AverageNs'])/1e3:9.1f} us  min {float(r['MinNs'])/1e3:8.1f}  max {float(r['MaxNs'])/1e3:10.1f}  {n[:90]}")
open(os.path.join(O, "ar_kernels.txt"), "w").write("\n".join(out) + "\n")
print("\n".join(out[:20]))
PY
rm -rf $T
