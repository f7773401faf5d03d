#!/bin/bash
# Where do the GPU's idle gaps in the headline run come from?  Kernel + HIP API + memory-copy trace
# of a short bench run (no PMC), summarised on the box: gaps by preceding step kind
# (tools/gap_steps.py) and the host API calls overlapping them (tools/gap_api.py).
# usage (GPU box): tools/prof_gaps.sh TAG [bench args...]  -> gpurun_out/gaps_TAG/
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; tag=$1; shift
O=$R/gpurun_out/gaps_$tag; mkdir -p $O; T=/tmp/gaps_$tag; rm -rf $T; mkdir -p $T
# (--memory-copy-trace with --hip-trace segfaulted rocprofv3 at exit after a complete run.)  The
# profiler's exit status is kept, but the CPU-only summaries below run on whatever traces it wrote.
cd /tmp && timeout -k 10 700 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $T -o run -- \
  python3 $R/bench.py --steps 8 --warmup 3 --no-hints-steps 0 "$@" > $O/bench.log 2>&1
rc=$?
grep '^{"metric"' $O/bench.log | cut -c1-300
k=$(find $T -name "*kernel_trace.csv" | head -1); a=$(find $T -name "*hip_api_trace.csv" | head -1)
m=$(find $T -name "*memory_copy_trace.csv" | head -1)
python3 $R/tools/gap_steps.py $k --min-us 200 --from-frac 0.5 > $O/gap_steps.txt 2>&1; head -40 $O/gap_steps.txt
timeout -k 5 600 python3 -u $R/tools/gap_api.py $k $a --min-us 500 2>&1 | tee $O/gap_api.txt | grep "^# api rows" | tail -1; grep -v "^# api rows" $O/gap_api.txt | head -40
[ -n "$m" ] && head -3 $m > $O/memcpy_head.csv && python3 - "$m" > $O/memcpy_summary.txt <<'PY'
import csv, sys, collections
c = collections.defaultdict(lambda: [0, 0.0, 0])
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Direction") or r.get("Operation") or "?"
    c[k][0] += 1
    c[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    c[k][2] += int(r.get("Size") or 0)
for k, (n, ms, b) in sorted(c.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:30s} n={n:8d} {ms:10.1f} ms {b / 1e6:10.1f} MB")
PY
cat $O/memcpy_summary.txt 2>/dev/null
rm -rf $T
exit $rc
