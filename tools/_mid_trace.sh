#!/bin/bash
# Kernel trace of the decode GEMM sweep at a few M: per-kernel durations
# (main split-K kernel vs its reduce kernel vs hipBLASLt).
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=$R/gpurun_out/midtrace; mkdir -p $O
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
  python3 $R/tools/gemm_mid_sweep.py --ms ${1:-96} > $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; exit 1; }
t=$(find $O -name "*kernel_trace.csv" | head -1)
python3 - "$t" > $O/kinds.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"][:70]
    g = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]), int(r["Workgroup_Size_X"]))
    agg[(n, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(agg.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    print(f"{len(v):6d} med {v[len(v)//2]:8.2f}us  grid {g}  {n}")
PY
cat $O/sweep.log | grep "^M"; head -80 $O/kinds.txt; rm -f $t
