#!/bin/bash
# Kernel trace + PMC passes (one counter group per rocprofv3 run, no trace domains) over any python tool.
# usage (GPU box): tools/pmc.sh TAG python3 tools/prof_prefill_replay.py --samples 30   (env picks variants)
# -> gpurun_out/pmc_TAG/{kernel_stats.csv,p1.csv,p2.csv,p3.csv} and a per-kernel average summary.
R=${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; tag=$1; shift; O=$R/gpurun_out/pmc_$tag; mkdir -p $O; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${tag}_kt -o run -- "$@" > $O/kt.log 2>&1 || exit 1
cp $(find /tmp/${tag}_kt -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d /tmp/${tag}_p1 -o run -- "$@" > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d /tmp/${tag}_p2 -o run -- "$@" > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d /tmp/${tag}_p3 -o run -- "$@" > $O/p3.log 2>&1 || exit 1
for p in p1 p2 p3; do cp $(find /tmp/${tag}_$p -name "*counter_collection.csv" | head -1) $O/$p.csv; done
O=$O python3 - <<'PY'
import csv, collections, os
O = os.environ["O"]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for p in ("p1", "p2", "p3"):
    for r in csv.DictReader(open(f"{O}/{p}.csv")):
        k = r["Kernel_Name"].split("(")[0][-48:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:12]:
    print(k, {c: round(v / max(1, n[(k, c)])) for c, v in d.items()})
PY
