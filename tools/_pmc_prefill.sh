#!/bin/bash
# PMC passes (one counter group per run, no trace domains) over replayed prefill attention launches.
# usage: tools/_pmc_prefill.sh TAG [trace]    (K8SRCA_PF_W8 in the environment picks the kernel)
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; cd /tmp; tag=${1:-pf}; O=$R/gpurun_out/pmc_$tag; mkdir -p $O
TR=${2:-$R/profiles/r3/shape_trace_steady.jsonl}
P="python3 $R/tools/prof_prefill_replay.py --trace $TR --samples 30"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${tag}_kt -o run -- $P > $O/kt.log 2>&1 || exit 1
cp $(find /tmp/${tag}_kt -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d /tmp/${tag}_p1 -o run -- $P > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d /tmp/${tag}_p2 -o run -- $P > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d /tmp/${tag}_p3 -o run -- $P > $O/p3.log 2>&1 || exit 1
for p in p1 p2 p3; do cp $(find /tmp/${tag}_$p -name "*counter_collection.csv" | head -1) $O/$p.csv; done
O=$O python3 - <<'PY'
import csv, collections, os
O = os.environ["O"]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for p in ("p1", "p2", "p3"):
    for r in csv.DictReader(open(f"{O}/{p}.csv")):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "prefill" in k or "merge" in k:
        print(k, {c: round(v / max(1, n[(k, c)])) for c, v in d.items()})
PY
