#!/bin/bash
# Item-4 probe: the bench with every scratch / partial buffer NaN-poisoned at
# allocation and the per-layer non-finite flags on (knobs poison,
# nonfinite_check).  A kernel that reads memory no kernel wrote turns into
# NaN logits -> NON_FINITE rows / flags, instead of silently stale data.
# usage (GPU box): tools/probe_nonfinite.sh TAG [bench args]  -> gpurun_out/probe_TAG/
R=${GRAFT_REPO_ROOT:-.}; tag=$1; shift; O=$R/gpurun_out/probe_$tag; mkdir -p $O; cd $R
K8SRCA_POISON=1 K8SRCA_NONFINITE_CHECK=1 timeout -k 10 500 python3 bench.py "$@" > $O/bench.json 2> $O/bench.err
rc=$?; tail -3 $O/bench.err
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["engine"]
print("value", d["value"], "sanity", d["sanity"], "errors", d["errors"],
      {k: e.get(k) for k in ("nonfinite_rows", "nonfinite_flag_steps", "nonfinite_first_layer", "ends")},
      "sampled/analysis", d["work_per_analysis"]["sampled_tokens"])
PY
exit $rc
