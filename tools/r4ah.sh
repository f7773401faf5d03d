#!/bin/bash
# round 4: the closing profile run generated ~22 tokens per analysis (normal: ~960) -- reproduce under
# rocprofv3 with the default tree, then with the previous prefill merge (K8SRCA_PF_MERGE16=0)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4ah; mkdir -p $O
s() { python3 -c "import json; d=[json.loads(l) for l in open('$1') if l.startswith('{\"metric')][-1]; print('$1', d['value'], d['work_per_analysis'], d['engine']['graph_steps'])"; }
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-hints-steps 0 > $GRAFT_REPO_ROOT/$O/prof_default.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_default.log; exit 1; }
cd $GRAFT_REPO_ROOT; s $O/prof_default.log; cd /tmp
K8SRCA_PF_MERGE16=0 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/p2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-hints-steps 0 > $GRAFT_REPO_ROOT/$O/prof_merge4.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_merge4.log; exit 1; }
cd $GRAFT_REPO_ROOT; s $O/prof_merge4.log
