#!/bin/bash
# (tools/splitk_an_ab.py was removed with the reverted kernel change; results in profiles/r4/splitk_an/)
# round 4: split-count-templated split-K add+norm -- norm kernel tests (bit-identity vs reduce + rmsnorm), A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4am; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "splitk or rmsnorm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 200 python3 -u tools/splitk_an_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
