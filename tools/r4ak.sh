#!/bin/bash
# round 4, last GPU check: the whole GPU suite + smoke on the final tree (sampler non-finite guard,
# tp-sim fused stand-in), then the 70B TP=8 tp-sim projection with the fused-collective stand-in
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
NO_BENCH=1 bash tools/gpu_check.sh r4final6 || exit 1
bash tools/r4aj.sh || exit 1
