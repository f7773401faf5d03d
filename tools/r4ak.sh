#!/bin/bash
# round 4, last GPU check of the final tree (sampler non-finite guard, decode reduce prefetch form,
# tp-sim fused stand-in): the whole GPU suite + smoke + the driver-contract bench, then the 70B TP=8
# tp-sim projection with the fused-collective stand-in
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/gpu_check.sh r4final6 || exit 1
bash tools/r4aj.sh || exit 1
