# full GPU suite (shared-GPU TP / EP tests with a capped collective grid), then the decode GEMM A/B of the
# hand-issued LDS reads (K8SRCA_GLDS_HAND)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u tools/glds_hand_ab.py > $O/glds_hand.txt 2>&1 || { tail -5 $O/glds_hand.txt; exit 1; }
grep '^{' $O/glds_hand.txt | cut -c1-220
