# the TP=2 shared-GPU tests alone (did the closing check's failure reproduce?), then with the round-4
# prefill defaults switched back (fixed-target planner, VAR 4 attention) to bisect
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_tp_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tp.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tp.log | tail -12
[ $rc -eq 0 ] && exit 0
K8S_PF_OVERHEAD_PAGES=0 K8SRCA_PF_W8=4 timeout -k 10 400 python3 -u -m pytest tests/test_tp_gpu.py -x -v --timeout 150 --timeout-method thread -k graph_replay_matches > $O/tp_old.log 2>&1
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tp_old.log | tail -5
