# Round-end rehearsal: smoke(), the GPU suite, then the driver's headline contract
export TMPDIR=/tmp; O=gpurun_out/final2; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; e=$?; tail -1 $O/gpu_tests.log; [ $e -eq 0 ] || exit $e
timeout -k 10 450 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; e=$?; grep '^{' $O/bench.log | cut -c1-200; exit $e
