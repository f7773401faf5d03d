# GPU suite, the driver's headline contract, then a kernel-trace profile of it (tag $1)
export TMPDIR=/tmp; O=gpurun_out/v5; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; e=$?; tail -2 $O/gpu_tests.log; [ $e -eq 0 ] || exit $e
timeout -k 10 450 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; e=$?; grep '^{' $O/bench.log | cut -c1-300; [ $e -eq 0 ] || exit $e
bash tools/prof_driver.sh $1 > $O/prof.log 2>&1; e=$?; head -c 300 $O/prof.log; exit $e
