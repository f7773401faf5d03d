# GPU suite, then a kernel-trace profile of the headline contract (tag given as $1)
export TMPDIR=/tmp; mkdir -p gpurun_out/v3
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v3/gpu_tests.log 2>&1; e=$?; tail -3 gpurun_out/v3/gpu_tests.log; [ $e -eq 0 ] || exit $e
bash tools/prof_driver.sh $1 > gpurun_out/v3/prof.log 2>&1; e=$?; head -c 600 gpurun_out/v3/prof.log; exit $e
