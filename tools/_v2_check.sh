export TMPDIR=/tmp; mkdir -p gpurun_out/v2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rope" > gpurun_out/v2/rope_tests.log 2>&1; e=$?; tail -3 gpurun_out/v2/rope_tests.log; [ $e -eq 0 ] || exit $e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v2/gpu_tests.log 2>&1; e=$?; tail -3 gpurun_out/v2/gpu_tests.log; [ $e -eq 0 ] || exit $e
timeout -k 10 450 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/v2/bench.log 2>&1; e=$?; tail -1 gpurun_out/v2/bench.log | cut -c1-400; exit $e
