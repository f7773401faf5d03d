export TMPDIR=/tmp; mkdir -p gpurun_out/grp
timeout -k 10 300 python tools/gemm_mid_sweep.py --model llama3-8b --emit > gpurun_out/grp/sweep_8b.txt 2>&1 || { tail -5 gpurun_out/grp/sweep_8b.txt; exit 1; }
cp k8s_llm_rca_amd/data/gemm_dispatch_llama3-8b.json gpurun_out/grp/
grep -h "per-layer" gpurun_out/grp/sweep_8b.txt
grep -h "^M 128\|^M  64" gpurun_out/grp/sweep_8b.txt | cut -c1-250
timeout -k 10 240 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/grp/gpu_tests.log 2>&1 || { tail -20 gpurun_out/grp/gpu_tests.log; exit 1; }
tail -1 gpurun_out/grp/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/grp/bench.log 2>&1 || { tail -5 gpurun_out/grp/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/grp/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; t=d['throughput']; print(d['value'], d['p50_latency_s'], t['avg_decode_batch'])"
