# Interleaved A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the default
set -e
for v in 1 0 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py > gpurun_out/ab_kernarg_$v.log 2>&1
  echo "kernarg=$v $(grep -o '"value": [0-9.]*\|"p50_latency_s": [0-9.]*' gpurun_out/ab_kernarg_$v.log | tr '\n' ' ')"
done
