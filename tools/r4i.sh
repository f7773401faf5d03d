# headline under rocprofv3 (kernel summary) + one interleaved A/B round of the gemm_big dispatch
# + the 70B TP=8 per-rank gemm_big table
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r4i
bash tools/prof_driver.sh r4i || exit 1
timeout -k 10 600 python -u tools/big_gemm_ab.py --model llama3-70b --tp 8 --ms 512,1024,2048,3072,4096,6144,8192 --pipes 1 --rounds 3 --out gpurun_out/r4i/ab70.jsonl --emit gpurun_out/r4i/gemm_big_llama3-70b-tp8.json > gpurun_out/r4i/ab70.log 2>&1 || { tail -5 gpurun_out/r4i/ab70.log; exit 1; }
tail -1 gpurun_out/r4i/ab70.log | cut -c1-600
bash tools/ab.sh big2 1 "K8SRCA_BIG_GEMM=0" "K8SRCA_BIG_GEMM=1" -- --steps 20 --warmup 5
