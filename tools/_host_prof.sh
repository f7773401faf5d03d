export TMPDIR=/tmp; mkdir -p gpurun_out/hostprof
K8S_RCA_PROFILE_ENGINE=/tmp/eng.prof timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/hostprof/bench.log 2>&1 || { tail -5 gpurun_out/hostprof/bench.log; exit 1; }
python3 - <<'PY' > gpurun_out/hostprof/stats.txt
import pstats
p = pstats.Stats('/tmp/eng.prof')
p.sort_stats('tottime').print_stats(45)
p.sort_stats('cumtime').print_stats(60)
PY
head -120 gpurun_out/hostprof/stats.txt | cut -c1-160
