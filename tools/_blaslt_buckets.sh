# bucketed hipBLASLt tuning, then the recorded-step replay with and without the new table
export TMPDIR=/tmp; O=gpurun_out/blaslt_buckets; mkdir -p $O
timeout -k 10 700 python3 tools/blaslt_tune_buckets.py --emit --out $O/blaslt_algos_llama3-8b.json > $O/tune.txt 2>&1 || { tail -5 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt | tail -60
timeout -k 10 200 env K8S_BLASLT_ALGOS=0 python3 tools/blaslt_ab.py > $O/heur.txt 2>&1 || { tail -5 $O/heur.txt; exit 1; }
timeout -k 10 200 env K8S_BLASLT_ALGOS=1 python3 tools/blaslt_ab.py > $O/table.txt 2>&1 || { tail -5 $O/table.txt; exit 1; }
tail -n 9 $O/heur.txt $O/table.txt
