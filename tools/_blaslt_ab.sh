# hipBLASLt heuristic vs swept table vs table + ladder padding on the recorded prefill-sized GEMMs
export TMPDIR=/tmp; O=gpurun_out/blaslt_ab; mkdir -p $O
timeout -k 10 200 env K8S_BLASLT_ALGOS=0 python3 tools/blaslt_ab.py > $O/heur.txt 2>&1 || { tail -5 $O/heur.txt; exit 1; }
timeout -k 10 200 env K8S_BLASLT_ALGOS=1 python3 tools/blaslt_ab.py > $O/table.txt 2>&1 || { tail -5 $O/table.txt; exit 1; }
timeout -k 10 200 env K8S_BLASLT_ALGOS=1 python3 tools/blaslt_ab.py --pad > $O/table_pad.txt 2>&1 || { tail -5 $O/table_pad.txt; exit 1; }
tail -n 9 $O/heur.txt $O/table.txt $O/table_pad.txt
