R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; cd /tmp; O=$R/gpurun_out/pmc
mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1
$R/tools/gpu_steps.sh 300 \
 "rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/prof_attn.py --S 8 --q 512 --ctx 3000" \
 "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 $R/tools/prof_attn.py --S 8 --q 512 --ctx 3000 --iters 3" \
 "rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- python3 $R/tools/prof_attn.py --S 8 --q 512 --ctx 3000 --iters 3" \
 "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/p3 -o run -- python3 $R/tools/prof_attn.py --S 8 --q 512 --ctx 3000 --iters 3" > $O/steps.log 2>&1
grep -i "mfma\|lds\|SQ_WAIT\|TCC_HIT\|TCC_MISS\|SQ_BUSY" $O/counters_list.txt | head -60 > $O/counters_grep.txt
find $O -name "*kernel_trace.csv" -size +5M -delete
tail -20 $O/steps.log
