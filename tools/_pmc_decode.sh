R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; cd /tmp; O=$R/gpurun_out/pmcd
mkdir -p $O
$R/tools/gpu_steps.sh 300 \
 "rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/prof_attn.py --mode decode --S 96 --ctx 3400 --iters 20" \
 "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU --output-format csv -d $O/p1 -o run -- python3 $R/tools/prof_attn.py --mode decode --S 96 --ctx 3400 --iters 3" \
 "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/p2 -o run -- python3 $R/tools/prof_attn.py --mode decode --S 96 --ctx 3400 --iters 3" \
 "rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $O/p3 -o run -- python3 $R/tools/prof_attn.py --mode decode --S 96 --ctx 3400 --iters 3" > $O/steps.log 2>&1
find $O -name "*kernel_trace.csv" -size +5M -delete
grep -c "exit 0" $O/steps.log
