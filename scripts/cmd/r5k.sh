# round 5: VALU issue model — per-instruction-class issue rates (probe) and the dual-issue /
# per-type counters of the probe, the clip search and the act loss kernel
set -u
O=gpurun_out/r5k
mkdir -p $O
A="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"
SRCH="--mode search --workload llama3-8b --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
ACT="--mode act --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
bash scripts/gpu_run.sh r5k \
 "probe:200:scripts/valu_probe --ghz 2.4" \
 "probe_pmc_a:90:timeout -s KILL 80 rocprofv3 --pmc $A --output-format csv -d $O/probe_a -o p -- scripts/valu_probe" \
 "probe_pmc_b:90:timeout -s KILL 80 rocprofv3 --pmc $B --output-format csv -d $O/probe_b -o p -- scripts/valu_probe" \
 "search_a:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $A --output-format csv -d $O/search_a -o p -- python bench.py $SRCH" \
 "search_b:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $B --output-format csv -d $O/search_b -o p -- python bench.py $SRCH" \
 "act_a:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $A --output-format csv -d $O/act_a -o p -- python bench.py $ACT" \
 "act_b:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $B --output-format csv -d $O/act_b -o p -- python bench.py $ACT"
