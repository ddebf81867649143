# round 5: counters of the one-pass weight column-sum kernel (act path) — what bounds it
set -u
O=gpurun_out/r5z
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES TCC_EA0_RDREQ_sum TCC_HIT_sum GRBM_GUI_ACTIVE"
AB="scripts/act_search_bench.py --iters 2 --groups gate_up"
bash scripts/gpu_run.sh r5z \
 "pmc_a:150:timeout -s KILL 140 rocprofv3 --kernel-include-regex wcolsum_fused_kernel --pmc $A --output-format csv -d $O/pmc_a -o p -- python $AB" \
 "pmc_b:150:timeout -s KILL 140 rocprofv3 --kernel-include-regex wcolsum_fused_kernel --pmc $B --output-format csv -d $O/pmc_b -o p -- python $AB" \
 "trace:150:timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace -o t --output-format csv -- python $AB"
