#!/bin/bash
# round 6 final tree (after the search / act kernel trims), part A: traffic + VALU (slot) records and
# summaries (part B, scripts/cmd/r6y.sh: bench lines on the recorded files, smoke, GPU suite)
set -u
O=gpurun_out/r6fk
mkdir -p $O
V="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
A="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"
SRCH="--mode search --workload llama3-8b"
ACT="--mode act"
P="--steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
T=$O/pmc_traffic.json
VJ=$O/pmc_valu.json
cp profiles/round6/pmc_traffic.json $T
cp profiles/round6/pmc_valu.json $VJ
bash scripts/gpu_run.sh r6fk \
 "prof70:700:STEPS=20 TRAFFIC_OUT=$T COMMIT=r6fk bash scripts/profile_round.sh r6fk/l70" \
 "prof8f16:600:STEPS=20 WL_ARGS='--workload llama3-8b --dtype f16' TRAFFIC_KEY=llama3-8b.b4.asym.packed.f16 TRAFFIC_OUT=$T COMMIT=r6fk bash scripts/profile_round.sh r6fk/l8f16" \
 "pmc_search:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $V --output-format csv -d $O/pmc_search -o p -- python bench.py $SRCH $P" \
 "pmc_act:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $V --output-format csv -d $O/pmc_act -o p -- python bench.py $ACT $P" \
 "valu_json:60:python scripts/pmc_valu.py --pmc-dir $O/pmc_search --kernel awq_fast_kernel --units-per-dispatch 80302612480 --key llama3-8b.b4.asym.packed.search10of20 --sources fast --commit r6fk --out $VJ && python scripts/pmc_valu.py --pmc-dir $O/pmc_act --kernel act_loss_kernel --units-per-dispatch 623153737.142857 --key act.llama3-8b-block.t512.g20.bf16.b4.asym --sources act --commit r6fk --out $VJ" \
 "search_a:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $A --output-format csv -d $O/search_a -o p -- python bench.py $SRCH $P" \
 "search_b:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $B --output-format csv -d $O/search_b -o p -- python bench.py $SRCH $P" \
 "act_a:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $A --output-format csv -d $O/act_a -o p -- python bench.py $ACT $P" \
 "act_b:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $B --output-format csv -d $O/act_b -o p -- python bench.py $ACT $P"
