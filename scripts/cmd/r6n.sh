#!/bin/bash
# act loss kernel re-recorded after the round-6 trims (r6m): VALU slot pass, per-type counters,
# bench line and kernel trace
set -u
O=gpurun_out/r6n
mkdir -p $O
cp profiles/round6/pmc_valu.json $O/pmc_valu.json
V="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
A="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"
ACT="--mode act"
P="--steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
VJ=$O/pmc_valu.json
bash scripts/gpu_run.sh r6n \
 "pmc_act:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $V --output-format csv -d $O/pmc_act -o p -- python bench.py $ACT $P" \
 "valu_json:60:python scripts/pmc_valu.py --pmc-dir $O/pmc_act --kernel act_loss_kernel --units-per-dispatch 623153737.142857 --key act.llama3-8b-block.t512.g20.bf16.b4.asym --sources act --commit r6n --out $VJ" \
 "act_a:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $A --output-format csv -d $O/act_a -o p -- python bench.py $ACT $P" \
 "act_b:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $B --output-format csv -d $O/act_b -o p -- python bench.py $ACT $P" \
 "bench_act:400:python bench.py $ACT --valu-json $VJ" \
 "trace_act:300:rocprofv3 --kernel-trace --stats -d $O/trace_act -o act --output-format csv -- python bench.py $ACT --no-cpu-baseline --valu-json $VJ"
