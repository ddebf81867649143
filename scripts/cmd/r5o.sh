# round 5: act loss kernel with the LDS-DMA table ring — VALU slot record, bench line, trace;
# then the full GPU suite and smoke on the final tree
set -u
O=gpurun_out/r5o
mkdir -p $O
cp profiles/round5/pmc_valu.json $O/pmc_valu.json
V="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
ACT="--mode act"
VJ=$O/pmc_valu.json
bash scripts/gpu_run.sh r5o \
 "pmc_act:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $V --output-format csv -d $O/pmc_act -o p -- python bench.py $ACT --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling" \
 "valu_json:60:python scripts/pmc_valu.py --pmc-dir $O/pmc_act --kernel act_loss_kernel --units-per-dispatch 623153737.142857 --key act.llama3-8b-block.t512.g20.bf16.b4.asym --sources act --commit r5o --out $VJ" \
 "bench_act:400:python bench.py $ACT --valu-json $VJ" \
 "trace_act:300:rocprofv3 --kernel-trace --stats -d $O/trace_act -o act --output-format csv -- python bench.py $ACT --no-cpu-baseline --valu-json $VJ" \
 pytest smoke
