# round 5 final tree (after the act-path changes): traffic + VALU (slot) records, rocprof summaries, bench lines, full GPU suite
set -u
O=gpurun_out/r5u
mkdir -p $O
V="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
SRCH="--mode search --workload llama3-8b"
ACT="--mode act"
T=$O/pmc_traffic.json
VJ=$O/pmc_valu.json
bash scripts/gpu_run.sh r5u \
 "prof70:700:STEPS=20 TRAFFIC_OUT=$T COMMIT=r5u bash scripts/profile_round.sh r5u/l70" \
 "prof8f16:600:STEPS=20 WL_ARGS='--workload llama3-8b --dtype f16' TRAFFIC_KEY=llama3-8b.b4.asym.packed.f16 TRAFFIC_OUT=$T COMMIT=r5u bash scripts/profile_round.sh r5u/l8f16" \
 "pmc_search:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $V --output-format csv -d $O/pmc_search -o p -- python bench.py $SRCH --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling" \
 "pmc_act:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $V --output-format csv -d $O/pmc_act -o p -- python bench.py $ACT --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling" \
 "valu_json:60:python scripts/pmc_valu.py --pmc-dir $O/pmc_search --kernel awq_fast_kernel --units-per-dispatch 80302612480 --key llama3-8b.b4.asym.packed.search10of20 --sources fast --commit r5u --out $VJ && python scripts/pmc_valu.py --pmc-dir $O/pmc_act --kernel act_loss_kernel --units-per-dispatch 623153737.142857 --key act.llama3-8b-block.t512.g20.bf16.b4.asym --sources act --commit r5u --out $VJ" \
 "bench:600:python bench.py --traffic-json $T" \
 "bench_f16:300:python bench.py --workload llama3-8b --dtype f16 --no-cpu-baseline --traffic-json $T" \
 "bench_search:400:python bench.py $SRCH --valu-json $VJ" \
 "bench_act:400:python bench.py $ACT --valu-json $VJ" \
 "trace_search:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_fast_kernel -d $O/trace_search -o s --output-format csv -- python bench.py $SRCH --no-cpu-baseline --valu-json $VJ" \
 "trace_act:300:rocprofv3 --kernel-trace --stats -d $O/trace_act -o act --output-format csv -- python bench.py $ACT --no-cpu-baseline --valu-json $VJ" \
 smoke \
 pytest
