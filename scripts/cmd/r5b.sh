# round 5: VALU rooflines of the grid-search kernels + ragged clip search
set -u
O=gpurun_out/r5b
V="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
SRCH="--mode search --workload llama3-8b"
ACT="--mode act"
bash scripts/gpu_run.sh r5b \
 "pytest=tests/test_scale_search.py tests/test_cli.py -k 'search'" \
 "bench_search:400:python bench.py $SRCH --no-cpu-baseline" \
 "bench_act:400:python bench.py $ACT --no-cpu-baseline" \
 "pmc_search:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex awq_fast_kernel --pmc $V --output-format csv -d $O/pmc_search -o p -- python bench.py $SRCH --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling" \
 "pmc_act:200:timeout -s KILL 150 rocprofv3 --kernel-include-regex act_loss_kernel --pmc $V --output-format csv -d $O/pmc_act -o p -- python bench.py $ACT --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling" \
 "valu_json:60:python scripts/pmc_valu.py --pmc-dir $O/pmc_search --kernel awq_fast_kernel --units-per-dispatch 80302612480 --key llama3-8b.b4.asym.packed.search10of20 --sources fast --commit r5b --out $O/pmc_valu.json && python scripts/pmc_valu.py --pmc-dir $O/pmc_act --kernel act_loss_kernel --units-per-dispatch 623153737.142857 --key act.llama3-8b-block.t512.g20.bf16.b4.asym --sources act --commit r5b --out $O/pmc_valu.json" \
 "bench_search2:400:python bench.py $SRCH --valu-json $O/pmc_valu.json" \
 "bench_act2:400:python bench.py $ACT --valu-json $O/pmc_valu.json" \
 "trace_act:300:rocprofv3 --kernel-trace --stats -d $O/trace_act -o act --output-format csv -- python bench.py $ACT --no-cpu-baseline --valu-json $O/pmc_valu.json" \
 "trace_search:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_fast_kernel -d $O/trace_search -o s --output-format csv -- python bench.py $SRCH --no-cpu-baseline --valu-json $O/pmc_valu.json" \
 "sq_act:500:bash scripts/pmc_kernel.sh $O/pmc_act_full act_loss_kernel python bench.py $ACT --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling" \
 "sq_search:500:bash scripts/pmc_kernel.sh $O/pmc_search_full awq_fast_kernel python bench.py $SRCH --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
