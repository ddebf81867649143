# round 5, first call: private-method promotion parity, the bit-exact
# activation-aware table (item 2), the writer-failure fix, fp16 on the round-4
# streaming kernel (item 4)
set -u
bash scripts/gpu_run.sh r5a \
 "pytest=tests/test_private_methods.py tests/test_act_search.py" \
 "pytest=tests/test_cli.py -k 'failing_tensors or does_not_hang or bounded_rings_wrap'" \
 "bench_f16_l8:300:python bench.py --workload llama3-8b --dtype f16 --no-cpu-baseline" \
 "bench_f16_o350:300:python bench.py --workload opt-350m --dtype f16 --no-cpu-baseline" \
 "bench_bf16_l8:300:python bench.py --workload llama3-8b --no-cpu-baseline" \
 "prof:600:STEPS=20 WL_ARGS='--workload llama3-8b --dtype f16' TRAFFIC_KEY=llama3-8b.b4.asym.packed.f16 COMMIT=r5a bash scripts/profile_round.sh r5a/f16" \
 "sq:500:bash scripts/pmc_kernel.sh gpurun_out/r5a/pmc_f16_l8 awq_fast_kernel python bench.py --workload llama3-8b --dtype f16 --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling"
