# round 5: one-pass quantization of W * diag(s) (awq_quantize_groups_scaled) — tests, then
# the act block timings (apply+quantize vs the one-pass call, block total)
set -u
AB="python scripts/act_search_bench.py --iters 5"
steps=("pytest=tests/test_act_search.py tests/test_gpu_parity.py tests/test_scale_search.py")
for rnd in 1 2; do
  for dt in bf16 f16; do steps+=("a_${dt}_$rnd:120:$AB --dtype $dt"); done
done
steps+=("bench_act:400:python bench.py --mode act --no-cpu-baseline --valu-json profiles/round5/pmc_valu.json")
bash scripts/gpu_run.sh r5w "${steps[@]}"
