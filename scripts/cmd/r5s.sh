# round 5: one-pass weight column sums with next-stage prefetch + the workspace scale table:
# bit-exactness, then the act block against the two-pass weight-mean build
set -u
AB="python scripts/act_search_bench.py --iters 5"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=("pytest=tests/test_act_search.py tests/test_cpu_host.py")
for rnd in 1 2; do
  for dt in bf16 f16; do
    steps+=("a_new_${dt}_$rnd:120:$AB --dtype $dt" "a_base_${dt}_$rnd:120:$AB --dtype $dt --lib $L/libawq_hip_r5base.so")
  done
done
bash scripts/gpu_run.sh r5s "${steps[@]}"
