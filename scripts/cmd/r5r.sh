# round 5: one-pass weight column sums (act search duo w_mean) — bit-exactness, then the
# act block A/B against the two-pass build
set -u
AB="python scripts/act_search_bench.py --iters 5"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=("pytest=tests/test_act_search.py")
for rnd in 1 2; do
  for dt in bf16 f16; do
    steps+=("a_fused_${dt}_$rnd:120:$AB --dtype $dt" "a_2pass_${dt}_$rnd:120:$AB --dtype $dt --lib $L/libawq_hip_wm2pass.so")
  done
done
bash scripts/gpu_run.sh r5r "${steps[@]}"
